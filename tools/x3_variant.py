"""Experiment builds of the row kernel (NOT product): copies csrc/ to /tmp, applies text patches to
mlp_x3.hip, compiles it and links it with the in-tree objects into build/variants/<name>.so (for
SGN_HIP_LIB= same-box A/B, tools/x3_ab.sh / tools/ab_lib.sh).

  python tools/x3_variant.py <name> [patch ...]

patches:
  timing   s_memtime stamps of k_rows16 (NS = 2, 4 waves) at every chunk entry, after block3.2's MFMAs,
           at the tile end and the tile start, for the first 8 workgroups' waves; the in-kernel clock
           (s_memtime / s_memrealtime around the tile loop).  SGN_X3_TDBG=<file> dumps them after the
           first row launch (tools/x3_timing_ns2.py reads the dump).
  abl_dma  no weight LDS-DMA (wrong results)          abl_bar  no chunk-boundary waits / barrier
  abl_conv no hi/lo conversion of the chained layers   abl_epi  no block3.2 epilogue
  abl_pe   no PE(dists) sin/cos (block1.0's input constant)
  cabl_dma / cabl_bar / cabl_fs / cabl_out: the colour kernel (k_color16) without its weight DMA, its
           chunk-boundary waits and barriers, its f_s row loads, its output layer
The ablations compute wrong results by design: timing only."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sg-nerf_amd", "csrc")


def rep(s, old, new, count=1):
    n = s.count(old)
    if n != count:
        raise SystemExit(f"patch anchor found {n} times (want {count}): {old[:90]!r}")
    return s.replace(old, new)


TIMING_DECL = r'''
// ---- timing build (tools/x3_variant.py timing) ----
constexpr int TD_BLOCKS = 8, TD_W = 4, TD_EV = 2048, TD_PER = 32;
__device__ unsigned long long g_tdbg[TD_BLOCKS * TD_W * TD_EV];
__shared__ int g_titer[TD_W];
__device__ __forceinline__ void tstamp(int n) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (blockIdx.x < TD_BLOCKS && (threadIdx.x & 63) == 0 && w < TD_W) {
        const int it = g_titer[w];
        if (it >= 0 && it < (TD_EV - 4) / TD_PER)
            g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + it * TD_PER + n] = __builtin_amdgcn_s_memtime();
    }
}
'''


TDUMP = '''            // the dump is of the SGN_X3_TDBG_LAUNCH-th (default 6th) inference row launch
            static int tlaunch = 0;
            const char *tpath = getenv("SGN_X3_TDBG");
            const char *tl = getenv("SGN_X3_TDBG_LAUNCH");
            const int tgt = tl ? atoi(tl) : 6;
            const bool tme = tpath && !z && ns == 2 && ksb == 0 && i0 == 0 && ++tlaunch == tgt;
            void *tptr = nullptr;
            const size_t tn = sizeof(x3::g_tdbg);
            SGN_CHECK_HIP(hipGetSymbolAddress(&tptr, HIP_SYMBOL(x3::g_tdbg)));
            if (tme) SGN_CHECK_HIP(hipMemsetAsync(tptr, 0, tn, st));
            hipLaunchKernelGGL(kern, dim3((unsigned)(wg16 < wmax ? wg16 : wmax)), dim3(x3::TPBR), 0, st, a);
            if (tme) {
                std::vector<unsigned long long> hb(tn / 8);
                SGN_CHECK_HIP(hipMemcpyAsync(hb.data(), tptr, tn, hipMemcpyDeviceToHost, st));
                SGN_CHECK_HIP(hipStreamSynchronize(st));
                if (FILE *f = fopen(tpath, "wb")) { fwrite(hb.data(), 8, tn / 8, f); fclose(f); }
            }'''


def patch(s, p):
    if p == "timing":
        s = rep(s, "__device__ __forceinline__ int cur_slot(int s) { return s; }",
                TIMING_DECL + "__device__ __forceinline__ int cur_slot(int s) { return s; }")
        s = rep(s, '''    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}''', '''    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (Net::NL == 4 && Net::NW == 4) tstamp(N);
}''')
        s = rep(s, '''    for (int tile = xt.first; tile < xt.end; tile += xt.step) {
        const int base = tile * WGS;''', '''    if (lane == 0 && w < TD_W) g_titer[w] = -1;
    const bool tdo = !SAVE && KB == 0 && NS == 2 && blockIdx.x < TD_BLOCKS && lane == 0;
    if (tdo) {
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 4] = __builtin_amdgcn_s_memtime();
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 3] = __builtin_amdgcn_s_memrealtime();
    }
    for (int tile = xt.first; tile < xt.end; tile += xt.step) {
        if (lane == 0 && w < TD_W) g_titer[w] += 1;
        if (!SAVE && KB == 0 && NS == 2) tstamp(29);
        const int base = tile * WGS;''')
        s = rep(s, '''        // everything prefetched has landed (the chunk boundaries waited vmcnt(0)): hide the loads''',
                '''        if (!SAVE && KB == 0 && NS == 2) tstamp(27);
        // everything prefetched has landed (the chunk boundaries waited vmcnt(0)): hide the loads''')
        s = rep(s, '''            for (int q = 0; q < NS; ++q) epi_end(e[q], ldsi, nA[q], nB[q], ix[q].s);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}''', '''            for (int q = 0; q < NS; ++q) epi_end(e[q], ldsi, nA[q], nB[q], ix[q].s);
        }
        if (!SAVE && KB == 0 && NS == 2) tstamp(28);
    }
    if (tdo) {
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 2] = __builtin_amdgcn_s_memtime();
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 1] = __builtin_amdgcn_s_memrealtime();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}''')
        s = patch(s, "tdump")
    elif p == "timing2":
        # light stamps: 8 per tile at the layer boundaries of k_rows16<0, false, false, 2> (no chunk stamps)
        s = rep(s, "__device__ __forceinline__ int cur_slot(int s) { return s; }", r'''
constexpr int TD_BLOCKS = 8, TD_W = 4, TD_EV = 2048, TD_PER = 8;
__device__ unsigned long long g_tdbg[TD_BLOCKS * TD_W * TD_EV];
__device__ __forceinline__ void tst(bool on, int w, int it, int n) {
    if (on && it < (TD_EV - 4) / TD_PER)
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + it * TD_PER + n] = __builtin_amdgcn_s_memtime();
}
__device__ __forceinline__ int cur_slot(int s) { return s; }''')
        s = rep(s, '''    for (int tile = xt.first; tile < xt.end; tile += xt.step) {
        const int base = tile * WGS;''', '''    const bool tdo = !SAVE && KB == 0 && NS == 2 && blockIdx.x < TD_BLOCKS && lane == 0;
    if (tdo) {
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 4] = __builtin_amdgcn_s_memtime();
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 3] = __builtin_amdgcn_s_memrealtime();
    }
    int tit = -1;
    for (int tile = xt.first; tile < xt.end; tile += xt.step) {
        ++tit;
        tst(tdo, w, tit, 0);
        const int base = tile * WGS;''')
        for a, b in (("            run_layer_ns<Net, 0, false, std::conditional_t<SAVE, VmZero, VmL0<NS>>, 0, 0, !SAVE>(", 1),
                     ("        run_layer_ns<Net, 1, false, VmZero, 0, 0, !SAVE>(wb, ldsi, slot, w, lane, lz, accB, [&](auto k) {", 2),
                     ("        run_layer_ns<Net, L2, false, VmZero, 0, 0, !SAVE>(wb, ldsi, slot, w, lane, lz, acc2, [&](auto k) {", 3),
                     ("            run_layer_ns<Net, L3, true, std::conditional_t<SAVE, VmZero, VmL3P0<NS>>, 0, 0, !SAVE>(", 4)):
            s = rep(s, a, " " * (len(a) - len(a.lstrip())) + f"tst(tdo, w, tit, {b});\n" + a)
        s = rep(s, "            run_layer_ns<Net, L3, true, VmZero, 1, 8>(wb, ldsi, slot, w, lane, lz, acc, [&](auto k) {",
                "            tst(tdo, w, tit, 5);\n            run_layer_ns<Net, L3, true, VmZero, 1, 8>(wb, ldsi, slot, w, lane, lz, acc, [&](auto k) {")
        s = rep(s, "        // everything prefetched has landed (the chunk boundaries waited vmcnt(0)): hide the loads",
                "        tst(tdo, w, tit, 6);\n        // everything prefetched has landed (the chunk boundaries waited vmcnt(0)): hide the loads")
        s = rep(s, '''            for (int q = 0; q < NS; ++q) epi_end(e[q], ldsi, nA[q], nB[q], ix[q].s);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}''', '''            for (int q = 0; q < NS; ++q) epi_end(e[q], ldsi, nA[q], nB[q], ix[q].s);
        }
        tst(tdo, w, tit, 7);
    }
    if (tdo) {
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 2] = __builtin_amdgcn_s_memtime();
        g_tdbg[(blockIdx.x * TD_W + w) * TD_EV + TD_EV - 1] = __builtin_amdgcn_s_memrealtime();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}''')
        s = patch(s, "tdump")
    elif p == "tdump":
        s = rep(s, '''            hipLaunchKernelGGL(kern, dim3((unsigned)(wg16 < wmax ? wg16 : wmax)), dim3(x3::TPBR), 0, st, a);''',
                TDUMP)
    elif p == "v_wait":
        # one lgkmcnt wait per fragment pair: the lo fragment (loaded after hi) is used first
        s = rep(s, '''                    if constexpr (TRANS) {
                        c = mfma16(B.b[s].hi, Ah, c);
                        c = mfma16(B.b[s].lo, Ah, c);
                        c = mfma16(B.b[s].hi, Al, c);
                    } else {
                        c = mfma16(Ah, B.b[s].hi, c);
                        c = mfma16(Ah, B.b[s].lo, c);
                        c = mfma16(Al, B.b[s].hi, c);
                    }''', '''                    if constexpr (TRANS) {
                        c = mfma16(B.b[s].hi, Al, c);
                        c = mfma16(B.b[s].lo, Ah, c);
                        c = mfma16(B.b[s].hi, Ah, c);
                    } else {
                        c = mfma16(Al, B.b[s].hi, c);
                        c = mfma16(Ah, B.b[s].lo, c);
                        c = mfma16(Ah, B.b[s].hi, c);
                    }''')
    elif p == "v_dma":
        # contiguous pieces per wave: wave w moves pieces w PW .. w PW + PW - 1 of a chunk; four consecutive
        # pieces share one soffset / M0, the instruction offset (0..3 KiB) steps through them
        s = rep(s, '''template <class Net, int N, int J, int NWv = NW16>
__device__ __forceinline__ void dma_piece(const WBlob &wb, char *dst, int w, int lane, int) {
    using S = Sched<Net>;
    constexpr int nf = 2 * S::pairs(N);
    const int i = w + NWv * J;
    if (NWv * (J + 1) <= nf || i < nf)  // wave-uniform
        lds_dma_1k(wb, dst + NWv * J * 1024, w, lane, S::off(N) + (uint32_t)(NWv * J * 1024));
}''', '''template <class Net, int N, int J, int NWv = NW16>
__device__ __forceinline__ void dma_piece(const WBlob &wb, char *dst, int w, int lane, int) {
    using S = Sched<Net>;
    constexpr int nf = 2 * S::pairs(N);
    constexpr int PW = (nf + NWv - 1) / NWv;
    const int i = w * PW + J;
    if (nf % NWv == 0 || i < nf) {  // wave-uniform
        uint32_t soff = S::off(N) + (uint32_t)((J & ~3) * 1024);
        asm volatile("" : "+s"(soff));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wb.rsrc,
                                                 (__attribute__((address_space(3))) void *)(dst + (w * PW + (J & ~3)) * 1024),
                                                 16, lane * 16 + w * PW * 1024, soff, (J & 3) * 1024, 0);
    }
}''')
    elif p == "v_pipe":
        # block3.2 pass 0: k-step K + 1's input converted in the middle of k-step K's MFMAs (its fragments are
        # kept for pass 1 anyway, so both being live costs no registers)
        s = rep(s, '''template <class Net, int L, bool TRANS = false, class Vm = VmZero, int P = 0, int AOFF = 0, int NS, int NA,
          class SlotT, class InFn, class PostFn = NoHook, class EndFn = NoHook, class MidFn = NoHook>''',
                '''template <class Net, int L, bool TRANS = false, class Vm = VmZero, int P = 0, int AOFF = 0, bool PIPE = false,
          int NS, int NA, class SlotT, class InFn, class PostFn = NoHook, class EndFn = NoHook, class MidFn = NoHook>''')
        s = rep(s, '''    static_assert(AOFF + TP <= NA, "accumulator view");
    static_for<nch(ly)>([&](auto cc) {''', '''    static_assert(AOFF + TP <= NA, "accumulator view");
    X3S<NS> Bn;
    if constexpr (PIPE) Bn = in(std::integral_constant<int, 0>{});
    static_for<nch(ly)>([&](auto cc) {''')
        s = rep(s, '''            if constexpr (NS > 1 && KK > 0) __builtin_amdgcn_sched_barrier(0);
            const X3S<NS> B = in(std::integral_constant<int, C * ly.kc + KK>{});''', '''            constexpr int KS = C * ly.kc + KK;
            if constexpr (NS > 1 && KK > 0 && !PIPE) __builtin_amdgcn_sched_barrier(0);
            X3S<NS> B;
            if constexpr (PIPE) B = Bn;
            else B = in(std::integral_constant<int, KS>{});''')
        s = rep(s, '''                mid(std::integral_constant<int, (C * ly.kc + KK) * TP + t>{});''', '''                mid(std::integral_constant<int, (C * ly.kc + KK) * TP + t>{});
                if constexpr (PIPE && t == TP / 2 - 1 && KS + 1 < ly.ks) Bn = in(std::integral_constant<int, KS + 1>{});''')
        s = rep(s, '''            run_layer_ns<Net, L3, true, std::conditional_t<SAVE, VmZero, VmL3P0<NS>>, 0, 0>(''',
                '''            run_layer_ns<Net, L3, true, std::conditional_t<SAVE, VmZero, VmL3P0<NS>>, 0, 0, !SAVE>(''')
    elif p == "v_pipeall":
        # (after v_pipe) every row-kernel layer converts k-step K + 1's input during k-step K's MFMAs
        s = rep(s, "            run_layer_ns<Net, 0, false, std::conditional_t<SAVE, VmZero, VmL0<NS>>>(",
                "            run_layer_ns<Net, 0, false, std::conditional_t<SAVE, VmZero, VmL0<NS>>, 0, 0, !SAVE>(")
        s = rep(s, "        run_layer_ns<Net, 1>(wb, ldsi, slot, w, lane, lz, accB, [&](auto k) {",
                "        run_layer_ns<Net, 1, false, VmZero, 0, 0, !SAVE>(wb, ldsi, slot, w, lane, lz, accB, [&](auto k) {")
        s = rep(s, "        run_layer_ns<Net, L2>(wb, ldsi, slot, w, lane, lz, acc2, [&](auto k) {",
                "        run_layer_ns<Net, L2, false, VmZero, 0, 0, !SAVE>(wb, ldsi, slot, w, lane, lz, acc2, [&](auto k) {")
    elif p == "v_mix":
        # LeakyReLU on the raw accumulator (asm max into the tied 0.01 a) and the 2^-s scale folded into
        # the compiler's v_fma_mix{lo,hi}_f16 hi / lo conversion: 4 VALU per value instead of 5, same bits
        s = rep(s, '''__device__ __forceinline__ X3B lrelu_split8(const float (&a)[8], float inv) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = lrelu_x3(a[j] * inv);
    return split8(v);
}''', '''__device__ __forceinline__ X3B lrelu_split8(const float (&a)[8], float inv) {
    float l[8];
    _Float16 h[8], o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) l[j] = lrelu_x3(a[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (_Float16)__builtin_fmaf(l[j], inv, 0.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)__builtin_fmaf(l[j], inv, -(float)h[j]);
    return X3B{h8{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]}, h8{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]}};
}''')
    elif p == "v_early":
        # chunk start before the barrier: every wave LDS-DMAs its own copy of the chunk's first fragment pair
        # (pieces 0 and 1, identical bytes to the same LDS address), so after its own vmcnt wait it can read
        # pair 0 and issue that pair's MFMAs; the workgroup barrier follows them (its wait overlaps the MFMAs)
        s = rep(s, '''// LDS-DMA of stream chunk N into `dst`: 2 * pairs 1-KiB pieces, wave w (of NWv) moves pieces''', '''// piece p (0 or 1) of chunk N by any wave: the chunk's first fragment pair, duplicated per wave
template <class Net, int N, int P>
__device__ __forceinline__ void dma_dup(const WBlob &wb, char *dst, int lane) {
    uint32_t soff = Sched<Net>::off(N) + (uint32_t)(P * 1024);
    asm volatile("" : "+s"(soff));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wb.rsrc, (__attribute__((address_space(3))) void *)(dst + P * 1024), 16,
                                             lane * 16, soff, 0, 0);
}
// LDS-DMA of stream chunk N into `dst`: 2 * pairs 1-KiB pieces, wave w (of NWv) moves pieces''')
        s = rep(s, '''    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    if constexpr (VM == 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else  // vmcnt[3:0] | expcnt 7 | lgkmcnt 15 | vmcnt[5:4] << 14 (gfx9 encoding: wait on vmcnt only)
        __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (15 << 8) | ((VM >> 4) << 14));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}''', '''    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    if constexpr (VM == 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else  // vmcnt[3:0] | expcnt 7 | lgkmcnt 15 | vmcnt[5:4] << 14 (gfx9 encoding: wait on vmcnt only)
        __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (15 << 8) | ((VM >> 4) << 14));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}''')
        # the prologue chunk: every wave also moves pieces 0 and 1
        s = rep(s, '''            lds_dma_1k(wb, dst + NWv * J * 1024, w, lane, S::off(N) + (uint32_t)(NWv * J * 1024));
    });
}''', '''            lds_dma_1k(wb, dst + NWv * J * 1024, w, lane, S::off(N) + (uint32_t)(NWv * J * 1024));
    });
    dma_dup<Net, N, 0>(wb, dst, lane);
    dma_dup<Net, N, 1>(wb, dst, lane);
}''')
        s = rep(s, '''        h8 fh[PD], fl[PD];
#pragma unroll
        for (int f = 0; f < PD; ++f) {
            fh[f] = frag(f, 0);
            fl[f] = frag(f, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * PD, 0);''', '''        h8 fh[PD], fl[PD];
        fh[0] = frag(0, 0);   // pair 0: this wave's own copy, landed at its vmcnt wait
        fl[0] = frag(0, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);''')
        s = rep(s, '''                const h8 Ah = fh[F % PD], Al = fl[F % PD];
                if constexpr (F + PD < NF) {
                    fh[F % PD] = frag(F + PD, 0);
                    fl[F % PD] = frag(F + PD, 1);
                }''', '''                const h8 Ah = fh[F % PD], Al = fl[F % PD];
                if constexpr (F > 0 && F + PD < NF) {
                    fh[F % PD] = frag(F + PD, 0);
                    fl[F % PD] = frag(F + PD, 1);
                }''')
        s = rep(s, '''                constexpr int NSP = NF / 2 > 0 ? NF / 2 : 1;
                if constexpr (F < NSP) {''', '''                if constexpr (F == 0) {
                    // the other waves' pieces: barrier after this wave's first MFMAs, then the queue
                    __builtin_amdgcn_sched_barrier(0);
                    __builtin_amdgcn_s_barrier();
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int f = 1; f <= PD; ++f)
                        if (f < NF) {
                            fh[f % PD] = frag(f, 0);
                            fl[f % PD] = frag(f, 1);
                        }
                    dma_dup<Net, NN, 0>(wb, dnext, lane);
                    dma_dup<Net, NN, 1>(wb, dnext, lane);
                }
                constexpr int NSP = NF / 2 > 0 ? NF / 2 : 1;
                if constexpr (F < NSP) {''')
    elif p == "v_early3":
        # block3.2's input converted during block3.0's last k-step (the VALU-free ext k-step), tiles 2J, 2J + 1
        # after tile 2J + 3's MFMAs, so block3.2's pass 0 runs without conversion VALU
        s = rep(s, '''        auto &in2 = pick<(KB > 0)>(accA, accB);
        auto &acc2 = pick<(KB > 0)>(accB, accA);
        const float inv_in2 = KB > 0 ? inv7 : inv1;''', '''        auto &in2 = pick<(KB > 0)>(accA, accB);
        auto &acc2 = pick<(KB > 0)>(accB, accA);
        const float inv_in2 = KB > 0 ? inv7 : inv1;
        X3B in3[NS][8];
        constexpr int LASTK = (Net::L[L2].ks - 1) * 16;''')
        s = rep(s, '''                    nx[q].ray = nx[q].sval ? a.samp_ray[nx[q].s] : 0;
                }
            }
        });''', '''                    nx[q].ray = nx[q].sval ? a.samp_ray[nx[q].s] : 0;
                }
            }
        }, NoHook{}, [&](auto f) {
            constexpr int F = decltype(f)::value;
            if constexpr (F >= LASTK + 3 && ((F - LASTK) & 1) == 1) {
                constexpr int J = (F - LASTK - 3) / 2;
#pragma unroll
                for (int q = 0; q < NS; ++q) in3[q][J] = chain_k(q, acc2[q], inv2, std::integral_constant<int, J>{}, a.z3);
            }
        });
#pragma unroll
        for (int q = 0; q < NS; ++q) in3[q][7] = chain_k(q, acc2[q], inv2, std::integral_constant<int, 7>{}, a.z3);''')
        s = rep(s, '''            X3B in3[NS][8];
            run_layer_ns<Net, L3, true, std::conditional_t<SAVE, VmZero, VmL3P0<NS>>, 0, 0, !SAVE>(
                wb, ldsi, slot, w, lane, lz, acc, [&](auto k) {
                    constexpr int K = decltype(k)::value;
                    X3S<NS> o;
#pragma unroll
                    for (int q = 0; q < NS; ++q) {
                        in3[q][K] = chain_k(q, acc2[q], inv2, k, a.z3);
                        o.b[q] = in3[q][K];
                    }
                    return o;
                }, NoHook{}, first_chunk_loads);''', '''            run_layer_ns<Net, L3, true, std::conditional_t<SAVE, VmZero, VmL3P0<NS>>, 0, 0>(
                wb, ldsi, slot, w, lane, lz, acc, [&](auto k) {
                    X3S<NS> o;
#pragma unroll
                    for (int q = 0; q < NS; ++q) o.b[q] = in3[q][decltype(k)::value];
                    return o;
                }, NoHook{}, first_chunk_loads);''')
    elif p == "v_epic":
        # the epilogue's per-lane constants (block3.2 bias and alpha weight of unit 16 T + r, T = 0..15) read
        # into registers once per tile (8 ds_read_b128, one wait) instead of one LDS read + wait per step
        s = rep(s, '''    float inv3;
};''', '''    float inv3;
};
struct EpiC {
    float b[16], wa[16];
};''')
        s = rep(s, '''    auto epi_step = [&](Epi16 &e, const char *ldsi, const f32x4 (&ac)[16], auto tc) {
        constexpr int T = decltype(tc)::value;
        const float wau = ((const float *)(ldsi + YT16_OFF))[320 + r * 20 + T];  // 2^-s3 alpha weight''',
                '''    EpiC ec;
    auto epi_consts = [&](const char *ldsi) {
        const f32x4 *yb = (const f32x4 *)(ldsi + YT16_OFF + r * 80), *yw = (const f32x4 *)(ldsi + YT16_OFF + 1280 + r * 80);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f32x4 u = yb[j], v = yw[j];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ec.b[4 * j + i] = u[i];
                ec.wa[4 * j + i] = v[i];
            }
        }
    };
    auto epi_step = [&](Epi16 &e, const char *ldsi, const f32x4 (&ac)[16], auto tc) {
        constexpr int T = decltype(tc)::value;
        const float wau = ec.wa[T];  // 2^-s3 alpha weight''')
        s = rep(s, '''            const float hv = lrelu_x3(__builtin_fmaf(ac[T][i], e.inv3, ((const float *)(ldsi + YT16_OFF))[r * 20 + T]));''',
                '''            const float hv = lrelu_x3(__builtin_fmaf(ac[T][i], e.inv3, ec.b[T]));''')
        s = rep(s, '''            for (int q = 0; q < NS; ++q) epi_begin(e[q], ldsi, rw[q].wgt, nA[q], nB[q], ce[q], eslot[q] < nslots);''',
                '''            for (int q = 0; q < NS; ++q) epi_begin(e[q], ldsi, rw[q].wgt, nA[q], nB[q], ce[q], eslot[q] < nslots);
            epi_consts(ldsi);''')
    elif p == "cabl_dma":   # colour kernel: no weight LDS-DMA
        s = rep(s, """    using S = Sched<Net>;
    constexpr int nf = 2 * S::pairs(N);
    static_for<(nf + NWv - 1) / NWv>([&](auto jj) {""", """    using S = Sched<Net>;
    constexpr int nf = 2 * S::pairs(N);
    if constexpr (Net::NL == 3) return;
    static_for<(nf + NWv - 1) / NWv>([&](auto jj) {""")
        s = rep(s, """    constexpr int PW = (nf + NWv - 1) / NWv;
    const int i = w * PW + J;""", """    constexpr int PW = (nf + NWv - 1) / NWv;
    if constexpr (Net::NL == 3) return;
    const int i = w * PW + J;""")
    elif p == "cabl_bar":   # colour kernel: no chunk-boundary waits / barrier
        s = rep(s, """    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    if constexpr (VM == 0)""", """    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    if constexpr (Net::NL == 3) return;
    if constexpr (VM == 0)""")
    elif p == "cabl_fs":    # colour kernel: no f_s row loads
        s = rep(s, """#pragma unroll
        for (int k = 0; k < 8; ++k) {
            fr[2 * k] = row[8 * k];
            fr[2 * k + 1] = row[8 * k + 1];
        }""", """        (void)row;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            fr[2 * k] = f32x4{0.25f, 0.5f, 0.125f, 1.f};
            fr[2 * k + 1] = f32x4{0.25f, 0.5f, 0.125f, 1.f};
        }""")
    elif p == "cabl_out":   # colour kernel: no output layer
        s = rep(s, """        float o[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            f32x4 wc[3];""", """        float o[3] = {c0[0][0], c0[1][1], c0[2][2]};
#pragma unroll
        for (int t = 0; t < 0; ++t) {
            f32x4 wc[3];""")
    elif p == "abl_dma":
        s = rep(s, '''    asm volatile("" : "+s"(soff));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(''', '''    return;
    asm volatile("" : "+s"(soff));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(''')
    elif p == "abl_bar":
        s = rep(s, '''    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}''', '''    if constexpr (!(Net::NL == 4 && Net::NW == 4)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
}''')
        s = rep(s, '''    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    if constexpr (VM == 0)''', '''    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    if constexpr (Net::NL == 4 && Net::NW == 4) {
    } else if constexpr (VM == 0)''')
    elif p == "abl_conv":
        s = rep(s, '''            return lrelu_split8(v, inv);
        };
        auto bias_init''', '''            if constexpr (!SAVE && KB == 0) {
                X3B o;
                o.hi = __builtin_bit_cast(h8, u32x4{__builtin_bit_cast(uint32_t, v[0]), __builtin_bit_cast(uint32_t, v[1]),
                                                    __builtin_bit_cast(uint32_t, v[2]), __builtin_bit_cast(uint32_t, v[3])});
                o.lo = __builtin_bit_cast(h8, u32x4{__builtin_bit_cast(uint32_t, v[4]), __builtin_bit_cast(uint32_t, v[5]),
                                                    __builtin_bit_cast(uint32_t, v[6]), __builtin_bit_cast(uint32_t, v[7])});
                return o;
            }
            return lrelu_split8(v, inv);
        };
        auto bias_init''')
    elif p == "abl_epi":
        s = rep(s, '''    auto epi_step = [&](Epi16 &e, const char *ldsi, const f32x4 (&ac)[16], auto tc) {
        constexpr int T = decltype(tc)::value;''', '''    auto epi_step = [&](Epi16 &e, const char *ldsi, const f32x4 (&ac)[16], auto tc) {
        constexpr int T = decltype(tc)::value;
        if constexpr (KB == 0 && !SAVE) { e.fsv[T & 3] = ac[T][0]; if constexpr ((T & 3) == 3) { if (e.fs_have) e.fs_dst[16 * (T - 3)] = e.fsv[0] + e.fsv[1] + e.fsv[2] + e.fsv[3]; } return; }''')
    elif p == "e_order":
        # MFMA order of a (k-step, tile) across the row sets grouped by weight fragment: (lo, hi_s) for every
        # row set, then (hi, lo_s), then (hi, hi_s) -- each accumulator sees the same three products in the
        # same order as before (bit-identical), the weight operand changes twice per 3 NS MFMAs
        s = rep(s, '''#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    f32x4 &c = acc[s][AOFF + t];
                    if constexpr (TRANS) {
                        c = mfma16(B.b[s].hi, Al, c);
                        c = mfma16(B.b[s].lo, Ah, c);
                        c = mfma16(B.b[s].hi, Ah, c);
                    } else {
                        c = mfma16(Al, B.b[s].hi, c);
                        c = mfma16(Ah, B.b[s].lo, c);
                        c = mfma16(Ah, B.b[s].hi, c);
                    }
                }''', '''if constexpr (TRANS) {
#pragma unroll
                    for (int s = 0; s < NS; ++s) acc[s][AOFF + t] = mfma16(B.b[s].hi, Al, acc[s][AOFF + t]);
#pragma unroll
                    for (int s = 0; s < NS; ++s) acc[s][AOFF + t] = mfma16(B.b[s].lo, Ah, acc[s][AOFF + t]);
#pragma unroll
                    for (int s = 0; s < NS; ++s) acc[s][AOFF + t] = mfma16(B.b[s].hi, Ah, acc[s][AOFF + t]);
                } else {
#pragma unroll
                    for (int s = 0; s < NS; ++s) acc[s][AOFF + t] = mfma16(Al, B.b[s].hi, acc[s][AOFF + t]);
#pragma unroll
                    for (int s = 0; s < NS; ++s) acc[s][AOFF + t] = mfma16(Ah, B.b[s].lo, acc[s][AOFF + t]);
#pragma unroll
                    for (int s = 0; s < NS; ++s) acc[s][AOFF + t] = mfma16(Ah, B.b[s].hi, acc[s][AOFF + t]);
                }''')
    elif p == "abl_pe":
        s = rep(s, '''                    for (int q = 0; q < NS; ++q) o.b[q] = pe_dists16_k<decltype(k)::value>(pr[q]);''',
                '''                    for (int q = 0; q < NS; ++q) {
                        if constexpr (!SAVE && KB == 0) {
                            const float c0 = pr[q].lo + (float)decltype(k)::value;
                            o.b[q] = X3B{__builtin_bit_cast(h8, u32x4{__builtin_bit_cast(uint32_t, c0), 0u, 0u, 0u}),
                                         __builtin_bit_cast(h8, u32x4{0u, __builtin_bit_cast(uint32_t, c0), 0u, 0u})};
                        } else {
                            o.b[q] = pe_dists16_k<decltype(k)::value>(pr[q]);
                        }
                    }''')
    else:
        raise SystemExit(f"unknown patch {p}")
    return s


def patch_tx(s, p):
    """patches of train_x3.hip (the fp32 training GEMMs)"""
    if p == "tx_rows2":
        # backward-data / forward rows GEMMs at K 256 / 288: 64-column weight blocks (64 KiB of LDS), two
        # workgroups per CU (two waves per SIMD hide each other's load / store latency)
        s = rep(s, '''template <int KS, int WN, bool P1 = false>
__global__ __launch_bounds__(TPB, 1) void k_x3rows(GemmK g) {''', '''template <int KS, int WN, bool P1 = false, int OCC = 1>
__global__ __launch_bounds__(TPB, OCC) void k_x3rows(GemmK g) {''')
        s = rep(s, '''        const bool w96 = ((g.N + 95) / 96) * 96 < ((g.N + 127) / 128) * 128;
        const int BN = w96 ? 96 : 128;''', '''        const bool w96 = ((g.N + 95) / 96) * 96 < ((g.N + 127) / 128) * 128;
        const bool occ2 = !p1 && (g.K + 15) / 16 > 8;
        const int BN = occ2 ? 64 : w96 ? 96 : 128;''')
        s = rep(s, '''        int gy = 256 / nb;''', '''        int gy = (occ2 ? 512 : 256) / nb;''')
        s = rep(s, '''        } else if (ks <= 16) {
            if (w96) hipLaunchKernelGGL((k_x3rows<16, 3>), grid, dim3(TPB), 0, st, k);
            else hipLaunchKernelGGL((k_x3rows<16, 4>), grid, dim3(TPB), 0, st, k);
        } else {
            if (w96) hipLaunchKernelGGL((k_x3rows<18, 3>), grid, dim3(TPB), 0, st, k);
            else hipLaunchKernelGGL((k_x3rows<18, 4>), grid, dim3(TPB), 0, st, k);
        }''', '''        } else if (ks <= 16) {
            hipLaunchKernelGGL((k_x3rows<16, 2, false, 2>), grid, dim3(TPB), 0, st, k);
        } else {
            hipLaunchKernelGGL((k_x3rows<18, 2, false, 2>), grid, dim3(TPB), 0, st, k);
        }''')
    elif p == "tx_tn2":
        # weight gradients at M 256: 256 x 64 blocks, two workgroups per CU (80 KiB of LDS each)
        s = rep(s, '''template <int WM, int WN, bool P1 = false>
__global__ __launch_bounds__(TPB, 1) void k_x3tn(GemmK g) {''', '''template <int WM, int WN, bool P1 = false, int OCC = 1>
__global__ __launch_bounds__(TPB, OCC) void k_x3tn(GemmK g) {''')
        s = rep(s, '''        const int BN = g.N <= 32 ? 32 : (BM == 128 && g.N <= 160) ? 160 : 96;''',
                '''        const int BN = g.N <= 32 ? 32 : (BM == 128 && g.N <= 160) ? 160 : BM == 256 ? 64 : 96;''')
        s = rep(s, '''        } else if (BM == 256 && BN == 96) hipLaunchKernelGGL((k_x3tn<2, 3>), grid, dim3(TPB), 0, st, k);''',
                '''        } else if (BM == 256 && BN == 64) hipLaunchKernelGGL((k_x3tn<2, 2, false, 2>), grid, dim3(TPB), 0, st, k);''')
    elif p == "tx_tn3":
        # weight gradients at M 256: 128 x 96 blocks, two workgroups per CU (56 KiB of LDS each)
        s = rep(s, '''template <int WM, int WN, bool P1 = false>
__global__ __launch_bounds__(TPB, 1) void k_x3tn(GemmK g) {''', '''template <int WM, int WN, bool P1 = false, int OCC = 1>
__global__ __launch_bounds__(TPB, OCC) void k_x3tn(GemmK g) {''')
        s = rep(s, '''        const int BM = g.M > 128 ? 256 : 128;''', '''        const int BM = 128;''')
        s = rep(s, '''        else if (BN == 96) hipLaunchKernelGGL((k_x3tn<1, 3>), grid, dim3(TPB), 0, st, k);''',
                '''        else if (BN == 96 && g.M > 128) hipLaunchKernelGGL((k_x3tn<1, 3, false, 2>), grid, dim3(TPB), 0, st, k);
        else if (BN == 96) hipLaunchKernelGGL((k_x3tn<1, 3>), grid, dim3(TPB), 0, st, k);''')
    elif p == "txa_noA":   # k_x3rows ablation: no A loads after the first tile (the split kept)
        s = rep(s, '''            an.load(16 * s, hk, a[s]);  // the next tile's k-step s''', '''#pragma unroll
            for (int e = 0; e < 8; ++e) asm volatile("" : "+v"(a[s][e]));''')
    elif p == "txa_nomask":   # k_x3rows ablation: no mask loads
        s = rep(s, '''                    mk[t][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rmk, off, 0, 0));''',
                '''                    mk[t][r] = off == 7u ? 0.f : 1.f;''')
    elif p == "txa_nostore":   # k_x3rows ablation: no output stores (amax kept)
        s = rep(s, '''                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v1), ro1,
                                                          o1 ? (uint32_t)(((int64_t)row * g.ldo + n) * 4) : OOB, 0, 0);''', '')
    elif p == "txa_nostage":   # k_x3rows ablation: no weight staging loads
        s = rep(s, '''        load8(g.B, rsB, n0 + 32 * t + (fl & 31), 16 * s + 8 * (fl >> 5), g.B.nrows, v);''',
                '''#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (float)(fl + e);''')
    elif p == "txa_nomfma":   # k_x3rows ablation: no MFMAs (operands kept live)
        s = rep(s, '''                    acc[t] = mfma32(x.lo, bh, acc[t]);
                    acc[t] = mfma32(x.hi, bl, acc[t]);
                }
                acc[t] = mfma32(x.hi, bh, acc[t]);
            }
        }
        // epilogue''', '''                    asm volatile("" :: "v"(x.lo), "v"(bl));
                }
                asm volatile("" :: "v"(x.hi), "v"(bh));
            }
        }
        // epilogue''')
    elif p == "dwa_nomfma":   # k_x3dw ablation: no MFMAs (fragments kept live)
        s = rep(s, """                    acc[a][b] = mfma32(af[a].lo, bf[b].hi, acc[a][b]);
                    acc[a][b] = mfma32(af[a].hi, bf[b].lo, acc[a][b]);
                    acc[a][b] = mfma32(af[a].hi, bf[b].hi, acc[a][b]);""",
                """                    asm volatile("" :: "v"(af[a].lo), "v"(af[a].hi), "v"(bf[b].lo), "v"(bf[b].hi));""")
    elif p == "dwa_noconv":   # k_x3dw ablation: no B conversion
        s = rep(s, """        if (st + 1 < nst) convert(st + 1);""", "")
    elif p == "dwa_noA":   # k_x3dw ablation: no A fragment reads / split (B's fragments reused)
        s = rep(s, """                af[a] = split8_mix(v, fa);""", """                af[a] = X3Pair{h8{}, h8{}};
                asm volatile("" :: "v"(v[0]));""")
        s = rep(s, """                for (int e = 0; e < 8; ++e) v[e] = src[256 * e];""",
                """                for (int e = 0; e < 1; ++e) v[e] = src[256 * e];""")
    elif p == "dwa_nodma":   # k_x3dw ablation: no DMA (LDS as it is)
        s = rep(s, """        for (int e = 0; e < 8; ++e) dma16(ra.r1, slot + (8 * w + e) * 1024, av, (rs + e) * ald);""",
                """        for (int e = 0; e < 8; ++e) asm volatile("" :: "v"(av));""")
        s = rep(s, """                dma16(rb.r1, dst, bv1[jj], rs * bld1);
            } else {""", """                asm volatile("" :: "v"(bv1[jj]));
            } else {""")
    elif p == "dwa_nobar":   # k_x3dw ablation: waits without the barrier
        s = rep(s, """    if (n == 14) asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)\\n\\ts_barrier" ::: "memory");
    else if (n == 11) asm volatile("s_waitcnt vmcnt(11) lgkmcnt(0)\\n\\ts_barrier" ::: "memory");
    else if (n == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\\n\\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\\n\\ts_barrier" ::: "memory");""",
                """    if (n == 14) asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)" ::: "memory");
    else if (n == 11) asm volatile("s_waitcnt vmcnt(11) lgkmcnt(0)" ::: "memory");
    else if (n == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");""")
    else:
        return None
    return s


def main():
    name, patches = sys.argv[1], sys.argv[2:]
    subprocess.check_call(["make", "-s", "-C", CSRC, "-j8"])
    top = f"/tmp/x3v_{name}"
    shutil.rmtree(top, ignore_errors=True)
    work = os.path.join(top, "pkg", "csrc")      # sgn_common.h includes ../../include/sgn_hip.h
    shutil.copytree(CSRC, work, ignore=shutil.ignore_patterns("build"))
    os.symlink(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    src = src0 = open(os.path.join(work, "mlp_x3.hip")).read()
    tsrc = tsrc0 = open(os.path.join(work, "train_x3.hip")).read()
    for p in patches:
        t = patch_tx(tsrc, p)
        if t is not None:
            tsrc = t
        else:
            src = patch(src, p)
    open(os.path.join(work, "mlp_x3.hip"), "w").write(src)
    open(os.path.join(work, "train_x3.hip"), "w").write(tsrc)
    targets = (["mlp_x3"] if src != src0 else []) + (["train_x3"] if tsrc != tsrc0 else [])
    out_dir = os.path.join(ROOT, "build", "variants")
    os.makedirs(out_dir, exist_ok=True)
    hipcc = "/opt/rocm/bin/hipcc"
    fl = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-munsafe-fp-atomics",
          "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include")]
    new_objs = []
    for t in targets:
        obj = os.path.join(work, t + ".o")
        extra = ["-fno-slp-vectorize"]   # both objects' Makefile flags
        subprocess.check_call([hipcc, *[f for f in fl if f != "-fno-slp-vectorize"], *extra, "-save-temps=obj", "-c",
                               os.path.join(work, t + ".hip"), "-o", obj])
        new_objs.append(obj)
    objs = [os.path.join(CSRC, "build", f) for f in sorted(os.listdir(os.path.join(CSRC, "build")))
            if f.endswith(".o") and f[:-2] not in targets]
    so = os.path.join(out_dir, name + ".so")
    subprocess.check_call([hipcc, "--offload-arch=gfx950", "-shared", "-Wl,-rpath,/opt/rocm/lib", "-o", so, *objs, *new_objs])
    print(so)


if __name__ == "__main__":
    main()
