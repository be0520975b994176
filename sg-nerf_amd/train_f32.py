"""The fp32 training step on hand-written kernels (precision "f32").

The reference's step (`optimize_parameters`, models/base_rendering_model.py:534-664;
models/mvs_points_volumetric_model.py:47-141) runs the aggregator, colour MLP, ray march and
losses forward in fp32 and differentiates them with torch autograd.  `F32Step` runs the same
arithmetic as a fixed sequence of HIP launches (csrc/train_x3.hip, csrc/mlp_x3.hip, csrc/loss.hip)
with every count kept on the device -- no host synchronisation, so the whole step can be replayed
as one captured graph:

  sgn_train_lists            deterministic work list + compact row offsets (prefix sums)
  sgn_aggregate_train_fwd_f32  k_pair_slots + k_rows16 (save mode): alpha_s, f_s, z1 / z2 / z3 rows
                             (SG: _sg, + block2_bpnet.0's zb)
  sgn_train_row_inputs       x0 = [emb | PE(emb) | PE(dists) | 1], extra channels, blend weights,
                             PE(viewdir); SG: sgn_train_row_gather, the rows' BPNet embedding
  colour forward             3 x sgn_x3_gemm (x W^T + b, LeakyReLU) + sgn_train_colour_head (rgb)
  sgn_loss_train             ray_dist + ray_march + losses and d feat, d conf (zero-one)
  colour backward            sgn_train_colour_head_bwd, 3 x dy W (masked), 3 x dy^T x (split-K)
  row backward               z4 = LReLU(z3) W3^T + b3; sgn_train_row_head (alpha, K-blend, delta4,
                             d conf); 4 x delta W (masked; SG 5); sgn_train_row_tail (d emb /
                             colour / dir); 4 x delta^T x (split-K; SG 5)
  sgn_reduce_partials        every weight / bias gradient into the flat gradient, fixed order

Rows r are the valid (sample, neighbour) pairs, sample-major (sample s owns rows
row_off[s] .. row_off[s] + samp_nnb[s]); items are the samples with a neighbour, ascending.
"""
import ctypes
import os

import torch

from . import _lib

# split-K partials of the weight-gradient GEMMs (rows / items cut into this many 32-aligned runs;
# 84 x 3 column blocks = one workgroup per CU for the row layers).  SGN_SPLITS_ROWS / _ITEMS
# override them for sweeps (tools/splits_sweep.sh).
SPLITS_ROWS = int(os.environ.get("SGN_SPLITS_ROWS", "84"))
SPLITS_ITEMS = int(os.environ.get("SGN_SPLITS_ITEMS", "128"))


def _addr(t, elem_off=0):
    return t.data_ptr() + elem_off * t.element_size()


def _operand(p, ld, ncols, kmajor, p2=None, ld2=0, csplit=None, ones_col=-1, act=0, amax=None, shift=None):
    o = _lib.X3Operand()
    o.p, o.p2 = p, p2
    o.ld, o.ld2 = int(ld), int(ld2)
    o.csplit = int(ncols if csplit is None else csplit)
    o.ncols, o.ones_col, o.act, o.kmajor = int(ncols), int(ones_col), int(act), int(kmajor)
    o.amax, o.shift = amax, shift
    return o


def _rows_gemm(a, b, M, N, K, rows, out, ldo, bias=None, act=0, mask=None, ldm=0, out_cols=None, out2=None, ldo2=0,
               amax_out=None, amax_out2=None):
    g = _lib.X3GemmArgs()
    g.a, g.b = a, b
    g.mode, g.M, g.N, g.K = 0, int(M), int(N), int(K)
    g.d_rows, g.bias, g.act, g.mask, g.ldm = rows, bias, int(act), mask, int(ldm)
    g.out, g.ldo = out, int(ldo)
    g.out_cols = int(N if out_cols is None else out_cols)
    g.out2, g.ldo2, g.amax_out, g.amax_out2 = out2, int(ldo2), amax_out, amax_out2
    return g


def _splitk_gemm(a, b, M, N, K, rows, part, splits):
    g = _lib.X3GemmArgs()
    g.a, g.b = a, b
    g.mode, g.M, g.N, g.K = 1, int(M), int(N), int(K)
    g.d_rows, g.part, g.splits = rows, part, int(splits)
    g.out_cols = int(N)
    return g


def _attach_bpack(gemms, device):
    """One workspace for the rows-mode launches' weight images (sgn_x3_gemm's bpack: the weight blocks are
    split once per call by a small launch, then DMA'd into every workgroup's LDS).  The launches run in
    stream order, so they share it.  Returns the buffer (keep it alive with the arguments)."""
    L = _lib.lib()
    rows = [g for g in gemms if g.mode == 0]
    n = max([int(L.sgn_x3_gemm_bpack_bytes(ctypes.byref(g))) for g in rows] + [16])
    buf = torch.empty(n, dtype=torch.uint8, device=device)
    for g in rows:
        g.bpack = buf.data_ptr()
    return buf


class F32Step:
    """Device buffers and pre-built launch arguments of the fp32 step for one batch capacity
    (R rays x SR samples x K neighbours), bound to one trainer's parameters and one query
    workspace.  `run` issues the step's launches on the current stream."""

    # amax words (max |x| of a delta tensor, written by its producer, read by its consumers)
    A_DY3, A_DY2, A_DY1, A_D4, A_D3, A_D2, A_D1, A_DB = range(8)

    def __init__(self, trainer, q, R):
        L = _lib.lib()
        o = trainer.opts
        self.trainer, self.R, self.K = trainer, R, o.K
        # SG-NeRF's block2_bpnet.0 between block1.2 and block3.0 (point_aggregators.py:345-354)
        self.sg, self.D = trainer.sg, trainer.variant[1]
        dev = trainer.device
        self.cap = cap = max(R * o.SR, 1)
        self.rows_cap = rows = cap * o.K
        self.q = q
        self.qo = q.abi()
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.row_off = torch.zeros(cap, **i32)
        self.counts = torch.zeros(4, **i32)
        self.lists_ws = torch.empty(int(L.sgn_train_lists_workspace_bytes(cap)), dtype=torch.uint8, device=dev)
        self.feat = torch.zeros(cap, 4, **f32)
        self.z = [torch.empty(rows, 256, **f32) for _ in range(4)]     # z1, z2, z3, z4 -> delta4
        if self.sg:   # block2_bpnet.0's pre-activation and delta, the rows' BPNet embedding
            self.zb = torch.empty(rows, 256, **f32)
            self.db = torch.empty(rows, 256, **f32)
            self.bprow = torch.empty(rows, self.D, **f32) if self.D else None
        self.ws32 = torch.empty(int(L.sgn_aggregate_workspace_bytes_f32(cap)), dtype=torch.uint8, device=dev)
        # k_rows16's blended features: fp32 [cap][256] inside the workspace (the ABI names where)
        fs_off = int(L.sgn_aggregate_fs_offset_f32(self.ws32.numel(), cap))
        assert fs_off >= 0, "the aggregate workspace must hold every item's f_s row"
        self.fs = self.ws32[fs_off:fs_off + cap * 256 * 4].view(torch.float32).view(cap, 256)
        self.x0 = torch.empty(rows, 288, **f32)
        self.ext = torch.empty(rows, 8, **f32)
        self.rw = torch.empty(rows, 2, **f32)
        self.vpe = torch.empty(cap, 32, **f32)
        self.h = [torch.empty(cap, 128, **f32) for _ in range(3)]       # colour h1, h2, h3
        self.dy = [torch.empty(cap, 128, **f32) for _ in range(3)]      # colour dy1, dy2, dy3
        self.dfs = torch.empty(cap, 256, **f32)
        self.d = [torch.empty(rows, 256, **f32) for _ in range(3)]      # delta1, delta2, delta3
        self.dext = torch.empty(rows, 8, **f32)
        self.dx0 = torch.empty(rows, 224, **f32)
        self.amax = torch.zeros(16, dtype=torch.int32, device=dev)
        self.dfeat = torch.empty(cap, 4, **f32)
        self.losses = torch.zeros(8, **f32)
        self.full = torch.empty(max(R, 1), 3, **f32)
        self.mask = torch.empty(max(R, 1), dtype=torch.int8, device=dev)
        self.loss_ws = torch.empty(max(int(L.sgn_loss_workspace_bytes(R, o.SR)), 16), dtype=torch.uint8, device=dev)
        self.part_rows = [torch.empty(SPLITS_ROWS, 256, n, **f32)
                          for n in (257, 264, 257, 285) + ((257 + self.D,) if self.sg else ())]
        self.part_col = [torch.empty(SPLITS_ITEMS, 128, n, **f32) for n in (129, 129, 281)]
        self.part_c6 = torch.empty(int(L.sgn_train_head_partial_floats(0)), **f32)
        self.part_a = torch.empty(int(L.sgn_train_head_partial_floats(1)), **f32)
        self._build()

    # -- the launch arguments (pointers of persistent buffers: built once) ----------------------
    def _build(self):
        tr = self.trainer
        m, flat, shift = tr.mlp, tr.mlp.flat, tr.packer32.shift
        g = flat.grad
        layer_ix = {name: i for i, (name, *_) in enumerate(m.layers)}

        def W(name):
            off, o, i = m.slices[name]
            return _addr(flat, off), o, i

        def Bv(name):
            off, o, i = m.slices[name]
            return _addr(flat, off + o * i)

        def S(name):
            return _addr(shift, layer_ix[name])

        amax = [_addr(self.amax, i) for i in range(16)]
        n_items, n_rows = _addr(self.counts, 0), _addr(self.counts, 1)
        cap, rc = self.cap, self.rows_cap
        h1, h2, h3 = (_addr(t) for t in self.h)
        dy1, dy2, dy3 = (_addr(t) for t in self.dy)
        z1, z2, z3, z4 = (_addr(t) for t in self.z)
        d1, d2, d3 = (_addr(t) for t in self.d)
        fs, vpe = _addr(self.fs), _addr(self.vpe)
        G = []
        # ---- colour forward: h = LReLU(x W^T + b) ----------------------------------------------
        w, o_, i_ = W("color_branch.0")
        G.append(("cf0", _rows_gemm(_operand(fs, 256, 280, 0, p2=vpe, ld2=32, csplit=256),
                                    _operand(w, i_, i_, 0, shift=S("color_branch.0")), cap, o_, i_, n_items, h1, 128,
                                    bias=Bv("color_branch.0"), act=1)))
        for name, x, y in (("color_branch.2", h1, h2), ("color_branch.4", h2, h3)):
            w, o_, i_ = W(name)
            G.append(("cf", _rows_gemm(_operand(x, 128, 128, 0), _operand(w, i_, i_, 0, shift=S(name)), cap, o_, i_,
                                       n_items, y, 128, bias=Bv(name), act=1)))
        self.g_colour_fwd = G
        # ---- colour backward: dy_prev = (dy W) * LReLU'(h_prev); d f_s = dy1 W0[:, :256] ----------
        G = []
        for name, dyi, mk, dyo, ai, ao in (("color_branch.4", dy3, h2, dy2, self.A_DY3, self.A_DY2),
                                           ("color_branch.2", dy2, h1, dy1, self.A_DY2, self.A_DY1)):
            w, o_, i_ = W(name)
            G.append((name, _rows_gemm(_operand(dyi, 128, 128, 0, amax=amax[ai]), _operand(w, i_, i_, 1, shift=S(name)),
                                       cap, i_, o_, n_items, dyo, 128, mask=mk, ldm=128, amax_out=amax[ao])))
        w, o_, i_ = W("color_branch.0")
        G.append(("dfs", _rows_gemm(_operand(dy1, 128, 128, 0, amax=amax[self.A_DY1]),
                                    _operand(w, i_, 256, 1, shift=S("color_branch.0")), cap, 256, o_, n_items,
                                    _addr(self.dfs), 256)))
        # colour weight gradients (split-K over the items)
        pc = self.part_col
        G.append(("dWc4", _splitk_gemm(_operand(dy3, 128, 128, 1, amax=amax[self.A_DY3]),
                                       _operand(h2, 128, 128, 1, ones_col=128), 128, 129, cap, n_items, _addr(pc[0]),
                                       SPLITS_ITEMS)))
        G.append(("dWc2", _splitk_gemm(_operand(dy2, 128, 128, 1, amax=amax[self.A_DY2]),
                                       _operand(h1, 128, 128, 1, ones_col=128), 128, 129, cap, n_items, _addr(pc[1]),
                                       SPLITS_ITEMS)))
        G.append(("dWc0", _splitk_gemm(_operand(dy1, 128, 128, 1, amax=amax[self.A_DY1]),
                                       _operand(fs, 256, 281, 1, p2=vpe, ld2=32, csplit=256), 128, 281, cap, n_items,
                                       _addr(pc[2]), SPLITS_ITEMS)))
        self.g_colour_bwd = G
        # ---- block3.2 forward again: z4 = LReLU(z3) W3^T + b3 -----------------------------------
        w, o_, i_ = W("block3.2")
        self.g_z4 = _rows_gemm(_operand(z3, 256, 256, 0, act=1), _operand(w, i_, i_, 0, shift=S("block3.2")), rc, o_, i_,
                               n_rows, z4, 256, bias=Bv("block3.2"))
        # ---- row backward chain ----------------------------------------------------------------
        G = []
        w, o_, i_ = W("block3.2")
        G.append(("d3", _rows_gemm(_operand(z4, 256, 256, 0, amax=amax[self.A_D4]), _operand(w, i_, i_, 1, shift=S("block3.2")),
                                   rc, 256, 256, n_rows, d3, 256, mask=z3, ldm=256, amax_out=amax[self.A_D3])))
        w, o_, i_ = W("block3.0")
        if self.sg:   # block3.0's input is block2_bpnet.0's output: its delta, then block1.2's
            db, zb = _addr(self.db), _addr(self.zb)
            G.append(("db", _rows_gemm(_operand(d3, 256, 256, 0, amax=amax[self.A_D3]),
                                       _operand(w, i_, i_, 1, shift=S("block3.0")), rc, 263, 256, n_rows, db, 256, mask=zb,
                                       ldm=256, out_cols=256, out2=_addr(self.dext), ldo2=8, amax_out=amax[self.A_DB])))
            w, o_, i_ = W("block2_bpnet.0")
            G.append(("d2", _rows_gemm(_operand(db, 256, 256, 0, amax=amax[self.A_DB]),
                                       _operand(w, i_, 256, 1, shift=S("block2_bpnet.0")), rc, 256, 256, n_rows, d2, 256,
                                       mask=z2, ldm=256, amax_out=amax[self.A_D2])))
        else:
            G.append(("d2", _rows_gemm(_operand(d3, 256, 256, 0, amax=amax[self.A_D3]),
                                       _operand(w, i_, i_, 1, shift=S("block3.0")), rc, 263, 256, n_rows, d2, 256, mask=z2,
                                       ldm=256, out_cols=256, out2=_addr(self.dext), ldo2=8, amax_out=amax[self.A_D2])))
        w, o_, i_ = W("block1.2")
        G.append(("d1", _rows_gemm(_operand(d2, 256, 256, 0, amax=amax[self.A_D2]), _operand(w, i_, i_, 1, shift=S("block1.2")),
                                   rc, 256, 256, n_rows, d1, 256, mask=z1, ldm=256, amax_out=amax[self.A_D1])))
        w, o_, i_ = W("block1.0")
        G.append(("dx0", _rows_gemm(_operand(d1, 256, 256, 0, amax=amax[self.A_D1]), _operand(w, i_, 224, 1, shift=S("block1.0")),
                                    rc, 224, 256, n_rows, _addr(self.dx0), 224)))
        self.g_row_bwd = G
        # ---- row weight gradients: delta^T [x | 1] ---------------------------------------------
        pr = self.part_rows
        self.g_row_dw = [
            _splitk_gemm(_operand(z4, 256, 256, 1, amax=amax[self.A_D4]), _operand(z3, 256, 256, 1, ones_col=256, act=1),
                         256, 257, rc, n_rows, _addr(pr[0]), SPLITS_ROWS),
            _splitk_gemm(_operand(d3, 256, 256, 1, amax=amax[self.A_D3]),
                         _operand(_addr(self.zb) if self.sg else z2, 256, 264, 1, p2=_addr(self.ext), ld2=8, csplit=256,
                                  act=1), 256, 264, rc, n_rows, _addr(pr[1]), SPLITS_ROWS),
            _splitk_gemm(_operand(d2, 256, 256, 1, amax=amax[self.A_D2]), _operand(z1, 256, 256, 1, ones_col=256, act=1),
                         256, 257, rc, n_rows, _addr(pr[2]), SPLITS_ROWS),
            _splitk_gemm(_operand(d1, 256, 256, 1, amax=amax[self.A_D1]), _operand(_addr(self.x0), 288, 285, 1),
                         256, 285, rc, n_rows, _addr(pr[3]), SPLITS_ROWS)]
        if self.sg:   # block2_bpnet.0: delta_b^T [LReLU(z2) | BPNet embedding | 1]
            D = self.D
            xb = (_operand(z2, 256, 256 + D, 1, p2=_addr(self.bprow), ld2=D, csplit=256, ones_col=256 + D, act=1) if D
                  else _operand(z2, 256, 256, 1, ones_col=256, act=1))
            self.g_row_dw.append(_splitk_gemm(_operand(_addr(self.db), 256, 256, 1, amax=amax[self.A_DB]), xb, 256, 257 + D,
                                              rc, n_rows, _addr(pr[4]), SPLITS_ROWS))
        # ---- partials -> flat gradient ----------------------------------------------------------
        segs = []

        def seg(part, splits, M, N, name, n_in, bias_col):
            off, o_, i_ = m.slices[name]
            s = _lib.PartialSegment()
            s.part, s.splits, s.M, s.N, s.n_in, s.bias_col, s.ldw = part, splits, M, N, n_in, bias_col, i_
            s.dst_w, s.dst_b = _addr(g, off), _addr(g, off + o_ * i_)
            segs.append(s)
        seg(_addr(pc[0]), SPLITS_ITEMS, 128, 129, "color_branch.4", 128, 128)
        seg(_addr(pc[1]), SPLITS_ITEMS, 128, 129, "color_branch.2", 128, 128)
        seg(_addr(pc[2]), SPLITS_ITEMS, 128, 281, "color_branch.0", 280, 280)
        hb = self.part_c6.numel() // (3 * 129)
        seg(_addr(self.part_c6), hb, 3, 129, "color_branch.6", 128, 128)
        seg(_addr(self.part_a), self.part_a.numel() // 257, 1, 257, "alpha_branch.0", 256, 256)
        seg(_addr(pr[0]), SPLITS_ROWS, 256, 257, "block3.2", 256, 256)
        seg(_addr(pr[1]), SPLITS_ROWS, 256, 264, "block3.0", 263, 263)
        seg(_addr(pr[2]), SPLITS_ROWS, 256, 257, "block1.2", 256, 256)
        seg(_addr(pr[3]), SPLITS_ROWS, 256, 285, "block1.0", 284, 284)
        if self.sg:
            seg(_addr(pr[4]), SPLITS_ROWS, 256, 257 + self.D, "block2_bpnet.0", 256 + self.D, 256 + self.D)
        self.segs = (_lib.PartialSegment * len(segs))(*segs)
        self.n_seg = len(segs)
        self.w6, self.b6 = W("color_branch.6")[0], Bv("color_branch.6")
        self.wa, self.ba = W("alpha_branch.0")[0], Bv("alpha_branch.0")
        self.grad_key = (flat.data_ptr(), g.data_ptr())
        self.bpack = _attach_bpack([gs for _, gs in self.g_colour_fwd + self.g_colour_bwd + self.g_row_bwd] +
                                   [self.g_z4] + self.g_row_dw, flat.device)

    # -- one step ------------------------------------------------------------------------------
    def run(self, pt, proj, blob, campos, rot, gt, lp):
        """Forward + backward of one batch after the query (gradients added into flat.grad and the
        point gradients; those must be zero / as the caller wants them).  Returns the device loss
        vector (sgn_loss_train's 8 floats), the rendered colour [R, 3] and the ray mask [R] (int8)."""
        L = _lib.lib()
        st = _lib.stream_handle()
        tr, K, qo = self.trainer, self.K, self.qo
        P = tr.points
        ck = _lib.check
        cap, p = self.cap, _lib.ptr

        def gemm(gs):
            ck(L.sgn_x3_gemm(ctypes.byref(gs), st), "sgn_x3_gemm")

        self.amax.zero_()
        ck(L.sgn_train_lists(p(self.q.counters), p(self.q.samp_nnb), cap, p(self.q.work), p(self.row_off), p(self.feat),
                             p(self.counts), p(self.lists_ws), st), "sgn_train_lists")
        if self.sg:
            ck(L.sgn_aggregate_train_fwd_f32_sg(1, self.D, p(tr.bpnet32) if self.D else None, p(proj), ctypes.byref(pt),
                                                ctypes.byref(qo), cap, K, p(blob), p(self.feat), p(self.z[0]),
                                                p(self.z[1]), p(self.zb), p(self.z[2]), p(self.row_off), p(self.ws32),
                                                self.ws32.numel(), st), "sgn_aggregate_train_fwd_f32_sg")
        else:
            ck(L.sgn_aggregate_train_fwd_f32(p(proj), ctypes.byref(pt), ctypes.byref(qo), cap, K, p(blob), p(self.feat),
                                             p(self.z[0]), p(self.z[1]), p(self.z[2]), p(self.row_off), p(self.ws32),
                                             self.ws32.numel(), st), "sgn_aggregate_train_fwd_f32")
        ck(L.sgn_train_row_inputs(ctypes.byref(pt), ctypes.byref(qo), K, p(self.row_off), p(self.counts), p(self.x0),
                                  p(self.ext), p(self.rw), p(self.vpe), st), "sgn_train_row_inputs")
        if self.D:
            ck(L.sgn_train_row_gather(ctypes.byref(qo), K, p(self.row_off), p(self.counts), p(tr.bpnet32), self.D,
                                      p(self.bprow), st), "sgn_train_row_gather")
        for _, gs in self.g_colour_fwd:
            gemm(gs)
        ck(L.sgn_train_colour_head(ctypes.byref(qo), p(self.counts), p(self.h[2]), self.w6, self.b6, p(self.feat), st),
           "sgn_train_colour_head")
        ck(L.sgn_loss_train(ctypes.byref(lp), p(campos), p(rot), self.R, ctypes.byref(qo), p(self.feat), p(gt),
                            p(P.points_conf), p(self.full), p(self.mask), p(self.losses), p(self.dfeat),
                            p(P.points_conf.grad), p(self.loss_ws), self.loss_ws.numel(), st), "sgn_loss_train")
        ck(L.sgn_train_colour_head_bwd(ctypes.byref(qo), p(self.counts), p(self.h[2]), self.w6, self.b6, p(self.dfeat),
                                       p(self.dy[2]), ctypes.c_void_p(_addr(self.amax, self.A_DY3)), p(self.part_c6), st),
           "sgn_train_colour_head_bwd")
        for _, gs in self.g_colour_bwd:
            gemm(gs)
        gemm(self.g_z4)
        ck(L.sgn_train_row_head(ctypes.byref(pt), ctypes.byref(qo), K, p(self.row_off), p(self.counts), p(self.z[3]),
                                p(self.dfs), p(self.dfeat), p(self.rw), self.wa, self.ba, p(P.points_conf.grad),
                                ctypes.c_void_p(_addr(self.amax, self.A_D4)), p(self.part_a), st), "sgn_train_row_head")
        for _, gs in self.g_row_bwd:
            gemm(gs)
        grads = _lib.PointGrads(P.points_embeding.grad.data_ptr(), P.points_color.grad.data_ptr(),
                                P.points_dir.grad.data_ptr(), P.points_conf.grad.data_ptr())
        ck(L.sgn_train_row_tail(ctypes.byref(pt), ctypes.byref(qo), K, p(self.row_off), p(self.counts), p(self.dx0),
                                p(self.dext), ctypes.byref(grads), st), "sgn_train_row_tail")
        for gs in self.g_row_dw:
            gemm(gs)
        ck(L.sgn_reduce_partials(self.n_seg, self.segs, st), "sgn_reduce_partials")
        return self.losses, self.full[:self.R], self.mask[:self.R]


class ColourStep:
    """The colour MLP, the losses and their backward for the f16 training step on the same hand-written
    kernels as F32Step (precision "f16" only changes the row MLP): items are the query's work-list
    positions (k_agg_rows' f_s rows), `cap` of them at most, the device count at q.counters[1].
    Per step (PE(viewdir) arrives from sgn_colour_inputs): 3 x sgn_x3_gemm forward + sgn_train_colour_head
    (rgb into feat), sgn_loss_train,
    the colour backward (head, 2 masked dy W, d f_s = dy1 W0[:, :256]; one fp16 product per multiply-add,
    the step's delta precision), the three weight gradients as
    split-K partials and one sgn_reduce_partials into the flat gradient.  No autograd, no host sync: it
    runs inside the f16 step's captured graph."""

    A_DY3, A_DY2, A_DY1 = range(3)

    def __init__(self, trainer, q, cap, fs32, vdir, feat, R, products=1):
        """products: of the backward GEMMs, 1 (the f16 step's delta precision: one fp16 product per
        multiply-add) or 3 (split-fp16 at fp32 accuracy); the forward keeps 3, so the rendered colour and
        the losses are the eager fp32 colour MLP's."""
        L = _lib.lib()
        self.trainer, self.q, self.cap, self.R = trainer, q, max(cap, 1), R
        self.products = products
        self.qo = q.abi()
        dev = trainer.device
        f32 = dict(dtype=torch.float32, device=dev)
        cap = self.cap
        self.fs32, self.vdir, self.feat = fs32, vdir, feat
        self.vpe = torch.zeros(cap, 32, **f32)     # sgn_colour_inputs: PE(viewdir), the ones column 24, zeros
        self.h = [torch.empty(cap, 128, **f32) for _ in range(3)]
        self.dy = [torch.empty(cap, 128, **f32) for _ in range(3)]
        self.dfs = torch.empty(cap, 256, **f32)
        self.amax = torch.zeros(4, dtype=torch.int32, device=dev)
        self.dfeat = torch.zeros(feat.shape[0] + 1, 4, **f32)   # + the padding items' zero row
        self.losses = torch.zeros(8, **f32)
        self.full = torch.empty(max(R, 1), 3, **f32)
        self.mask = torch.empty(max(R, 1), dtype=torch.int8, device=dev)
        self.loss_ws = torch.empty(max(int(L.sgn_loss_workspace_bytes(R, trainer.opts.SR)), 16), dtype=torch.uint8,
                                   device=dev)
        self.part_col = [torch.empty(SPLITS_ITEMS, 128, n, **f32) for n in (129, 129, 281)]
        self.part_c6 = torch.empty(int(L.sgn_train_head_partial_floats(0)), **f32)
        self._build()

    def _build(self):
        tr = self.trainer
        m, flat, shift = tr.mlp, tr.mlp.flat, tr.packer32.shift
        g = flat.grad
        layer_ix = {name: i for i, (name, *_) in enumerate(m.layers)}

        def W(name):
            off, o, i = m.slices[name]
            return _addr(flat, off), o, i

        def Bv(name):
            off, o, i = m.slices[name]
            return _addr(flat, off + o * i)

        def S(name):
            return _addr(shift, layer_ix[name])

        amax = [_addr(self.amax, i) for i in range(4)]
        n_items = _addr(self.q.counters, 1)         # the work-list length
        cap = self.cap
        h1, h2, h3 = (_addr(t) for t in self.h)
        dy1, dy2, dy3 = (_addr(t) for t in self.dy)
        fs, vpe = _addr(self.fs32), _addr(self.vpe)
        w, o_, i_ = W("color_branch.0")
        G = [_rows_gemm(_operand(fs, 256, 280, 0, p2=vpe, ld2=32, csplit=256), _operand(w, i_, i_, 0, shift=S("color_branch.0")),
                        cap, o_, i_, n_items, h1, 128, bias=Bv("color_branch.0"), act=1)]
        for name, x, y in (("color_branch.2", h1, h2), ("color_branch.4", h2, h3)):
            w, o_, i_ = W(name)
            G.append(_rows_gemm(_operand(x, 128, 128, 0), _operand(w, i_, i_, 0, shift=S(name)), cap, o_, i_, n_items,
                                y, 128, bias=Bv(name), act=1))
        self.g_fwd = G
        G = []
        for name, dyi, mk, dyo, ai, ao in (("color_branch.4", dy3, h2, dy2, self.A_DY3, self.A_DY2),
                                           ("color_branch.2", dy2, h1, dy1, self.A_DY2, self.A_DY1)):
            w, o_, i_ = W(name)
            G.append(_rows_gemm(_operand(dyi, 128, 128, 0, amax=amax[ai]), _operand(w, i_, i_, 1, shift=S(name)), cap, i_, o_,
                                n_items, dyo, 128, mask=mk, ldm=128, amax_out=amax[ao]))
        w, o_, i_ = W("color_branch.0")
        G.append(_rows_gemm(_operand(dy1, 128, 128, 0, amax=amax[self.A_DY1]), _operand(w, i_, 256, 1, shift=S("color_branch.0")),
                            cap, 256, o_, n_items, _addr(self.dfs), 256))
        pc = self.part_col
        G.append(_splitk_gemm(_operand(dy3, 128, 128, 1, amax=amax[self.A_DY3]), _operand(h2, 128, 128, 1, ones_col=128),
                              128, 129, cap, n_items, _addr(pc[0]), SPLITS_ITEMS))
        G.append(_splitk_gemm(_operand(dy2, 128, 128, 1, amax=amax[self.A_DY2]), _operand(h1, 128, 128, 1, ones_col=128),
                              128, 129, cap, n_items, _addr(pc[1]), SPLITS_ITEMS))
        G.append(_splitk_gemm(_operand(dy1, 128, 128, 1, amax=amax[self.A_DY1]),
                              _operand(fs, 256, 281, 1, p2=vpe, ld2=32, csplit=256), 128, 281, cap, n_items, _addr(pc[2]),
                              SPLITS_ITEMS))
        self.g_bwd = G
        for gs in self.g_bwd:
            gs.products = self.products
        segs = []

        def seg(part, splits, M, N, name, n_in, bias_col):
            off, o_, i_ = m.slices[name]
            s = _lib.PartialSegment()
            s.part, s.splits, s.M, s.N, s.n_in, s.bias_col, s.ldw = part, splits, M, N, n_in, bias_col, i_
            s.dst_w, s.dst_b = _addr(g, off), _addr(g, off + o_ * i_)
            segs.append(s)
        seg(_addr(pc[0]), SPLITS_ITEMS, 128, 129, "color_branch.4", 128, 128)
        seg(_addr(pc[1]), SPLITS_ITEMS, 128, 129, "color_branch.2", 128, 128)
        seg(_addr(pc[2]), SPLITS_ITEMS, 128, 281, "color_branch.0", 280, 280)
        seg(_addr(self.part_c6), self.part_c6.numel() // (3 * 129), 3, 129, "color_branch.6", 128, 128)
        self.segs = (_lib.PartialSegment * len(segs))(*segs)
        self.n_seg = len(segs)
        self.w6, self.b6 = W("color_branch.6")[0], Bv("color_branch.6")
        self.bpack = _attach_bpack(self.g_fwd + self.g_bwd, flat.device)

    def run(self, campos, rot, gt, lp):
        """Colour forward into feat[.].yzw, the losses, the colour backward: returns the loss vector
        (sgn_loss_train's 8 floats), full [R, 3], mask [R] (int8), d f_s [cap, 256] and d feat [S, 4]
        (alpha's gradient in .x); the colour weight gradients are added into flat.grad, the zero-one
        gradients into points_conf.grad."""
        L = _lib.lib()
        st = _lib.stream_handle()
        ck, p = _lib.check, _lib.ptr
        tr, qo = self.trainer, self.qo
        P = tr.points
        cnt = ctypes.c_void_p(_addr(self.q.counters, 1))
        # self.vpe (PE(viewdir) | 1 | 0) was written by sgn_colour_inputs with the items' other inputs
        self.amax.zero_()
        for gs in self.g_fwd:
            ck(L.sgn_x3_gemm(ctypes.byref(gs), st), "sgn_x3_gemm")
        ck(L.sgn_train_colour_head(ctypes.byref(qo), cnt, p(self.h[2]), self.w6, self.b6, p(self.feat), st),
           "sgn_train_colour_head")
        ck(L.sgn_loss_train(ctypes.byref(lp), p(campos), p(rot), self.R, ctypes.byref(qo), p(self.feat), p(gt),
                            p(P.points_conf), p(self.full), p(self.mask), p(self.losses), p(self.dfeat),
                            p(P.points_conf.grad), p(self.loss_ws), self.loss_ws.numel(), st), "sgn_loss_train")
        # d f_s of the padding items stays 0: the f16 backward's loss scale is the max over all cap rows
        self.dfs.zero_()
        ck(L.sgn_train_colour_head_bwd(ctypes.byref(qo), cnt, p(self.h[2]), self.w6, self.b6, p(self.dfeat), p(self.dy[2]),
                                       ctypes.c_void_p(_addr(self.amax, self.A_DY3)), p(self.part_c6), st),
           "sgn_train_colour_head_bwd")
        for gs in self.g_bwd:
            ck(L.sgn_x3_gemm(ctypes.byref(gs), st), "sgn_x3_gemm")
        ck(L.sgn_reduce_partials(self.n_seg, self.segs, st), "sgn_reduce_partials")
        return self.losses, self.full[:self.R], self.mask[:self.R], self.dfs, self.dfeat
