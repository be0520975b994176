"""Training step on the HIP kernels.

The reference trains through torch autograd (`optimize_parameters`,
models/base_rendering_model.py:534-664; models/mvs_points_volumetric_model.py:47-141).  Here the
whole step -- the NeuralPoints gather, the per-row MLP + alpha + K-blend of PointAggregator
(point_aggregators.py:868-959, :561-786), the colour MLP, ray_dist / ray_march and the losses,
and all their gradients -- runs as hand-written HIP launches; torch only allocates buffers and
all-reduces gradients.  Two arithmetic modes, as the renderer has:

precision "f32" (the reference's fp32 arithmetic; `_backward_f32`, train_f32.F32Step):
  query        sgn_query (jittered depths, is_train) -> the point Adam's launch (sgn_adam_rows: the
               previous step's deferred update, this step's rows brought forward, their distinct list)
  projection   sgn_point_project_f32_subset: block1.0's per-point part for that list's points only
  forward      k_rows16 in save mode (block1.0 / 1.2 / 3.0 pre-activations per row; SG: + block2_bpnet)
  colour+loss  the colour MLP on k_x3rows (3 fp16 products per fp32 product), sgn_loss_train
  backward     k_row_head / masked backward-data GEMMs / k_row_tail (point gradients), the split-K
               weight gradients on k_x3dw / k_x3tn and one fixed-order sgn_reduce_partials
  no host synchronisation on one GPU.

precision "f16" (fp16-operand MFMA, fp32 accumulation; `backward`):
  query        sgn_query -> the point Adam's launch, then the step's one host sync (sample /
               work-item counts, read after an event on the query's pinned copy)
  forward      sgn_aggregate_train_fwd (k_agg_rows save mode): f_s (fp16) and alpha per sample,
               the row layers' inputs saved
  colour+loss  one captured HIP graph (ColourStep: sgn_colour_inputs, the colour MLP on k_x3rows,
               sgn_loss_train, the colour backward and its weight gradients), or the same stage
               eagerly (use_graph = False) through loss_hip.LossStage and torch autograd of the
               colour MLP -- the graph's parity reference in the tests
  backward     sgn_aggregate_backward (k_agg_bwd): deltas of the 4 row layers, d alpha-logit, point
               gradients, under a power-of-two loss scale; dW = delta^T x per row layer on k_f16dw
               (sgn_f16_weight_grad, split-K fp32 partials) and the alpha branch's weighted column
               sums, all added into the flat gradient by one sgn_grad_accumulate

Both: bucketed all-reduce (RCCL) of the flat MLP gradient and a sparse all-gather of the touched
point rows under DP, then two Adam groups (lr 5e-4 / plr 2e-3, iter_exponential_decay): the MLP's
on sgn_adam_step_multi, the points' on the row-sparse exact sgn_adam_rows (PointAdam(rows=True):
bit-identical to the dense update, applied at the next step's launch or at a flush).  The plane background model's per-ray colour (inputs['bg_ray']) enters the
loss stage as T_bg * bg_ray.

MLP weights live in ONE flat fp32 parameter (LAYERS order), so the MFMA blobs are re-packed on
the device every step by index gathers (sgn_gather_segments / sgn_pack_scaled_f32).
"""
import ctypes
import gc
import os

import torch
import torch.nn as nn
import torch.distributed as dist
import torch.nn.functional as F

from . import _lib
from .opts import HotPathOpts
from .train import PointParams, _allreduce_buckets, _allreduce_point_rows, _pe, gather_counts, touched_rows
from .loss_hip import LossStage
from .weights import BPNET, LAYERS, layers_for, strip_prefix

N_F32 = 2056


class FlatMLP(nn.Module):
    """The 9 viewmlp layers (+ SG's block2_bpnet.0 after them) in one flat fp32 parameter: per
    layer weight (row-major) then bias."""

    def __init__(self, state, device, layers=LAYERS):
        super().__init__()
        state = strip_prefix(state)
        self.layers = list(layers)
        parts, self.slices, off = [], {}, 0
        for name, o, i, _ in self.layers:
            parts += [torch.as_tensor(state[name + ".weight"]).float().reshape(-1),
                      torch.as_tensor(state[name + ".bias"]).float().reshape(-1)]
            self.slices[name] = (off, o, i)
            off += o * i + o
        self.flat = nn.Parameter(torch.cat(parts).to(device))
        self._dst = {}   # grad_sink: flat-gradient index maps per layer

    def w(self, name, t=None):
        off, o, i = self.slices[name]
        return (self.flat if t is None else t)[off:off + o * i].view(o, i)

    def b(self, name, t=None):
        off, o, i = self.slices[name]
        return (self.flat if t is None else t)[off + o * i:off + o * i + o]

    def f(self, name, x):
        return F.linear(x, self.w(name), self.b(name))

    def grad_sink(self, name):
        """For train.aggregate (the fp32 step): a callable adding a layer's dW = gz^T x (split-K
        partials, one sgn_grad_accumulate launch) and db = sum gz into flat.grad; None for the
        alpha branch (one output unit: its dW stays an autograd GEMM, not an M = 1 batched GEMM)."""
        off, o, i = self.slices[name]
        g = self.flat.grad
        if g is None or o < 16:
            return None
        dst = self._dst.get(name)
        if dst is None:
            dst = self._dst[name] = (off + torch.arange(o * i, device=g.device)).to(torch.int32)

        def sink(gz, x):
            parts, tail = _fp32_rows_parts(gz, x, DW_CHUNK_COLOUR)
            _grad_into(g, dst, parts, tail)
            g[off + o * i:off + o * i + o].add_(gz.sum(0))
        return sink

    def state(self):
        out = {}
        for name, *_ in self.layers:
            out[name + ".weight"] = self.w(name).detach().clone()
            out[name + ".bias"] = self.b(name).detach().clone()
        return out


class _PackerF32:
    """Device-side packing of the fp32-faithful blob (mlp_x3.hip: (hi, lo) fp16 fragment pairs of
    2^s-scaled weights + the fp32 section) from the flat parameter, through the layout's index maps
    (sgn_mlp_pack_index_f32): per layer the shift s = 14 - e with max |W| = f 2^e (frexp), as
    layer_shift does on the host, then hi = fp16(2^s w), lo = fp16(2^s w - hi).  Equals
    weights.pack_mlp(state, precision="f32") bit for bit (tests/test_train_gpu.py)."""

    YK_ZERO, YK_W, YK_B, YK_BS, YK_INV, YK_ONE, YK_WINV = range(7)

    def __init__(self, device, mlp: "FlatMLP", variant=(0, 0)):
        L = _lib.lib()
        self.n16b = int(L.sgn_mlp_layout_f32(0))
        n32 = int(L.sgn_mlp_layout_f32(1))
        self.total = int(L.sgn_mlp_packed_bytes_f32(*variant))

        def imap(which, n):
            a = (ctypes.c_int32 * n)()
            _lib.check(L.sgn_mlp_pack_index_f32(*variant, which, a, n), "sgn_mlp_pack_index_f32")
            return torch.frombuffer(bytearray(a), dtype=torch.int32).long()
        # the maps are decoded and bounds-checked on the host; the device only gathers
        nl, nflat = len(mlp.layers), mlp.flat.numel()
        woff = torch.tensor([mlp.slices[n][0] for n, *_ in mlp.layers], dtype=torch.long)
        wlen = torch.tensor([mlp.slices[n][1] * mlp.slices[n][2] for n, *_ in mlp.layers], dtype=torch.long)
        blen = torch.tensor([mlp.slices[n][1] for n, *_ in mlp.layers], dtype=torch.long)
        self.wspan = [(int(a), int(a + b)) for a, b in zip(woff, wlen)]
        c16 = imap(0, self.n16b // 2)
        v16 = c16 >= 0
        c16 = torch.clamp(c16, min=0)
        l16 = (c16 >> 20) & 0x3FF
        assert int(l16[v16].max()) < nl, "fragment map names a layer the flat parameter lacks"
        l16 = torch.where(v16, l16, 0)
        e16 = torch.where(v16, c16 & 0xFFFFF, 0)
        assert bool((e16 < wlen[l16]).all()), "fragment map element out of range"
        c32 = imap(1, n32)
        k32 = c32 >> 26
        l32 = (c32 >> 20) & 63
        e32 = c32 & 0xFFFFF
        uses_w = (k32 == self.YK_W) | (k32 == self.YK_WINV)
        uses_b = (k32 == self.YK_B) | (k32 == self.YK_BS)
        uses_l = uses_w | uses_b | (k32 == self.YK_INV)
        assert int(l32[uses_l].max()) < nl, "fp32 map names a layer the flat parameter lacks"
        l32 = torch.where(uses_l, l32, 0)
        fw32 = torch.where(uses_w, woff[l32] + e32, 0)
        fb32 = torch.where(uses_b, woff[l32] + wlen[l32] + e32, 0)
        assert bool((e32[uses_w] < wlen[l32[uses_w]]).all() and (e32[uses_b] < blen[l32[uses_b]]).all())
        f16 = woff[l16] + e16
        assert int(f16.max()) < nflat and int(fw32.max()) < nflat and int(fb32.max()) < nflat
        assert nflat < (1 << 22) and nl <= 16 and int(k32.max()) <= self.YK_WINV
        # one int32 code per blob element for sgn_pack_scaled_f32: flat index | layer << 22 | lo / kind << 26
        code16 = torch.where(v16, f16 | (l16 << 22) | (((c16 >> 30) & 1) << 26), -1)
        code32 = torch.where(uses_w, fw32, fb32) | (l32 << 22) | (k32 << 26)
        self.code16 = code16.to(torch.int32).to(device)
        self.code32 = code32.to(torch.int32).to(device)
        self.n_layers = nl
        self.woff = (ctypes.c_int64 * nl)(*[int(a) for a, _ in self.wspan])
        self.wlen = (ctypes.c_int64 * nl)(*[int(b - a) for a, b in self.wspan])
        self.shift = torch.zeros(16, dtype=torch.int32, device=device)
        self.blob = torch.zeros(self.total, dtype=torch.uint8, device=device)
        assert self.n16b == 2 * self.code16.numel() and self.n16b + 4 * self.code32.numel() <= self.total

    def pack(self, flat):
        """Per-layer shifts and both blob sections from the flat parameter: two launches."""
        flat = flat.detach()
        assert flat.is_contiguous() and flat.dtype == torch.float32
        _lib.check(_lib.lib().sgn_pack_scaled_f32(
            _lib.ptr(flat), flat.numel(), self.n_layers, self.woff, self.wlen, _lib.ptr(self.code16), self.code16.numel(),
            _lib.ptr(self.code32), self.code32.numel(), _lib.ptr(self.shift), _lib.ptr(self.blob[:self.n16b]),
            _lib.ptr(self.blob[self.n16b:]), _lib.stream_handle()), "sgn_pack_scaled_f32")
        return self.blob


class _Packer:
    """Device-side re-packing of the forward and transposed MFMA blobs from the flat weights
    (variant (1, bpnet_dim): the SG blob, block2_bpnet.0's fragments and bias after the base)."""

    def __init__(self, device, variant=(0, 0)):
        L = _lib.lib()
        self.variant = variant
        self.base = int(L.sgn_mlp_packed_bytes())
        self.total = int(L.sgn_mlp_packed_bytes_sg(*variant)) if variant != (0, 0) else self.base
        self.off_f32 = int(L.sgn_mlp_section(0))
        self.off_split = int(L.sgn_mlp_section(1))
        self.tbytes = int(L.sgn_train_tblob_bytes())

        def imap(fn, name, *args, n):
            """The layout's index map (flat index + 1, 0 = zero) as flat indices (-1 = zero)."""
            a = (ctypes.c_int32 * n)()
            _lib.check(fn(*args, a, n), name)
            return (torch.frombuffer(bytearray(a), dtype=torch.int32) - 1).to(device)
        self.i16 = imap(L.sgn_mlp_pack_index, "sgn_mlp_pack_index", 0, n=self.off_f32 // 2)
        self.i32 = imap(L.sgn_mlp_pack_index, "sgn_mlp_pack_index", 1, n=N_F32)
        self.isp = imap(L.sgn_mlp_pack_index, "sgn_mlp_pack_index", 2, n=(self.base - self.off_split) // 2)
        if variant != (0, 0):
            self.off_bb = self.total - 4 * 256                   # block2_bpnet bias (fp32, acc order)
            self.iwb = imap(L.sgn_mlp_pack_index_sg, "sgn_mlp_pack_index_sg", *variant, 3,
                            n=(self.off_bb - self.base) // 2)
            self.ibb = imap(L.sgn_mlp_pack_index_sg, "sgn_mlp_pack_index_sg", *variant, 4, n=256)
            self.it = imap(L.sgn_train_pack_index_sg, "sgn_train_pack_index_sg", variant[1], n=self.tbytes // 2)
        else:
            self.it = imap(L.sgn_train_pack_index, "sgn_train_pack_index", n=self.tbytes // 2)
        self.blob = torch.zeros(self.total, dtype=torch.uint8, device=device)
        self.tblob = torch.zeros(self.tbytes, dtype=torch.uint8, device=device)
        # (index map, destination bytes, fp16?) -- every section of both blobs in one gather launch
        segs = [(self.i16, self.blob[:self.off_f32], 1), (self.i32, self.blob[self.off_f32:self.off_f32 + 4 * N_F32], 0),
                (self.isp, self.blob[self.off_split:self.base], 1)]
        if variant != (0, 0):
            segs += [(self.iwb, self.blob[self.base:self.off_bb], 1), (self.ibb, self.blob[self.off_bb:], 0)]
        segs.append((self.it, self.tblob, 1))
        for idx, dst, h in segs:
            assert dst.numel() == idx.numel() * (2 if h else 4)
        self._segs = (_lib.GatherSegment * len(segs))(*[_lib.GatherSegment(idx.data_ptr(), dst.data_ptr(), idx.numel(), h, 0)
                                                       for idx, dst, h in segs])

    def pack(self, flat):
        flat = flat.detach()
        assert flat.is_contiguous() and flat.dtype == torch.float32
        _lib.check(_lib.lib().sgn_gather_segments(len(self._segs), self._segs, _lib.ptr(flat), flat.numel(),
                                                  _lib.stream_handle()), "sgn_gather_segments")
        return self.blob, self.tblob


def _colmap(which, n, device):
    a = (ctypes.c_int32 * n)()
    _lib.check(_lib.lib().sgn_train_colmap(which, a, n), "sgn_train_colmap")
    return torch.frombuffer(bytearray(a), dtype=torch.int32).long().to(device)


# loss-stage graphs: capacity bucket (items / samples) and how many captured graphs are kept
GRAPH_BUCKET = int(os.environ.get("SGN_GRAPH_BUCKET", "8192"))
GRAPH_CACHE = 8


def _grad_into(g, dst, parts, tail=None, scale=None):
    """g[dst[j]] += (sum of the partials [nb, n] (+ tail)) (/ scale): one sgn_grad_accumulate launch."""
    n = dst.numel()
    seg = _lib.GradSegment(parts.data_ptr(), tail.data_ptr() if tail is not None else None, dst.data_ptr(), n, n,
                           parts.numel() // n, 0)
    _lib.check(_lib.lib().sgn_grad_accumulate(1, ctypes.byref(seg), _lib.ptr(scale), _lib.ptr(g),
                                              _lib.stream_handle()), "sgn_grad_accumulate")


class _LinearInto(torch.autograd.Function):
    """F.linear (fp32) of a weight / bias held in the flat parameter whose gradients the backward
    ADDS into the flat gradient (split-K weight partials through sgn_grad_accumulate, the bias sum
    in place) instead of returning them through autograd -- which would zero-fill a full-size
    gradient per parameter view, copy the slice in and add it back: six launches per layer."""

    @staticmethod
    def forward(ctx, x, w, b, g, dst_w, off_b):
        ctx.save_for_backward(x, w)
        ctx.g, ctx.dst_w, ctx.off_b = g, dst_w, off_b
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gz):
        x, w = ctx.saved_tensors
        gz = gz.contiguous()
        parts, tail = _fp32_rows_parts(gz, x, DW_CHUNK_COLOUR)
        _grad_into(ctx.g, ctx.dst_w, parts, tail)
        ctx.g[ctx.off_b:ctx.off_b + w.shape[0]].add_(gz.sum(0))
        return (gz @ w if ctx.needs_input_grad[0] else None), None, None, None, None, None


# rows per split-K batch of the colour layers' fp32 weight gradients
DW_CHUNK_COLOUR = int(os.environ.get("SGN_DW_CHUNK_COLOUR", "4096"))


def _fp32_rows_parts(gz, x, chunk):
    """gz^T x (fp32) over the rows as split-K partials ([nb, M, N], tail [M, N] or None)."""
    rows = gz.shape[0]
    nb = rows // chunk if chunk > 0 else 0
    if nb <= 1:
        return (gz.t() @ x)[None].contiguous(), None
    body = nb * chunk
    parts = torch.bmm(gz[:body].view(nb, chunk, gz.shape[1]).transpose(1, 2), x[:body].reshape(nb, chunk, x.shape[1]))
    tail = (gz[body:].t() @ x[body:]).contiguous() if body < rows else None
    return parts.contiguous(), tail


class PointAdam(torch.optim.Adam):
    """torch.optim.Adam (same param_groups, state keys and state_dict) whose step is one
    sgn_adam_step_multi launch per parameter group; with zero_grad the launch also clears the
    gradients, so the next step skips their fill pass.  For the dense ~47 M-element point group
    and the MLP's flat parameter."""

    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8, zero_grad=True, rows=False, flush_every=256):
        """rows: row-sparse exact mode (one group of <= 4 tensors sharing their first dimension, the
        points; sgn_adam_rows).  A row is brought forward only when something reads it, replaying the
        zero-gradient steps it missed, so it equals the dense update bit for bit whenever read.  The
        step's own update is deferred to the next step's first launch: set_rows(list) applies the
        pending step to the previous step's rows and brings the new list's rows to the current step in
        one pass; flush() (state_dict, the model's renders; every flush_every steps, which bounds the
        replay) brings every row.  The narrow tensors' moments (widths <= 8, e.g. colour, dir, conf: 7
        floats a row) share one [N, 16] buffer, m in columns 0-7 and v in 8-15, and the state holds views
        of it: a row's moments are one 64-byte access instead of six scattered 4-12 byte ones."""
        super().__init__(params, lr=lr, betas=betas, eps=eps)
        self.zero_grad_in_step = zero_grad
        self.rows_mode = rows
        if rows:
            ps = self.param_groups[0]["params"]
            if len(self.param_groups) != 1 or not 1 <= len(ps) <= 4:
                raise ValueError("PointAdam(rows=True): one parameter group of 1 .. 4 tensors")
            n = ps[0].shape[0]
            if any(p.shape[0] != n or not p.is_contiguous() or p.dtype != torch.float32 for p in ps):
                raise ValueError("PointAdam(rows=True): contiguous fp32 tensors sharing the first dimension")
            dev = ps[0].device
            self.n_rows = n
            widths = [p.numel() // n for p in ps]
            self._width = (ctypes.c_int32 * len(ps))(*widths)
            self._narrow, off = {}, 0   # tensor index -> its columns' offset in the packed moments
            for i, w in enumerate(widths):
                if w <= 8 and off + w <= 8:
                    self._narrow[i] = (off, w)
                    off += w
            self._mv = torch.zeros(n, 16, dtype=torch.float32, device=dev) if self._narrow else None
            self._mstride = (ctypes.c_int32 * len(ps))(*[16 if i in self._narrow else w for i, w in enumerate(widths)])
            self._last = torch.zeros(n, dtype=torch.int32, device=dev)   # the step each row holds
            self._claim = torch.zeros(n, dtype=torch.int32, device=dev)   # claim tags (launch tags start at 1)
            self._claim2 = torch.zeros(n, dtype=torch.int32, device=dev)
            self._sched = torch.zeros(2 * 1024, dtype=torch.float32, device=dev)
            self._ws = None
            self._pend = [None, None]   # two pend lists: the previous step's is read while the next is written
            self._pi = 0
            self._tag = 0
            self._rows = None           # the step's list (set_rows) once its rows are brought forward
            self._pending = None        # (pend buffer, length bound): the rows of the step not yet applied
            self._flushed = 0           # every row holds at least this step
            self.flush_every = flush_every

    # -- row-sparse mode ------------------------------------------------------------------------
    def _state_step(self):
        """The group's step count (0 before the first step); creates the state tensors."""
        for i, p in enumerate(self.param_groups[0]["params"]):
            s = self.state[p]
            if not s:
                s["step"] = torch.tensor(0.0)
                if i in self._narrow:
                    s["exp_avg"], s["exp_avg_sq"] = self._mv_views(i)
                else:
                    s["exp_avg"] = torch.zeros_like(p)
                    s["exp_avg_sq"] = torch.zeros_like(p)
        return int(self.state[self.param_groups[0]["params"][0]]["step"].item())

    def _mv_views(self, i):
        """Tensor i's exp_avg / exp_avg_sq as views of the packed narrow moments (zero at creation)."""
        o, w = self._narrow[i]
        return self._mv[:, o:o + w], self._mv[:, 8 + o:8 + o + w]

    def _buf(self, t, nbytes):
        if t is None or t.numel() < nbytes:
            t = torch.empty(nbytes, dtype=torch.uint8, device=self._last.device)
        return t

    def _launch(self, step, apply, rows=None, count=None, count_is64=False, count_mul=1, n_max=None, pend=False,
                lr=None):
        """One sgn_adam_rows call: list 1 (rows, or every row), the pending list as list 2 when applying a
        deferred step, row 0; with pend, list 1's distinct rows go to the next pend buffer."""
        g = self.param_groups[0]
        ps = g["params"]
        n = len(ps)
        arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() if t is not None else None for t in ts])  # noqa: E731
        if step >= self._sched.numel() // 2:   # grow the per-step constant table (entries kept)
            grown = torch.zeros(max(2 * self._sched.numel(), 2 * (step + 1)), dtype=torch.float32,
                                device=self._sched.device)
            grown[:self._sched.numel()] = self._sched
            self._sched = grown
        b1, b2 = g["betas"]
        self._tag = (self._tag + 1) & 0x7fffffff
        n_max = self.n_rows if n_max is None else n_max
        L = _lib.lib()
        prev = self._pending if apply and rows is not None else None
        lr = float(g["lr"]) if lr is None else lr
        n2 = prev[1] if prev is not None else 0
        self._ws = self._buf(self._ws, int(L.sgn_adam_rows_workspace_bytes(min(n_max + n2 + 1, self.n_rows))))
        pb = None
        if pend:
            self._pi ^= 1
            pb = self._pend[self._pi] = self._buf(self._pend[self._pi],
                                                  int(L.sgn_adam_rows_pend_bytes(min(n_max + 1, self.n_rows))))
        _lib.check(L.sgn_adam_rows(
            n, arr(ps), arr([p.grad if apply else None for p in ps]), arr([self.state[p]["exp_avg"] for p in ps]),
            arr([self.state[p]["exp_avg_sq"] for p in ps]), self._width, self._mstride, self.n_rows,
            _lib.ptr(rows) if rows is not None else None, _lib.ptr(count) if count is not None else None,
            int(count_is64), count_mul, n_max, 1,
            prev[0].data_ptr() + 16 if prev is not None else None, prev[0].data_ptr() if prev is not None else None,
            n2, _lib.ptr(self._last), _lib.ptr(self._claim), _lib.ptr(self._claim2), self._tag,
            _lib.ptr(self._ws), self._ws.numel(), _lib.ptr(pb) if pb is not None else None,
            pb.numel() if pb is not None else 0, _lib.ptr(self._sched), lr, b1, b2, float(g["eps"]),
            step, int(apply), int(self.zero_grad_in_step), _lib.stream_handle()), "sgn_adam_rows")
        return pb

    def set_rows(self, rows, count=None, count_is64=False, count_mul=1, n_max=None):
        """The rows the coming step reads and changes: an int32 device list (-1 / duplicates allowed)
        with its device count (int32 or int64, times count_mul) or host length n_max.  One launch
        applies the deferred previous step to its rows and brings these rows (and row 0) to the current
        step; returns the step's distinct rows (int32 from byte 16 of the returned buffer, int64 count
        at byte 0, list-1 ids >= n_rows at byte 8)."""
        assert self.rows_mode and rows.dtype == torch.int32 and rows.is_contiguous()
        n_max = rows.numel() if n_max is None else n_max
        t = self._state_step()
        pd = self._pending
        pb = self._launch(t, apply=pd is not None, rows=rows, count=count, count_is64=count_is64,
                          count_mul=count_mul, n_max=n_max, pend=True, lr=pd[2] if pd is not None else None)
        self._pending = None
        self._rows = (pb, min(n_max + 1, self.n_rows))
        return pb

    def set_update_rows(self, rows):
        """Under DP: the rows the step's update changes (every rank's, int32 device, host length) --
        they replace the step's pend list (a launch gathers their distinct rows now)."""
        assert self.rows_mode and rows.dtype == torch.int32 and rows.is_contiguous()
        t = self._state_step()
        pb = self._launch(t, apply=False, rows=rows, n_max=rows.numel(), pend=True)
        self._rows = (pb, min(rows.numel() + 1, self.n_rows))

    @torch.no_grad()
    def flush(self):
        """Bring every row to the current step (before anything outside the step reads the tensors)."""
        if not self.rows_mode:
            return
        t = self._state_step()
        pd = self._pending
        if pd is not None or t > self._flushed:
            self._launch(t, apply=pd is not None, lr=pd[2] if pd is not None else None)
            self._pending = None
            self._flushed = t

    def state_dict(self):
        self.flush()
        return super().state_dict()

    def zero_grad(self, set_to_none=True):
        """A deferred step reads its gradient at the next launch: apply it before the gradient goes."""
        if self.rows_mode and self._pending is not None:
            self.flush()
        super().zero_grad(set_to_none)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        if self.rows_mode:   # the loaded tensors are a dense state: every row holds its step
            for i, p in enumerate(self.param_groups[0]["params"]):
                s = self.state[p]
                if i in self._narrow and s:   # back into the packed moments
                    for key, view in zip(("exp_avg", "exp_avg_sq"), self._mv_views(i)):
                        view.copy_(s[key].reshape(view.shape))
                        s[key] = view
            t = self._state_step()
            self._last.fill_(t)
            self._flushed = t
            self._pending = None
            self._rows = None

    @torch.no_grad()
    def step(self, closure=None):
        """One sgn_adam_step_multi launch per parameter group (tensors sharing a step count); in the
        row-sparse mode the step is recorded as pending on the rows set_rows listed (applied by the next
        set_rows or flush), or applied to every row at once without such a list."""
        assert closure is None
        if self.rows_mode:
            if self._pending is not None:   # the previous step was never applied: its gradient is this one
                self.flush()
            t = self._state_step() + 1
            for p in self.param_groups[0]["params"]:
                self.state[p]["step"] += 1
            r = self._rows
            self._rows = None
            if r is None:
                self._launch(t, apply=True)
                self._flushed = t
            else:   # the step's lr travels with it: the update runs at the next set_rows / flush
                self._pending = (r[0], r[1], float(self.param_groups[0]["lr"]))
                if t - self._flushed >= self.flush_every:
                    self.flush()
            return None
        L = _lib.lib()
        st = _lib.stream_handle()
        for g in self.param_groups:
            b1, b2 = g["betas"]
            by_step = {}
            for p in g["params"]:
                if p.grad is None:
                    continue
                assert p.is_contiguous() and p.grad.is_contiguous() and p.dtype == torch.float32
                s = self.state[p]
                if not s:
                    s["step"] = torch.tensor(0.0)
                    s["exp_avg"] = torch.zeros_like(p)
                    s["exp_avg_sq"] = torch.zeros_like(p)
                s["step"] += 1
                by_step.setdefault(int(s["step"].item()), []).append(p)
            for step, ps in by_step.items():
                for i in range(0, len(ps), 8):
                    chunk = ps[i:i + 8]
                    n = len(chunk)
                    arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
                    _lib.check(L.sgn_adam_step_multi(
                        n, arr(chunk), arr([p.grad for p in chunk]), arr([self.state[p]["exp_avg"] for p in chunk]),
                        arr([self.state[p]["exp_avg_sq"] for p in chunk]), (ctypes.c_int64 * n)(*[p.numel() for p in chunk]),
                        float(g["lr"]), b1, b2, float(g["eps"]), step, int(self.zero_grad_in_step), st),
                        "sgn_adam_step_multi")
        return None


class HipTrainer:
    """One data-parallel training step per call on the HIP path (config 5)."""

    def __init__(self, points: PointParams, mlp_state, opts: HotPathOpts, device, lr=5e-4, plr=2e-3,
                 lr_decay_exp=0.1, lr_decay_iters=1_000_000, bucket_mb=64, querier=None, bpnet=None,
                 precision="f16"):
        """bpnet: the SG variant's BPNet point embedding [N, 96] (fp32, detached: it is an input,
        neural_points.py:662), needed when opts select block2_bpnet with predict_semantic = 1.
        precision "f16": the fp16-operand HIP forward + backward (k_agg_rows save mode, k_agg_bwd);
        "f32" (base viewmlp and SG): the reference's fp32 arithmetic -- the HIP fp32-faithful row
        kernel (k_rows16, 3 fp16 MFMA products per fp32 product) saves the row MLP's pre-activations
        and the backward runs through them on the same split-fp16 GEMMs (train_f32.F32Step)."""
        self.device = torch.device(device)
        self.opts = opts.check_supported()
        self.variant = tuple(opts.bpnet_variant)
        self.sg = self.variant != (0, 0)
        if precision not in ("f16", "f32"):
            raise ValueError("precision: 'f16' or 'f32'")
        self.precision = precision
        self.points = points
        self.mlp = FlatMLP(mlp_state, self.device, layers_for(*self.variant))
        self.bpnet16 = self.bpnet32 = None
        if self.variant[1]:
            if bpnet is None:
                raise ValueError("block2_bpnet with predict_semantic = 1 needs the BPNet point embedding")
            e = torch.as_tensor(bpnet).detach().to(self.device, torch.float32).reshape(-1, self.variant[1]).contiguous()
            self.bpnet16 = torch.empty(e.shape, dtype=torch.float16, device=self.device)
            _lib.check(_lib.lib().sgn_bpnet_pack(_lib.ptr(e), e.shape[0], e.shape[1], _lib.ptr(self.bpnet16),
                                                 _lib.stream_handle()), "sgn_bpnet_pack")
            if precision == "f32":   # the fp32 kernels read the embedding as it is
                self.bpnet32 = e
        self.point_params = [points.points_embeding, points.points_color, points.points_dir, points.points_conf]
        # the reference's two Adam groups (mvs_points_volumetric_model.py:100-108); fused: one
        # kernel per group for the dense 47 M-element point update instead of the foreach chain
        # kernel per group (sgn_adam_step, which also clears the gradient for the next step) instead
        # of the foreach chain; the MLP group's flat 0.35 M elements the same way
        fused = self.device.type == "cuda"
        if fused:
            self.opt_net = PointAdam([self.mlp.flat], lr=lr, betas=(0.9, 0.999))
            # row-sparse exact mode: a step updates the ~50 k rows it touches (each first replaying the
            # zero-gradient steps it missed) instead of streaming all 47 M elements; flushed before
            # anything else reads the points (sync_points)
            self.opt_pts = PointAdam(self.point_params, lr=plr, betas=(0.9, 0.999), rows=True)
        else:
            self.opt_net = torch.optim.Adam([self.mlp.flat], lr=lr, betas=(0.9, 0.999))
            self.opt_pts = torch.optim.Adam(self.point_params, lr=plr, betas=(0.9, 0.999))
        self._grads_clean = False  # the optimizers left every gradient zeroed
        self.base_lr = (lr, plr)
        self.decay = (lr_decay_exp, lr_decay_iters)
        self.step_count = 0
        self.bucket_elems = bucket_mb * (1 << 20) // 4
        self.querier = querier
        self.packer = _Packer(self.device, self.variant)
        # the fp32-faithful blob (f32 step) and, for both precisions, the per-layer weight shifts the
        # split-fp16 GEMMs of the colour MLP read
        self.packer32 = _PackerF32(self.device, self.mlp, self.variant)
        # stored column p -> reference index; inverses: reference index -> stored column
        self.map_chain = _colmap(0, 256, self.device)
        self.map_x0 = _colmap(1, 288, self.device)
        self.map_h2 = _colmap(2, 272, self.device)
        self.inv_chain = self._inverse(self.map_chain, 256)
        self.inv_x0 = self._inverse(self.map_x0, 284)
        self.inv_h2 = self._inverse(self.map_h2, 263)
        self._cap = 0
        # the f16 step's colour MLP, losses and their backward (train_f32.ColourStep on the HIP loss
        # stage) as one replayed HIP graph; use_graph = False runs the same stage eagerly (torch autograd
        # of the colour MLP into the HIP loss stage), the graph's parity reference in the tests
        self.use_graph = True
        self.loss_stage = LossStage(self.device)
        self._graphs = {}        # (capacity bucket, buffers) -> captured loss stage, LRU order
        self.graph_captures = 0
        self._flat_maps = {}

    @staticmethod
    def _inverse(m, n):
        inv = torch.full((n,), -1, dtype=torch.long, device=m.device)
        ok = m >= 0
        inv[m[ok]] = torch.nonzero(ok).reshape(-1)
        assert bool((inv >= 0).all())
        return inv

    # -- buffers -----------------------------------------------------------------------
    def _buffers(self, n_items, S_cap):
        dev = self.device
        if S_cap > getattr(self, "_scap", 0):
            self.feat = torch.zeros(S_cap, 4, dtype=torch.float32, device=dev)
            self._scap = S_cap
        if n_items > self._cap or not hasattr(self, "x0"):   # a first step without hits allocates too
            cap = max(128, ((n_items + 127) // 128) * 128)   # rows (8 per item) a multiple of 1024
            rows = cap * 8
            h = dict(dtype=torch.float16, device=dev)
            self.fs = torch.empty(cap, 256, **h)
            self.x0 = torch.empty(rows, 288, **h)
            self.h1 = torch.empty(rows, 256, **h)
            self.h2 = torch.empty(rows, 272, **h)
            self.h3 = torch.empty(rows, 256, **h)
            self.d = [torch.empty(rows, 256, **h) for _ in range(4)]  # d1..d4
            self.h4 = torch.empty(rows, 256, **h)
            if self.sg:  # block2_bpnet inputs h and deltas
                self.h2b = torch.empty(rows, 256, **h)
                self.db = torch.empty(rows, 256, **h)
            self.dza = torch.empty(rows, dtype=torch.float32, device=dev)
            self._cap = cap

    def _query(self, campos, raydir, near, far, labels=None):
        if self.querier is None:
            from .querier import LightningFastQuerier
            self.querier = LightningFastQuerier(self.device, self.opts)
        if self.opts.semantic_guidance:
            if labels is None:
                raise ValueError("semantic_guidance = 1: pass labels=(point_labels [N], ray_labels [R], seconds)")
            pl, rl, sec = labels
            return self.querier.query_samples(self.points.xyz, campos, raydir, near, far,
                                              torch.as_tensor(pl).to(self.device, torch.int32).reshape(-1).contiguous(),
                                              torch.as_tensor(rl).to(self.device, torch.int32).reshape(-1).contiguous(),
                                              sec)
        return self.querier.query_samples(self.points.xyz, campos, raydir, near, far)

    def _tables(self, campos, rot, raydir):
        pt = _lib.PointTables()
        P = self.points
        pt.xyz, pt.embedding, pt.color = P.xyz.data_ptr(), P.points_embeding.data_ptr(), P.points_color.data_ptr()
        pt.dir, pt.conf, pt.n_points = P.points_dir.data_ptr(), P.points_conf.data_ptr(), P.xyz.shape[0]
        pt.campos, pt.camrotc2w, pt.raydir = campos.data_ptr(), rot.data_ptr(), raydir.data_ptr()
        return pt

    _COLOUR = ("color_branch.0", "color_branch.2", "color_branch.4", "color_branch.6")

    def _colour(self, fs, v):
        """colour MLP (point_aggregators.py color_branch) on the flat parameter's weights (detached),
        the weight / bias gradients added straight into the flat gradient (_LinearInto)."""
        m = self.mlp
        g = m.flat.grad
        vpe = _pe(v, 4, ori=True)[..., 3:]
        c = torch.cat([fs, vpe], dim=-1)
        for name in self._COLOUR:
            dst = self._flat_maps.get(("colour", name))
            off, o, i = m.slices[name]
            if dst is None:
                dst = self._flat_maps[("colour", name)] = (off + torch.arange(o * i, device=self.device)).to(torch.int32)
            c = _LinearInto.apply(c, m.w(name).detach(), m.b(name).detach(), g, dst, off + o * i)
            if name != "color_branch.6":
                c = F.leaky_relu(c, 0.01)
        return torch.sigmoid(c) * (1 + 2 * 0.001) - 0.001

    def _loss_scale(self, dfs, dal):
        """2^-floor(log2(max |d|)) of the per-row deltas' inputs, on the device (sgn_pow2_scale)."""
        L = _lib.lib()
        if not hasattr(self, "_scale_ws"):
            self._scale_ws = torch.empty(int(L.sgn_pow2_scale_workspace_bytes()), dtype=torch.uint8, device=self.device)
        scale = torch.empty(1, dtype=torch.float32, device=self.device)
        _lib.check(L.sgn_pow2_scale(_lib.ptr(dfs), dfs.numel(), _lib.ptr(dal), dal.numel(), _lib.ptr(self._scale_ws),
                                    _lib.ptr(scale), _lib.stream_handle()), "sgn_pow2_scale")
        return scale

    def _touched(self, q, npts):
        """The step's touched points (sgn_touched_points: an int32 list in no particular order and
        its device count), for the single-GPU projection subset; no host sync, one launch."""
        dev = self.device
        if getattr(self, "_stamp_n", -1) != npts:
            self._stamp = torch.full((npts,), -1, dtype=torch.int32, device=dev)
            self._tlist = torch.empty(npts, dtype=torch.int32, device=dev)
            self._tcount = torch.zeros(3, dtype=torch.int64, device=dev)   # [2]: out-of-range ids met
            self._stamp_n, self._tstep = npts, 0
        step = self._tstep
        self._tstep = (step + 1) & 0x7fffffff
        if self._tstep == 0:   # the stamp table outlived 2^31 steps: start it again
            self._stamp_n = -1
        K = self.opts.K
        self._check_oob()
        _lib.check(_lib.lib().sgn_touched_points(_lib.ptr(q.pidx), _lib.ptr(q.counters), q.pidx.numel() // K, K, npts,
                                                 step, _lib.ptr(self._stamp), _lib.ptr(self._tlist),
                                                 _lib.ptr(self._tcount), _lib.stream_handle()), "sgn_touched_points")
        self._watch_oob(self._tcount[2:3])
        return self._tlist, self._tcount[step & 1]

    def _watch_oob(self, count):
        """The out-of-range neighbour count (a device int64) goes to pinned host memory without a sync;
        the next step (or check_touched()) reads it once the copy has landed and fails loudly on a
        query / point table mismatch (those points would never be projected or updated)."""
        self._check_oob()
        if not hasattr(self, "_oob_host"):
            self._oob_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self._oob_event = torch.cuda.Event()
        self._oob_host.copy_(count.reshape(1), non_blocking=True)
        self._oob_event.record()
        self._oob_pending = True

    def _check_oob(self, wait=False):
        """Raise if an earlier step's query named a point index >= n_points (sgn_touched_points'
        counter d_count2[2]); without wait only a copy that has already landed is read."""
        if not getattr(self, "_oob_pending", False):
            return
        if not wait and not self._oob_event.query():
            return
        self._oob_event.synchronize()
        self._oob_pending = False
        n = int(self._oob_host[0])
        if n:
            raise RuntimeError(f"training step: {n} neighbour indices >= n_points (query and point tables disagree)")

    def check_touched(self):
        """Wait for and check the last step's out-of-range neighbour counter (see _check_oob)."""
        self._check_oob(wait=True)

    # -- row-sparse point Adam --------------------------------------------------------------
    def _rows_adam(self):
        return isinstance(self.opt_pts, PointAdam) and self.opt_pts.rows_mode

    def _adam_rows(self, rows, count, count_is64, count_mul):
        """The step's point rows (a device list and count) to the row-sparse Adam: the deferred previous
        step applied and these rows brought to the current step before the forward reads them.  Returns
        the step's distinct rows (int32 list, int64 device count) or None (dense Adam); a list id >=
        n_points is reported at the next step (_watch_oob)."""
        if not self._rows_adam():
            return None
        pb = self.opt_pts.set_rows(rows, count, count_is64, count_mul)
        self._watch_oob(pb[8:16].view(torch.int64))
        return pb[16:].view(torch.int32), pb[:8].view(torch.int64)

    def _adam_union(self, all_idx):
        """Under DP the exchanged gradient covers every rank's rows: the update takes all of them."""
        if all_idx is not None and isinstance(self.opt_pts, PointAdam) and self.opt_pts.rows_mode:
            self.opt_pts.set_update_rows(all_idx.to(torch.int32))

    def sync_points(self):
        """Bring every point row to the optimizer's current step (the row-sparse Adam updates a row
        when a step touches it): call before reading the point tensors outside a step."""
        if isinstance(self.opt_pts, PointAdam):
            self.opt_pts.flush()

    # -- one step ------------------------------------------------------------------------
    def _bg_ray(self, bg_ray, R):
        """inputs['bg_ray'] (the plane background model's per-ray colour, [1, R, 3]) as a contiguous
        device [R, 3] fp32 tensor, or None (the constant white background)."""
        if bg_ray is None:
            return None
        bg_ray = torch.as_tensor(bg_ray).to(self.device, torch.float32).reshape(-1, 3).contiguous()
        if bg_ray.shape[0] != R:
            raise ValueError(f"bg_ray has {bg_ray.shape[0]} rays, the batch {R}")
        return bg_ray

    def backward(self, campos, rot, raydir, near, far, gt, labels=None, bg_ray=None):
        """Forward + backward + gradient all-reduce (no parameter update).  labels: (point_labels,
        ray_labels, seconds) for the semantic-guided query (semantic_guidance = 1).  bg_ray: the
        rays' background [1, R, 3] of the plane background model (inputs['bg_ray']): the composite
        and its gradient use T_bg * bg_ray per ray (neural_points_volumetric_model.py:175-177).
        Returns (loss parts, rendered colour [R,3], ray_mask [R])."""
        if self.precision == "f32":
            return self._backward_f32(campos, rot, raydir, near, far, gt, labels, bg_ray)
        o = self.opts
        dev = self.device
        campos = campos.reshape(3).to(dev, torch.float32).contiguous()
        rot = rot.reshape(3, 3).to(dev, torch.float32).contiguous()
        raydir = raydir.reshape(-1, 3).to(dev, torch.float32).contiguous()
        R = raydir.shape[0]
        bg_ray = self._bg_ray(bg_ray, R)
        q = self._query(campos, raydir, near, far, labels)
        dp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if not dp:   # the counts leave right after the query: the host waits for the query only
            if not hasattr(self, "_cnt_host"):
                self._cnt_host = torch.zeros(2, dtype=torch.int32, pin_memory=True)
                self._cnt_event = torch.cuda.Event()
            self._cnt_host.copy_(q.counters[:2], non_blocking=True)
            self._cnt_event.record()
        self._adam_rows(q.pidx, q.counters, False, o.K)
        # work that does not depend on the counts is queued before the step's one host sync, so the
        # GPU runs it while the host waits, and still has it queued when the host issues the rest
        blob, tblob = self.packer.pack(self.mlp.flat)
        for p in self.point_params + [self.mlp.flat]:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            elif not self._grads_clean:
                p.grad.zero_()
        self._grads_clean = False
        if dp:   # the point rows this rank's step can touch, and every rank's count, ride the same sync
            t_idx, t_cnt = touched_rows(q.pidx, q.counters[0], o.K, self.points.xyz.shape[0])
            sync = torch.cat([q.counters[:2].to(torch.int64), gather_counts(t_cnt)])
            S, n, *t_counts = (int(x) for x in sync.tolist())  # one host sync per step
        else:
            self._cnt_event.synchronize()   # one host sync per step, on the query's counts
            S, n = (int(x) for x in self._cnt_host.tolist())
        self._last_q = q
        graph = self.use_graph and dev.type == "cuda"
        if graph:
            self._buffers(R * o.SR, R * o.SR)   # static shapes: every buffer at the batch's capacity
        else:
            self._buffers(n, max(S, 1))
        L = _lib.lib()
        st = _lib.stream_handle()
        pt = self._tables(campos, rot, raydir)
        qo = q.abi()
        if graph:
            self.packer32.pack(self.mlp.flat)   # the colour GEMMs' weight shifts
            self.feat.zero_()                    # samples without neighbours keep zero features
        saved = _lib.AggSaved(self.x0.data_ptr(), self.h1.data_ptr(), self.h2.data_ptr(), self.h3.data_ptr())
        if n > 0 and self.sg:
            _lib.check(L.sgn_aggregate_train_fwd_sg(*self.variant, _lib.ptr(self.bpnet16), ctypes.byref(pt),
                                                    ctypes.byref(qo), n, o.K, _lib.ptr(blob), _lib.ptr(self.feat),
                                                    _lib.ptr(self.fs), ctypes.byref(saved), _lib.ptr(self.h2b), st),
                       "sgn_aggregate_train_fwd_sg")
        elif n > 0:
            _lib.check(L.sgn_aggregate_train_fwd(ctypes.byref(pt), ctypes.byref(qo), n, o.K, _lib.ptr(blob),
                                                 _lib.ptr(self.feat), _lib.ptr(self.fs), ctypes.byref(saved), st),
                       "sgn_aggregate_train_fwd")
        # ---- colour MLP + composite + losses (torch autograd, per sample / per ray) ----------
        if graph:
            out = self._graph_losses(q, campos, rot, raydir, gt, R, S, n, bg_ray)
            total, parts, full, ray_mask = out["total"], dict(out["parts"]), out["full"], out["ray_mask"]
            dfs, dal, scale = out["dfs"], out["dal"], out["scale"]
        else:
            samp = q.work[:n]   # int32 indices throughout (no widening copies)
            fs_t = self.fs[:n].float().requires_grad_(True)
            alpha_t = self.feat[samp, 0].clone().requires_grad_(True)
            v = raydir[q.samp_ray[samp]]
            feat_s = torch.cat([alpha_t[:, None], self._colour(fs_t, v)], dim=-1)
            featS = torch.zeros(S, 4, device=dev).index_put((samp,), feat_s)
            validS = torch.zeros(S, dtype=torch.bool, device=dev)
            validS[samp] = True
            qd = {"ray_ns": q.ray_ns[:R], "ray_soff": q.ray_soff[:R], "samp_ray": q.samp_ray[:S],
                  "samp_locw": q.samp_locw[:S * 3].view(S, 3), "pidx": q.pidx[:S * o.K].view(S, o.K)}
            total, parts, full, ray_mask = self.loss_stage(self.points, qo, featS, campos, rot, gt, o, R, bg_ray=bg_ray)
            total.backward()
            if n > 0:
                dfs = fs_t.grad.contiguous()
                dal = alpha_t.grad.contiguous()
                scale = self._loss_scale(dfs, dal)
        # ---- HIP backward of the per-row part -----------------------------------------------
        if n > 0:
            deltas = _lib.AggDeltas(self.d[3].data_ptr(), self.d[2].data_ptr(), self.d[1].data_ptr(),
                                    self.d[0].data_ptr(), self.h4.data_ptr(), self.dza.data_ptr())
            P = self.points
            grads = _lib.PointGrads(P.points_embeding.grad.data_ptr(), P.points_color.grad.data_ptr(),
                                    P.points_dir.grad.data_ptr(), P.points_conf.grad.data_ptr())
            if self.sg:
                _lib.check(L.sgn_aggregate_backward_sg(*self.variant, ctypes.byref(pt), ctypes.byref(qo), n, o.K,
                                                       _lib.ptr(blob), _lib.ptr(tblob), ctypes.byref(saved),
                                                       _lib.ptr(self.h2b), _lib.ptr(dfs), _lib.ptr(dal),
                                                       _lib.ptr(scale), ctypes.byref(deltas), _lib.ptr(self.db),
                                                       ctypes.byref(grads), st), "sgn_aggregate_backward_sg")
            else:
                _lib.check(L.sgn_aggregate_backward(ctypes.byref(pt), ctypes.byref(qo), n, o.K, _lib.ptr(blob),
                                                    _lib.ptr(tblob), ctypes.byref(saved), _lib.ptr(dfs), _lib.ptr(dal),
                                                    _lib.ptr(scale), ctypes.byref(deltas), ctypes.byref(grads), st),
                           "sgn_aggregate_backward")
            self._weight_grads(n * 8, scale, q)
        self.allreduce_grads([self.mlp.flat])
        if dp:
            self._adam_union(_allreduce_point_rows([p.grad for p in self.point_params], t_idx, t_counts))
        parts["total"] = total.detach()
        return parts, full.detach(), ray_mask

    # -- fp32-faithful step ---------------------------------------------------------------------
    def _loss_params(self, bg_ray=None):
        o = self.opts
        lp = _lib.LossParams()
        lp.SR, lp.K = o.SR, o.K
        lp.vsize_z, lp.raydist_mode_unit = float(o.vsize[2]), int(o.raydist_mode_unit)
        for i in range(3):
            lp.bg[i] = 1.0
        lp.zero_one_weight, lp.zero_one_eps = 1e-4, 1e-3   # train_ft: zero_one weight 1e-4, epsilon 1e-3
        if bg_ray is not None:   # per-ray background [R, 3] (device, contiguous)
            lp.bg_ray = bg_ray.data_ptr()
        return lp

    def _backward_f32(self, campos, rot, raydir, near, far, gt, labels=None, bg_ray=None):
        """The reference's fp32 step on hand-written kernels (train_f32.F32Step): query, forward,
        colour MLP, losses and the whole backward as HIP launches with the counts on the device (no
        host sync on one GPU; under DP one for the touched-row counts).  The block1.0 projection P is
        recomputed for the points the step's rays touch only (~50 k of 1.2 M for a 4096-ray batch: the
        rows read no other point, and the weights change every step)."""
        from .train_f32 import F32Step
        o = self.opts
        dev = self.device
        campos = campos.reshape(3).to(dev, torch.float32).contiguous()
        rot = rot.reshape(3, 3).to(dev, torch.float32).contiguous()
        raydir = raydir.reshape(-1, 3).to(dev, torch.float32).contiguous()
        gt = gt.reshape(-1, 3).to(dev, torch.float32).contiguous()
        R = raydir.shape[0]
        bg_ray = self._bg_ray(bg_ray, R)
        q = self._query(campos, raydir, near, far, labels)
        blob = self.packer32.pack(self.mlp.flat)
        for p in self.point_params + [self.mlp.flat]:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            elif not self._grads_clean:
                p.grad.zero_()
        self._grads_clean = False
        L = _lib.lib()
        st = _lib.stream_handle()
        pt = self._tables(campos, rot, raydir)
        P = self.points
        npts = P.xyz.shape[0]
        nproj = int(L.sgn_point_proj_bytes_f32(npts))
        if getattr(self, "_proj32", None) is None or self._proj32.numel() < nproj:
            self._proj32 = torch.empty(max(nproj, 16), dtype=torch.uint8, device=dev)
        dp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        t_idx = t_cnt = None
        if dp:
            t_idx, t_cnt = touched_rows(q.pidx, q.counters[0], o.K, npts)
        if dp:   # every rank's touched rows ride the step's one sync (the point-row exchange)
            idx32, cnt = t_idx.to(torch.int32), t_cnt
            self._adam_rows(idx32, cnt, True, 1)
        else:    # the Adam's distinct-row list is the step's touched list (row 0 included)
            lst = self._adam_rows(q.pidx, q.counters, False, o.K)
            idx32, cnt = lst if lst is not None else self._touched(q, npts)
        _lib.check(L.sgn_point_project_f32_subset(ctypes.byref(pt), _lib.ptr(blob), _lib.ptr(idx32),
                                                  _lib.ptr(cnt), _lib.ptr(self._proj32), st),
                   "sgn_point_project_f32_subset")
        step = getattr(self, "_f32step", None)
        key = (R, q.work.data_ptr(), q.pidx.data_ptr(), self.mlp.flat.data_ptr(), self.mlp.flat.grad.data_ptr())
        if step is None or step.key != key:
            step = self._f32step = F32Step(self, q, R)
            step.key = key
        losses, full, mask = step.run(pt, self._proj32, blob, campos, rot, gt, self._loss_params(bg_ray))
        self._last_q = q
        # the step's buffers are reused by the next step: the losses, the colour and the mask out into
        # one fresh allocation (one launch), as the f16 step's graph outputs
        nl = losses.numel()
        buf = torch.empty(nl + 3 * R + -(-R // 4), dtype=torch.float32, device=dev)
        lo, full_o = buf[:nl], buf[nl:nl + 3 * R].view(R, 3)
        mask_o = buf[nl + 3 * R:].view(torch.int8)[:R]
        _lib.copy_segments([(losses, lo), (full, full_o), (mask, mask_o)])
        total = lo[0] + 3e-6 + 1e-4 * lo[1]
        parts = {"ray_masked_coarse_raycolor": lo[0], "ray_miss_coarse_raycolor": lo[2],
                 "coarse_raycolor": lo[3], "conf_coefficient": lo[1]}
        self.allreduce_grads([self.mlp.flat])
        if dp:
            t_counts = [int(x) for x in gather_counts(t_cnt).tolist()]
            self._adam_union(_allreduce_point_rows([p.grad for p in self.point_params], t_idx, t_counts))
        parts["total"] = total
        return parts, full_o, mask_o.bool()

    @property
    def last_query(self):
        """The last fp32 step's sample-major query as a dict (ray_ns, ray_soff, samp_ray, samp_locw,
        pidx): tests rerun fp32 autograd on the very samples the step used.  Reads S (host sync)."""
        q, o = self._last_q, self.opts
        R, S = q.R, int(q.counters[0].item())
        return {"ray_ns": q.ray_ns[:R], "ray_soff": q.ray_soff[:R], "samp_ray": q.samp_ray[:S],
                "samp_locw": q.samp_locw[:S * 3].view(S, 3), "pidx": q.pidx[:S * o.K].view(S, o.K)}

    # -- graph-captured loss stage -----------------------------------------------------------
    def _loss_body(self, st):
        """Colour MLP + composite + losses + their backward on the hand-written kernels over the batch's
        full sample capacity (R * SR entries, static shapes, no host sync): items past the device count
        n and samples past S are padding, zeroed on input and routed to sentinel rows, so the gradients
        equal the eager path's.  Runs inside a HIP graph capture (and its warm-up)."""
        o, dev, R = self.opts, self.device, st["R"]
        Sc, Nc = st["Sc"], st["Nc"]             # sample / item capacity of this graph
        q = st["q"]
        fs32, al32, v, samp = st["fs32"], st["al32"], st["v"], st["samp"]
        # one launch: items past the device count n are padding (zeros, ray 0, sentinel sample Sc)
        _lib.check(_lib.lib().sgn_colour_inputs(_lib.ptr(q.counters), _lib.ptr(q.work), _lib.ptr(q.samp_ray), Nc, Sc,
                                                _lib.ptr(self.fs), _lib.ptr(self.feat), _lib.ptr(st["raydir"]),
                                                _lib.ptr(fs32), _lib.ptr(al32), _lib.ptr(v), _lib.ptr(samp),
                                                _lib.ptr(st["col"].vpe),
                                                _lib.stream_handle()), "sgn_colour_inputs")
        # hand-written colour MLP, losses and backward (train_f32.ColourStep)
        losses, full, mask, dfs, dfeat = st["col"].run(st["campos"], st["rot"], st["gt"], self._loss_params(st["bg_ray"]))
        dal = dfeat[samp.long(), 0]          # per item (padding: the zero row Sc)
        scale = self._loss_scale(dfs, dal)
        total = losses[0] + 3e-6 + 1e-4 * losses[1]
        names = ["ray_masked_coarse_raycolor", "ray_miss_coarse_raycolor", "coarse_raycolor", "conf_coefficient"]
        return {"scalars": torch.stack([total, losses[0], losses[2], losses[3], losses[1]]), "names": names,
                "full": full, "ray_mask": mask, "dfs": dfs, "dal": dal, "scale": scale}

    def _graph_losses(self, q, campos, rot, raydir, gt, R, S, n, bg_ray=None):
        """Replay the captured loss stage for this step's capacity bucket (item / sample counts
        rounded up to GRAPH_BUCKET); captured on first use and again when a buffer it reads
        moved.  At most GRAPH_CACHE graphs are kept.  A step with a per-ray background (bg_ray)
        replays a graph of its own whose static bg_ray buffer the step's colours are copied into."""
        dev = self.device
        P, fl = self.points, self.mlp.flat
        cap = R * self.opts.SR
        Sc = min(cap, -(-max(S, 1) // GRAPH_BUCKET) * GRAPH_BUCKET)
        Nc = min(Sc, -(-max(n, 1) // GRAPH_BUCKET) * GRAPH_BUCKET)
        key = (R, Sc, Nc, q.work.data_ptr(), q.counters.data_ptr(), self.fs.data_ptr(), self.feat.data_ptr(),
               fl.data_ptr(), fl.grad.data_ptr(), P.points_conf.data_ptr(), P.points_conf.grad.data_ptr(),
               bg_ray is not None)
        st = self._graphs.pop(key, None)
        if st is not None:
            self._graphs[key] = st              # most recently used goes last (LRU eviction order)
        else:
            self.graph_captures += 1
            if len(self._graphs) >= GRAPH_CACHE:
                self._graphs.pop(next(iter(self._graphs)))
            st = {"key": key, "R": R, "Sc": Sc, "Nc": Nc, "q": q, "qabi": q.abi(),
                  "raydir": raydir.clone(), "gt": gt.reshape(-1, 3).to(dev, torch.float32).clone(),
                  "campos": campos.clone(), "rot": rot.clone(),
                  "bg_ray": None if bg_ray is None else bg_ray.clone(),
                  "fs32": torch.zeros(Nc, 256, device=dev), "al32": torch.zeros(Nc, device=dev),
                  "v": torch.zeros(Nc, 3, device=dev), "samp": torch.zeros(Nc, dtype=torch.int32, device=dev)}
            from .train_f32 import ColourStep
            st["col"] = ColourStep(self, q, Nc, st["fs32"], st["v"], self.feat, R)
            keep = [fl.grad.clone(), P.points_conf.grad.clone()]   # warm-up accumulates into them
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self._loss_body(st)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            # a garbage collection inside the capture would destroy dead objects that hold HIP resources (an
            # earlier trainer's graphs, streams, events), which invalidates a global-mode capture: keep the
            # collector off until the capture ends (no gc.collect() first: a full collection costs tens of ms
            # per capture, +0.3..0.9 ms per step over a 100-step run with one capture in it)
            gc_on = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g):
                    st["out"] = self._loss_body(st)
            finally:
                if gc_on:
                    gc.enable()
            fl.grad.copy_(keep[0])
            P.points_conf.grad.copy_(keep[1])
            st["graph"] = g
            self._graphs[key] = st
        g3 = gt.reshape(-1, 3)
        if g3.dtype != torch.float32 or g3.device != dev or not g3.is_contiguous():
            g3 = g3.to(dev, torch.float32).contiguous()
        # the step's inputs into the graph's static buffers: one launch
        _lib.copy_segments([(raydir, st["raydir"]), (g3, st["gt"]), (campos, st["campos"]), (rot, st["rot"])] +
                           ([] if bg_ray is None else [(bg_ray, st["bg_ray"])]))
        st["graph"].replay()
        out = st["out"]
        # the loss, its parts, the rendered colour and the ray mask out of the graph's buffers: one
        # launch into one fresh allocation (the caller may keep them across steps)
        nsc = out["scalars"].numel()
        o_full = 8 * (-(-nsc // 8))
        buf = torch.empty(o_full + 3 * R + -(-R // 4), dtype=torch.float32, device=dev)
        sc, full = buf[:nsc], buf[o_full:o_full + 3 * R].view(R, 3)
        ray_mask = buf[o_full + 3 * R:].view(torch.bool)[:R]
        _lib.copy_segments([(out["scalars"], sc), (out["full"], full), (out["ray_mask"], ray_mask)])
        return {"total": sc[0], "parts": {k: sc[1 + i] for i, k in enumerate(out["names"])},
                "full": full, "ray_mask": ray_mask,
                "dfs": out["dfs"], "dal": out["dal"], "scale": out["scale"]}

    def _dst_maps(self, name, x_cols, ix):
        """int32 maps from the MFMA storage order to the flat parameter for layer `name`: weight
        [256 stored units][x_cols stored columns] (-1: padding column) and bias [256 stored]."""
        maps = self._flat_maps.get(name)
        if maps is None:
            m, iu = self.mlp, self.inv_chain
            off, o, i = m.slices[name]
            fi = (iu[:, None] * x_cols + ix[None, :]).reshape(-1)   # stored index of each reference weight
            dw = torch.full((o * x_cols,), -1, dtype=torch.int32, device=self.device)
            dw[fi] = (off + torch.arange(o * i, device=self.device)).to(torch.int32)
            db = torch.full((o,), -1, dtype=torch.int32, device=self.device)
            db[iu] = (off + o * i + torch.arange(o, device=self.device)).to(torch.int32)
            maps = self._flat_maps[name] = (dw, db)
        return maps

    def _dw_parts(self, name, d, x, rows):
        """dW = d^T x and db = sum_r d[r] over the first `rows` rows (fp16 operands, fp32 accumulation) as
        split-K partials ([splits, 256, C], [splits, 256]) from sgn_f16_weight_grad (rows past `rows` are
        never read).  One pair of buffers per layer: the step's single sgn_grad_accumulate reads them all."""
        C = x.shape[1]
        bufs = self._dw_bufs.get(name)
        if bufs is None or bufs[0].shape[2] != C:
            splits = max(1, 256 // -(-C // 128))   # about one workgroup per CU
            bufs = self._dw_bufs[name] = (torch.empty(splits, 256, C, dtype=torch.float32, device=self.device),
                                          torch.empty(splits, 256, dtype=torch.float32, device=self.device))
        parts, pb = bufs
        _lib.check(_lib.lib().sgn_f16_weight_grad(_lib.ptr(d), d.stride(0), _lib.ptr(x), x.stride(0), C, rows,
                                                  parts.shape[0], _lib.ptr(parts), _lib.ptr(pb), _lib.stream_handle()),
                   "sgn_f16_weight_grad")
        return parts, pb

    def _weight_grads(self, rows, scale, q=None):
        """dW_l = delta_l^T x_l (sgn_f16_weight_grad: fp16 operands, fp32 split-K partials), db_l = sum
        delta_l; the partials summed, unscaled and unpermuted into the flat gradient by one
        sgn_grad_accumulate launch."""
        m = self.mlp
        g = m.flat.grad
        L = _lib.lib()
        st = _lib.stream_handle()
        rp = ((rows + 1023) // 1024) * 1024   # rows padded (the SG embedding gather's view)
        if not hasattr(self, "_dw_bufs"):
            self._dw_bufs = {}
        # the alpha branch's dWa = dza^T h4 and dba = sum dza as row-slab partials (one launch; the final sums
        # happen in the step's sgn_grad_accumulate); the row layers' bias gradients come with their weight
        # gradients (sgn_f16_weight_grad's column sums)
        if not hasattr(self, "_cs_ws"):
            self._cs_ws = torch.empty(int(L.sgn_colsum_workspace_bytes(1)) // 4, dtype=torch.float32,
                                      device=self.device)
        _lib.check(L.sgn_colsum_f16_weighted_parts(1, (ctypes.c_void_p * 1)(self.h4.data_ptr()),
                                                   (ctypes.c_void_p * 1)(self.dza.data_ptr()), rows, 256,
                                                   _lib.ptr(self._cs_ws), st), "sgn_colsum_f16_weighted_parts")
        ns = _lib.COLSUM_SLABS
        segs, keep = [], []

        def add(src, tail, dst):
            keep.append((src, tail))
            n = dst.numel()
            segs.append(_lib.GradSegment(src.data_ptr(), tail.data_ptr() if tail is not None else None,
                                         dst.data_ptr(), n, n, src.numel() // n, 0))
        if self.sg:
            # block2_bpnet.0: x = [h (chain order) | the row's BPNet embedding (natural order)]
            x = self.h2b[:rp]
            if self.variant[1]:
                # row r = item * 8 + k: rows k < K read pidx index s * K + k, rows k >= K are empty
                K = self.opts.K
                r = torch.arange(rp, device=self.device)
                item, k = r // 8, r % 8
                ok = (item < rows // 8) & (k < K)
                s_of = q.work[torch.where(ok, item, 0)].long()
                pid = torch.where(ok, q.pidx[s_of * K + torch.clamp(k, max=K - 1)].long(), -1)
                bp = self.bpnet16[torch.clamp(pid, min=0)]
                bp = torch.where((ok & (pid >= 0))[:, None], bp, torch.zeros((), dtype=bp.dtype, device=bp.device))
                x = torch.cat([x, bp], dim=1)
            ix = torch.cat([self.inv_chain, 256 + torch.arange(self.variant[1], device=self.device)])
            dw, db = self._dst_maps(BPNET, x.shape[1], ix)
            parts, pb = self._dw_parts(BPNET, self.db, x, rows)
            add(parts, None, dw)
            add(pb, None, db)
        for li, (name, d, x, ix) in enumerate((("block3.2", self.d[3], self.h3, self.inv_chain),
                                               ("block3.0", self.d[2], self.h2, self.inv_h2),
                                               ("block1.2", self.d[1], self.h1, self.inv_chain),
                                               ("block1.0", self.d[0], self.x0, self.inv_x0))):
            dw, db = self._dst_maps(name, x.shape[1], ix)
            parts, pb = self._dw_parts(name, d, x, rows)
            add(parts, None, dw)    # [256 stored][C stored]
            add(pb, None, db)
        # alpha branch: dWa = dza^T h4, dba = sum dza
        amaps = self._flat_maps.get("alpha_branch.0")
        if amaps is None:
            off, o, i = m.slices["alpha_branch.0"]
            dwa = torch.empty(256, dtype=torch.int32, device=self.device)
            dwa[self.inv_chain] = (off + torch.arange(256, device=self.device)).to(torch.int32)
            amaps = self._flat_maps["alpha_branch.0"] = (dwa, torch.full((1,), off + i, dtype=torch.int32,
                                                                        device=self.device))
        add(self._cs_ws[:ns * 256], None, amaps[0])         # [slabs][256] -> 256
        add(self._cs_ws[ns * 256:ns * 257], None, amaps[1])  # [slabs] -> 1
        _lib.check(L.sgn_grad_accumulate(len(segs), (_lib.GradSegment * len(segs))(*segs), _lib.ptr(scale),
                                         _lib.ptr(g), st), "sgn_grad_accumulate")

    def allreduce_grads(self, params):
        _allreduce_buckets([p.grad for p in params if p.grad is not None], self.bucket_elems)

    def _set_lr(self):
        exp, iters = self.decay
        f = exp ** (self.step_count / iters)  # iter_exponential_decay
        for opt, base in ((self.opt_net, self.base_lr[0]), (self.opt_pts, self.base_lr[1])):
            for gr in opt.param_groups:
                gr["lr"] = base * f

    def apply(self):
        self._set_lr()
        self.opt_net.step()
        self.opt_pts.step()
        self._grads_clean = all(isinstance(o, PointAdam) and o.zero_grad_in_step for o in (self.opt_net, self.opt_pts))
        self.step_count += 1

    def step(self, campos, rot, raydir, near, far, gt, labels=None, bg_ray=None):
        out = self.backward(campos, rot, raydir, near, far, gt, labels, bg_ray)
        self.apply()
        return out

    def mlp_state(self):
        return self.mlp.state()


def grads_named(trainer: HipTrainer):
    """Gradients under the reference names (for parity tests): MLP layers + point params."""
    m = trainer.mlp
    g = m.flat.grad
    out = {}
    for name, *_ in m.layers:
        out[name + ".weight"] = m.w(name, g).detach().clone()
        out[name + ".bias"] = m.b(name, g).detach().clone()
    P = trainer.points
    for k in ("points_embeding", "points_color", "points_dir", "points_conf"):
        out[k] = getattr(P, k).grad.detach().clone()
    return out
