"""Fused frame renderer: query -> MFMA aggregator -> composite, all on one stream,
no host synchronisation and no [R, SR, K, C] intermediates.

This is the product path behind NeuralPointsRayMarching.forward (ray_marching.py)
and bench.py.  Buffers are sized once per (R, SR) and reused.
"""
import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from .opts import HotPathOpts
from .querier import LightningFastQuerier
from .weights import mlp_variant, pack_mlp, strip_prefix


@dataclass
class RenderOut:
    rgb: torch.Tensor        # [R,3] fill_invalid'ed colour (bg for invalid rays)
    ray_mask: torch.Tensor   # [R] int8, reference ray_mask after masked_valid_ray
    bg_transmission: torch.Tensor  # [R] coarse_is_background (1 for invalid rays)
    opacity: torch.Tensor    # [R,SR] coarse_point_opacity (0 for invalid rays / empty slots)
    query: object            # QueryResult (sample-major, device)
    feat: torch.Tensor       # [S_cap,4] per-sample (alpha, r, g, b)
    blend: torch.Tensor      # [S_cap,8] weight * conf_coefficient (when want_blend)
    wnorm: torch.Tensor = None    # [S_cap,8] normalised weight (when want_weights)
    blendw: torch.Tensor = None   # [R,SR] alpha-blend weight o*T (when want_weights)


class PointTables:
    """Device-resident neural point cloud (contiguous fp32 tables)."""

    def __init__(self, xyz, embedding, color, dir, conf, device, bpnet=None):
        def t(x, cols):
            x = torch.as_tensor(x).reshape(-1, cols)
            return x.to(device=device, dtype=torch.float32).contiguous()
        self.xyz = t(xyz, 3)
        self.embedding = t(embedding, 32)
        self.color = t(color, 3)
        self.dir = t(dir, 3)
        self.conf = t(conf, 1)
        self.n = self.xyz.shape[0]
        self.bpnet16 = None
        self.bpnet32 = None
        if bpnet is not None:
            self.set_bpnet(bpnet)

    def set_bpnet(self, bpnet):
        """SG: bpnet_points_embedding [N, 96] (neural_points.py:653-665, detached there too)
        -> the fp16 table the aggregator gathers (sgn_bpnet_pack)."""
        b = torch.as_tensor(bpnet).reshape(-1, 96).to(device=self.xyz.device, dtype=torch.float32).contiguous()
        if b.shape[0] != self.n:
            raise ValueError(f"bpnet embedding has {b.shape[0]} rows for {self.n} points")
        self.bpnet32 = b  # fp32 table of the fp32-faithful aggregator
        self.bpnet16 = torch.empty(self.n, 96, dtype=torch.float16, device=self.xyz.device)
        with torch.cuda.device(self.xyz.device):
            _lib.check(_lib.lib().sgn_bpnet_pack(_lib.ptr(b), self.n, 96, _lib.ptr(self.bpnet16),
                                                 _lib.stream_handle()), "sgn_bpnet_pack")

    @classmethod
    def from_cloud(cls, pc, device):
        return cls(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, device, getattr(pc, "bpnet", None))


class HipRenderer:
    def __init__(self, points: PointTables, mlp_state, opts: HotPathOpts, device):
        self.device = torch.device(device)
        self.opts = opts.check_supported()
        self.points = points
        self.querier = LightningFastQuerier(self.device, opts)
        self.set_mlp(mlp_state)
        self._cap = None
        self._proj = None
        self._fp = None        # sgn_frame_points buffers (marks, list, counts) for the projection subset
        self._pending = []   # deferred fp16-range checks: (pinned flag copy, event)
        self._flag_host = None

    def set_mlp(self, mlp_state):
        self.mlp_state = {k: torch.as_tensor(v).detach().to("cpu", torch.float32)
                          for k, v in strip_prefix(mlp_state).items()}
        self.variant = mlp_variant(self.mlp_state)
        if self.variant != self.opts.bpnet_variant:
            raise ValueError(f"aggregator weights are block2_bpnet variant {self.variant}, options say "
                             f"{self.opts.bpnet_variant} (shading_feature_mlp_layer2_bpnet / predict_semantic)")
        self.f32 = self.opts.precision == "f32"
        self.packed = pack_mlp(self.mlp_state, self.device, self.opts.precision)
        # f32 mode's range fallback: plain fp32 weights for sgn_aggregate_exact, packed on first use; `exact`
        # turns on (for these weights) once a frame's activations left fp16 range
        self.packed_exact = None
        self.exact = False

    def _buffers(self, R):
        SR = self.opts.SR
        if self._cap is None or self._cap[0] < R:
            cap = max(R * SR, 1)
            dev = self.device
            self.feat = torch.empty(cap, 4, dtype=torch.float32, device=dev)
            self.blend = torch.empty(cap, self.opts.K, dtype=torch.float32, device=dev)
            L = _lib.lib()
            nb = int(L.sgn_aggregate_workspace_bytes_f32(cap) if self.f32 else L.sgn_aggregate_workspace_bytes(cap))
            self.agg_ws = torch.empty(nb, dtype=torch.uint8, device=dev)
            self.rgb = torch.empty(max(R, 1), 3, dtype=torch.float32, device=dev)
            self.mask = torch.empty(max(R, 1), dtype=torch.int8, device=dev)
            self.bgT = torch.empty(max(R, 1), dtype=torch.float32, device=dev)
            self.opacity = torch.empty(max(R, 1), SR, dtype=torch.float32, device=dev)
            self.wnorm = None
            self.blendw = None
            self._cap = (R, cap)

    def _flag(self):
        off = int(_lib.lib().sgn_aggregate_flag_offset_f32(self.agg_ws.numel()))
        return self.agg_ws[off:off + 4].view(torch.int32)

    def _range_check(self, mode, redo):
        """f32 mode: the colour stage flags samples whose decoded features are not finite (an
        activation outside fp16 range, mlp_x3.hip header).  "sync": check now (one stream sync) and,
        when flagged, re-run the frame's aggregation and composite on the plain-fp32 path (`redo`,
        sgn_aggregate_exact), which later frames then take directly; "deferred": copy the flag to
        pinned memory and check it after the NEXT frame has been enqueued (or at finish()), so frames
        stay pipelined -- a flagged frame raises there (its output was handed out already) and switches
        the renderer to the plain-fp32 path; False: no check."""
        if not self.f32 or not mode or self.exact:
            return
        if mode == "sync":
            flag = self._flag()
            if int(flag.item()) != 0:
                self.exact = True
                flag.zero_()
                redo()
            return
        if self._flag_host is None:
            self._flag_host = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(2)]
        prev = self._pending.pop(0) if self._pending else None   # at most one frame is pending
        buf = self._flag_host[1] if prev is not None and prev[0] is self._flag_host[0] else self._flag_host[0]
        buf.copy_(self._flag(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending.append((buf, ev))
        if prev is not None:
            self._raise_if_flagged(*prev)

    def _raise_if_flagged(self, buf, ev):
        ev.synchronize()
        if int(buf.item()) != 0:
            self.exact = True   # every later frame on the plain-fp32 path
            self._flag().zero_()
            raise _lib.SgnError("sgn_aggregate_f32: fp16 range exceeded -- an aggregator activation or point "
                                "feature reached |x| >= 65504, so the decoded features of a frame rendered with "
                                "check_range='deferred' are not finite; the renderer now uses the plain-fp32 path "
                                "(sgn_aggregate_exact): render that frame again")

    def finish(self):
        """Wait for the deferred range checks of the frames rendered so far (raises if one failed)."""
        while self._pending:
            self._raise_if_flagged(*self._pending.pop(0))

    def render(self, campos, camrotc2w, raydir, near, far, want_opacity=True, want_blend=False, marks=None,
               bg=None, want_weights=False, point_labels=None, ray_labels=None, seconds=None,
               count_traffic=False, check_range="sync"):
        """One frame.  `marks(name)` (optional) is called between stages on the host thread
        (bench.py records HIP events on the current stream there).  `bg`: 3 floats
        overriding opts.bg_color.  `want_weights`: also produce the normalised neighbour
        weights and the per-slot alpha-blend weights (reference `weight`, `blend_weight`).
        `point_labels` [N] / `ray_labels` [R] int32 (+ `seconds`): the SG semantic-guided kNN
        (semantic_guidance = 1, worldcoords.py:839-938).  `check_range`: the f32 mode's fp16-range
        guard ("sync" default: a frame whose activations leave fp16 range is re-rendered on the
        plain-fp32 path, sgn_aggregate_exact; "deferred" for pipelined frame loops + finish(), False)."""
        o = self.opts
        mark = marks or (lambda name: None)
        campos = campos.reshape(3).to(self.device, torch.float32).contiguous()
        rot = camrotc2w.reshape(3, 3).to(self.device, torch.float32).contiguous()
        raydir = raydir.reshape(-1, 3).to(self.device, torch.float32).contiguous()
        R = raydir.shape[0]
        self._buffers(R)
        if want_weights and self.wnorm is None:
            self.wnorm = torch.empty(self._cap[1], o.K, dtype=torch.float32, device=self.device)
            self.blendw = torch.empty(max(self._cap[0], 1), o.SR, dtype=torch.float32, device=self.device)
        if want_weights:
            self.wnorm.zero_()
        mark("query")
        if o.semantic_guidance == 1 and (point_labels is None or ray_labels is None):
            raise ValueError("semantic_guidance = 1 needs point_labels and ray_labels")
        q = self.querier.query_samples(self.points.xyz, campos, raydir, near, far, point_labels, ray_labels, seconds,
                                       count_traffic)
        L = _lib.lib()
        st = _lib.stream_handle()
        pt = _lib.PointTables()
        pt.xyz, pt.embedding, pt.color = self.points.xyz.data_ptr(), self.points.embedding.data_ptr(), self.points.color.data_ptr()
        pt.dir, pt.conf, pt.n_points = self.points.dir.data_ptr(), self.points.conf.data_ptr(), self.points.n
        pt.campos, pt.camrotc2w, pt.raydir = campos.data_ptr(), rot.data_ptr(), raydir.data_ptr()
        qo = q.abi()
        cap = R * o.SR
        nl, dim = self.variant
        if dim and self.points.bpnet16 is None:
            raise ValueError("block2_bpnet with predict_semantic = 1 needs the points' BPNet embedding (set_bpnet)")
        bp = (_lib.ptr(self.points.bpnet32) if self.f32 else _lib.ptr(self.points.bpnet16)) if dim else None
        def aggregate_exact():
            # the f32 mode's range fallback: the whole aggregator and colour MLP in plain fp32
            if self.packed_exact is None:
                self.packed_exact = pack_mlp(self.mlp_state, self.device, "exact")
            _lib.check(L.sgn_aggregate_exact(nl, dim, bp, ctypes.byref(pt), ctypes.byref(qo), cap, o.K,
                                             _lib.ptr(self.packed_exact), _lib.ptr(self.feat),
                                             _lib.ptr(self.blend) if want_blend else None,
                                             _lib.ptr(self.wnorm) if want_weights else None, _lib.ptr(self.agg_ws),
                                             self.agg_ws.numel(), _lib.stream_handle()), "sgn_aggregate_exact")

        # split block1.0: P[point] = W0a [feat | PE(feat)] + b0, once per frame, for the points the
        # frame's samples name only (sgn_frame_points: ~19 % of a config-2 frame's)
        mark("proj")
        nproj = int(L.sgn_point_proj_bytes_f32(self.points.n) if self.f32 else L.sgn_point_proj_bytes(self.points.n))
        if self._proj is None or self._proj.numel() < nproj:
            self._proj = torch.empty(max(nproj, 16), dtype=torch.uint8, device=self.device)
        if not self.exact:
            n = self.points.n
            if self._fp is None or self._fp[0] != n:
                self._fp = (n, torch.zeros(int(L.sgn_frame_points_mark_bytes(n)), dtype=torch.uint8, device=self.device),
                            torch.empty(n, dtype=torch.int32, device=self.device),
                            torch.zeros(2, dtype=torch.int64, device=self.device))
            _, marks, plist, pcount = self._fp
            _lib.check(L.sgn_frame_points(_lib.ptr(q.pidx), _lib.ptr(q.counters), q.pidx.numel() // o.K, o.K, n,
                                          _lib.ptr(marks), _lib.ptr(plist), _lib.ptr(pcount), st), "sgn_frame_points")
            project = L.sgn_point_project_f32_subset if self.f32 else L.sgn_point_project_subset
            _lib.check(project(ctypes.byref(pt), _lib.ptr(self.packed), _lib.ptr(plist), _lib.ptr(pcount),
                               _lib.ptr(self._proj), st), "point projection (subset)")
        for stage, name in ((1, "agg_rows"), (2, "agg_color")):
            mark(name)
            blend = _lib.ptr(self.blend) if want_blend else None
            wnorm = _lib.ptr(self.wnorm) if want_weights and stage == 1 else None
            if self.exact:
                if stage == 1:
                    aggregate_exact()
            elif self.f32:
                _lib.check(L.sgn_aggregate_f32(nl, dim, bp, _lib.ptr(self._proj), ctypes.byref(pt), ctypes.byref(qo), cap, o.K,
                                               _lib.ptr(self.packed), _lib.ptr(self.feat), blend, wnorm,
                                               _lib.ptr(self.agg_ws), self.agg_ws.numel(), stage, st), "sgn_aggregate_f32")
            else:
                _lib.check(L.sgn_aggregate_sg(nl, dim, bp, _lib.ptr(self._proj), ctypes.byref(pt), ctypes.byref(qo), cap,
                                              o.K, _lib.ptr(self.packed), _lib.ptr(self.feat), blend, wnorm,
                                              _lib.ptr(self.agg_ws), self.agg_ws.numel(), stage, st), "sgn_aggregate_sg")
        mark("composite")
        cp = _lib.CompositeParams()
        cp.SR, cp.vsize_z, cp.raydist_mode_unit = o.SR, float(o.vsize[2]), o.raydist_mode_unit
        if bg is None:
            bg = (1.0, 1.0, 1.0) if o.bg_color == "white" else (0.0, 0.0, 0.0)
        for i in range(3):
            cp.bg[i] = bg[i]

        def composite():
            _lib.check(L.sgn_composite(ctypes.byref(cp), _lib.ptr(campos), _lib.ptr(rot), _lib.ptr(raydir), R,
                                       _lib.ptr(q.t_table), q.per_ray_t, q.t_table.shape[-1], ctypes.byref(qo),
                                       _lib.ptr(self.feat), _lib.ptr(self.rgb), _lib.ptr(self.mask), _lib.ptr(self.bgT),
                                       _lib.ptr(self.opacity) if want_opacity else None,
                                       _lib.ptr(self.blendw) if want_weights else None, _lib.stream_handle()),
                       "sgn_composite")
        composite()
        mark("end")
        self._range_check(check_range, lambda: (aggregate_exact(), composite()))
        return RenderOut(self.rgb[:R], self.mask[:R], self.bgT[:R], self.opacity[:R], q, self.feat, self.blend,
                         self.wnorm if want_weights else None, self.blendw[:R] if want_weights else None)

    def points_projected(self):
        """The last frame's projected point count and the neighbour indices >= n_points met so far
        (host sync), or None before any frame (or on the plain-fp32 fallback path only)."""
        if self._fp is None:
            return None
        c, bad = (int(x) for x in self._fp[3].tolist())
        return c, bad

    def grid_info(self):
        return self.querier.grid_for(self.points.xyz).info()
