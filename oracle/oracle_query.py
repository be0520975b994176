"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of liboracle_query.so, the C
restatement of the reference query kernels (see query_ref.c for citations and
the "parity unpinned" status of this stage).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liboracle_query.so")


class Params(ctypes.Structure):
    _fields_ = [("shift", ctypes.c_float * 3), ("vs", ctypes.c_float * 3), ("dims", ctypes.c_int * 3),
                ("kernel", ctypes.c_int * 3), ("query", ctypes.c_int * 3), ("max_o", ctypes.c_int),
                ("P", ctypes.c_int), ("K", ctypes.c_int), ("SR", ctypes.c_int), ("r2", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("fix_occ0", ctypes.c_int)]


def build():
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(HERE, "query_ref.c")):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle_query.so"])


_L = None


def lib():
    global _L
    if _L is None:
        build()
        L = ctypes.CDLL(SO)
        P = ctypes.POINTER
        vp = ctypes.c_void_p
        L.sgnref_uniform.restype = ctypes.c_float
        L.sgnref_uniform.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.sgnref_grid_build.restype = ctypes.c_int64
        L.sgnref_grid_build.argtypes = [vp, ctypes.c_int64, P(Params), vp, vp, vp, vp, vp]
        L.sgnref_query.restype = None
        L.sgnref_query.argtypes = [P(Params), vp, vp, vp, vp, vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int,
                                   ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_uint64]
        L.sgnref_set_threads.restype = None
        L.sgnref_set_threads.argtypes = [ctypes.c_int]
        L.sgnref_knn_one.restype = ctypes.c_int
        L.sgnref_knn_one.argtypes = [P(Params), vp, vp, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_uint64]
        _L = L
    return _L


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def make_params(hyper, opts):
    p = Params()
    for a in range(3):
        p.shift[a] = float(hyper.shift[a])
        p.vs[a] = float(hyper.scaled_vsize[a])
        p.dims[a] = int(hyper.scaled_vdim[a])
        p.kernel[a] = int(opts.kernel_size[a])
        p.query[a] = int(opts.query_size[a])
    p.max_o, p.P, p.K, p.SR = int(opts.max_o), int(opts.P), int(opts.K), int(opts.SR)
    p.r2 = float(hyper.r2)
    p.seed = int(opts.reservoir_seed)
    p.fix_occ0 = int(opts.fix_occ0)
    return p


class OracleGrid:
    """Reference-structured grid (build_occ_vox, worldcoords.py:706-778)."""

    def __init__(self, xyz, hyper, opts):
        self.params = make_params(hyper, opts)
        self.xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        vol = int(np.prod(hyper.scaled_vdim.astype(np.int64)))
        d = [int(x) for x in hyper.scaled_vdim]
        self.coor_occ = np.empty(vol, np.int32)
        self.coor_2_occ = np.empty(vol, np.int32)
        self.occ_numpnts = np.empty(opts.max_o, np.int32)
        self.occ_2_pnts = np.empty(opts.max_o * opts.P, np.int32)
        self.occ_2_coor = np.empty(opts.max_o * 3, np.int32)
        self.occ_idx = lib().sgnref_grid_build(_p(self.xyz), self.xyz.shape[0], ctypes.byref(self.params),
                                               _p(self.coor_occ), _p(self.coor_2_occ), _p(self.occ_numpnts),
                                               _p(self.occ_2_pnts), _p(self.occ_2_coor))
        self.coor_occ = self.coor_occ.reshape(d)
        self.coor_2_occ = self.coor_2_occ.reshape(d)
        self.occ_2_pnts = self.occ_2_pnts.reshape(opts.max_o, opts.P)

    def query(self, campos, raydir, t_table, per_ray_t=False, point_labels=None, ray_labels=None, seconds=0):
        p = self.params
        raydir = np.ascontiguousarray(raydir, np.float32).reshape(-1, 3)
        campos = np.ascontiguousarray(campos, np.float32).reshape(3)
        t_table = np.ascontiguousarray(t_table, np.float32)
        R = raydir.shape[0]
        D = t_table.shape[-1]
        ray_ns = np.empty(R, np.int32)
        ray_d = np.empty(R * p.SR, np.int32)
        pidx = np.empty(R * p.SR * p.K, np.int32)
        loc_w = np.empty(R * p.SR * 3, np.float32)
        pl = None if point_labels is None else np.ascontiguousarray(point_labels, np.int32)
        rl = None if ray_labels is None else np.ascontiguousarray(ray_labels, np.int32)
        lib().sgnref_query(ctypes.byref(p), _p(self.xyz), _p(self.coor_occ), _p(self.coor_2_occ),
                           _p(self.occ_numpnts), _p(self.occ_2_pnts), _p(campos), _p(raydir), R, _p(t_table), D,
                           int(per_ray_t), _p(ray_ns), _p(ray_d), _p(pidx), _p(loc_w), _p(pl), _p(rl), int(seconds))
        return dict(ray_ns=ray_ns, ray_d=ray_d.reshape(R, p.SR), pidx=pidx.reshape(R, p.SR, p.K),
                    loc_w=loc_w.reshape(R, p.SR, 3))


def reference_layout(q):
    """Compacts an oracle query result into the reference's query_points
    outputs (worldcoords.py:833-954): (sample_pidx [R'',SR,K], sample_loc_w
    [R'',SR,3], ray_mask [R] int8)."""
    pidx, loc_w = q["pidx"], q["loc_w"]
    valid = (pidx >= 0).reshape(pidx.shape[0], -1).any(-1) & (q["ray_ns"] > 0)
    return pidx[valid], loc_w[valid], valid.astype(np.int8)
