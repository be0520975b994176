"""ctypes binding of libsgn_hip.so (C ABI: include/sgn_hip.h).

This is the only place the HIP library is loaded.  There is no fallback: if the
library is missing or a call fails, an exception is raised.  Pointers passed in
are raw device addresses of torch tensors (``tensor.data_ptr()``) and the
stream is ``torch.cuda.current_stream().cuda_stream``.
"""
import ctypes
import os

import torch  # noqa: F401  -- loads torch's libamdhip64 first so the .so binds to the same runtime

# SGN_HIP_LIB: another build of the same ABI (same-box A/B of kernel variants, tools/ab_lib.sh)
LIB_PATH = os.environ.get("SGN_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsgn_hip.so")
ABI_VERSION = 20
COLSUM_SLABS = 512   # SGN_COLSUM_SLABS

c_i32, c_i64, c_u64, c_f32, c_vp, c_sz = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64,
                                         ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t)


class GridParams(ctypes.Structure):
    _fields_ = [("shift", c_f32 * 3), ("vs", c_f32 * 3), ("dims", c_i32 * 3),
                ("kernel", c_i32 * 3), ("query", c_i32 * 3), ("max_o", c_i32), ("P", c_i32),
                ("fix_occ0", c_i32), ("seed", c_u64)]


class GridInfo(ctypes.Structure):
    _fields_ = [("n_points", c_i64), ("n_claimed", c_i64), ("n_slots", c_i64),
                ("n_listed", c_i64), ("volume", c_i64), ("device_bytes", c_i64)]


class QueryParams(ctypes.Structure):
    _fields_ = [("SR", c_i32), ("K", c_i32), ("D", c_i32), ("per_ray_t", c_i32), ("r2", c_f32),
                ("dense_out", c_i32), ("semantic", c_i32), ("seconds", c_u64),
                ("count_traffic", c_i32)]


class QueryOut(ctypes.Structure):
    _fields_ = [("ray_ns", c_vp), ("ray_soff", c_vp), ("samp_ray", c_vp), ("samp_d", c_vp),
                ("samp_nnb", c_vp), ("pidx", c_vp), ("work", c_vp), ("counters", c_vp),
                ("samp_locw", c_vp)]


class PointTables(ctypes.Structure):
    _fields_ = [("xyz", c_vp), ("embedding", c_vp), ("color", c_vp), ("dir", c_vp),
                ("conf", c_vp), ("n_points", c_i64), ("campos", c_vp), ("camrotc2w", c_vp),
                ("raydir", c_vp), ("pers", c_vp), ("samp_pers", c_vp)]


class AggSaved(ctypes.Structure):
    _fields_ = [("x0", c_vp), ("h1", c_vp), ("h2", c_vp), ("h3", c_vp)]


class AggDeltas(ctypes.Structure):
    _fields_ = [("d4", c_vp), ("d3", c_vp), ("d2", c_vp), ("d1", c_vp), ("h4", c_vp), ("dza", c_vp)]


class PointGrads(ctypes.Structure):
    _fields_ = [("embedding", c_vp), ("color", c_vp), ("dir", c_vp), ("conf", c_vp)]


class CompositeParams(ctypes.Structure):
    _fields_ = [("SR", c_i32), ("vsize_z", c_f32), ("raydist_mode_unit", c_i32), ("bg", c_f32 * 3)]


class LossParams(ctypes.Structure):
    _fields_ = [("SR", c_i32), ("K", c_i32), ("vsize_z", c_f32), ("raydist_mode_unit", c_i32), ("bg", c_f32 * 3),
                ("zero_one_weight", c_f32), ("zero_one_eps", c_f32), ("bg_ray", c_vp)]


class GradSegment(ctypes.Structure):
    _fields_ = [("src", c_vp), ("tail", c_vp), ("dst", c_vp), ("n", c_i64), ("stride", c_i64), ("nb", c_i32),
                ("reserved", c_i32)]


class GatherSegment(ctypes.Structure):
    _fields_ = [("idx", c_vp), ("dst", c_vp), ("n", c_i64), ("fp16", c_i32), ("reserved", c_i32)]


class X3Operand(ctypes.Structure):
    _fields_ = [("p", c_vp), ("p2", c_vp), ("ld", c_i64), ("ld2", c_i64), ("csplit", c_i32), ("ncols", c_i32),
                ("ones_col", c_i32), ("act", c_i32), ("kmajor", c_i32), ("amax", c_vp), ("shift", c_vp)]


class X3GemmArgs(ctypes.Structure):
    _fields_ = [("a", X3Operand), ("b", X3Operand), ("mode", c_i32), ("M", c_i32), ("N", c_i32), ("K", c_i32),
                ("d_rows", c_vp), ("bias", c_vp), ("act", c_i32), ("mask", c_vp), ("ldm", c_i64), ("out", c_vp),
                ("ldo", c_i64), ("out_cols", c_i32), ("out2", c_vp), ("ldo2", c_i64), ("amax_out", c_vp),
                ("amax_out2", c_vp), ("part", c_vp), ("splits", c_i32), ("products", c_i32), ("bpack", c_vp)]


class PartialSegment(ctypes.Structure):
    _fields_ = [("part", c_vp), ("splits", c_i32), ("M", c_i32), ("N", c_i32), ("n_in", c_i32), ("bias_col", c_i32),
                ("ldw", c_i32), ("dst_w", c_vp), ("dst_b", c_vp)]


# name -> (restype, argtypes); every symbol include/sgn_hip.h declares.
SIGNATURES = {
    "sgn_abi_version": (c_i32, []),
    "sgn_last_error": (ctypes.c_char_p, []),
    "sgn_grid_build": (c_i32, [c_vp, c_i64, ctypes.POINTER(GridParams), c_vp, ctypes.POINTER(c_vp)]),
    "sgn_grid_free": (c_i32, [c_vp]),
    "sgn_grid_get_info": (c_i32, [c_vp, ctypes.POINTER(GridInfo)]),
    "sgn_grid_export": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "sgn_depth_table_jitter": (c_i32, [c_f32, c_f32, c_i32, c_f32, c_i64, c_vp, c_vp, c_vp]),
    "sgn_query_workspace_bytes": (c_sz, [c_i64]),
    "sgn_query": (c_i32, [c_vp, ctypes.POINTER(QueryParams), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                          ctypes.POINTER(QueryOut), c_vp, c_sz, c_vp]),
    "sgn_mlp_packed_bytes": (c_sz, []),
    "sgn_mlp_pack": (c_i32, [ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_vp, c_vp]),
    "sgn_aggregate_workspace_bytes": (c_sz, [c_i64]),
    "sgn_aggregate": (c_i32, [ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i64, c_i32,
                              c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_i32, c_vp]),
    "sgn_mlp_packed_bytes_sg": (c_sz, [c_i32, c_i32]),
    "sgn_mlp_pack_sg": (c_i32, [c_i32, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_vp, c_vp]),
    "sgn_bpnet_pack": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    "sgn_point_proj_bytes": (c_sz, [c_i64]),
    "sgn_point_project": (c_i32, [ctypes.POINTER(PointTables), c_vp, c_vp, c_vp]),
    "sgn_mlp_section": (c_sz, [c_i32]),
    "sgn_aggregate_sg": (c_i32, [c_i32, c_i32, c_vp, c_vp, ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i64,
                                 c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_i32, c_vp]),
    "sgn_aggregate_train_fwd": (c_i32, [ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i64, c_i32, c_vp,
                                        c_vp, c_vp, ctypes.POINTER(AggSaved), c_vp]),
    "sgn_train_tblob_bytes": (c_sz, []),
    "sgn_train_pack_t": (c_i32, [ctypes.POINTER(c_vp), c_vp, c_vp]),
    "sgn_mlp_pack_index": (c_i32, [c_i32, ctypes.POINTER(c_i32), c_i64]),
    "sgn_train_pack_index": (c_i32, [ctypes.POINTER(c_i32), c_i64]),
    "sgn_train_colmap": (c_i32, [c_i32, ctypes.POINTER(c_i32), c_i32]),
    "sgn_aggregate_backward": (c_i32, [ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i32, c_i32, c_vp, c_vp,
                                       ctypes.POINTER(AggSaved), c_vp, c_vp, c_vp, ctypes.POINTER(AggDeltas),
                                       ctypes.POINTER(PointGrads), c_vp]),
    "sgn_aggregate_train_fwd_sg": (c_i32, [c_i32, c_i32, c_vp, ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut),
                                           c_i64, c_i32, c_vp, c_vp, c_vp, ctypes.POINTER(AggSaved), c_vp, c_vp]),
    "sgn_aggregate_backward_sg": (c_i32, [c_i32, c_i32, ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i32,
                                          c_i32, c_vp, c_vp, ctypes.POINTER(AggSaved), c_vp, c_vp, c_vp, c_vp,
                                          ctypes.POINTER(AggDeltas), c_vp, ctypes.POINTER(PointGrads), c_vp]),
    "sgn_train_pack_t_sg": (c_i32, [ctypes.POINTER(c_vp), c_i32, c_vp, c_vp]),
    "sgn_mlp_pack_index_sg": (c_i32, [c_i32, c_i32, c_i32, ctypes.POINTER(c_i32), c_i64]),
    "sgn_train_pack_index_sg": (c_i32, [c_i32, ctypes.POINTER(c_i32), c_i64]),
    "sgn_adam_step": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                               ctypes.c_double, c_i64, c_i32, c_vp]),
    "sgn_adam_step_multi": (c_i32, [c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                                     ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, c_i64, c_i32, c_vp]),
    "sgn_adam_rows_workspace_bytes": (c_sz, [c_i64]),
    "sgn_adam_rows_pend_bytes": (c_sz, [c_i64]),
    "sgn_adam_rows": (c_i32, [c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                              ctypes.POINTER(c_vp), ctypes.POINTER(c_i32), ctypes.POINTER(c_i32), c_i64, c_vp, c_vp,
                              c_i32, c_i32, c_i64,
                              c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_vp, c_sz, c_vp, c_sz, c_vp,
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_i64, c_i32, c_i32,
                              c_vp]),
    "sgn_point_project_subset": (c_i32, [ctypes.POINTER(PointTables), c_vp, c_vp, c_vp, c_vp, c_vp]),
    "sgn_frame_points_mark_bytes": (c_sz, [c_i64]),
    "sgn_frame_points": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "sgn_colsum_workspace_bytes": (c_sz, [c_i32]),
    "sgn_colsum_f16": (c_i32, [c_i32, ctypes.POINTER(c_vp), c_i64, c_i32, c_vp, c_vp, c_vp]),
    "sgn_colsum_f16_weighted": (c_i32, [c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_i64, c_i32, c_vp, c_vp,
                                        c_vp]),
    "sgn_colsum_f16_weighted_parts": (c_i32, [c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_i64, c_i32, c_vp,
                                              c_vp]),
    "sgn_grad_accumulate": (c_i32, [c_i32, ctypes.POINTER(GradSegment), c_vp, c_vp, c_vp]),
    "sgn_zero_segments": (c_i32, [c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_vp]),
    "sgn_copy_segments": (c_i32, [c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_vp]),
    "sgn_gather_segments": (c_i32, [c_i32, ctypes.POINTER(GatherSegment), c_vp, c_i64, c_vp]),
    "sgn_pack_scaled_f32": (c_i32, [c_vp, c_i64, c_i32, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), c_vp, c_i64, c_vp,
                                    c_i64, c_vp, c_vp, c_vp, c_vp]),
    "sgn_colour_inputs": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_vp]),
    "sgn_pow2_scale_workspace_bytes": (c_sz, []),
    "sgn_pow2_scale": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "sgn_touched_points": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "sgn_mlp_packed_bytes_f32": (c_sz, [c_i32, c_i32]),
    "sgn_mlp_pack_f32": (c_i32, [c_i32, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_vp, c_vp]),
    "sgn_mlp_pack_f32_host": (c_i32, [c_i32, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_vp]),
    "sgn_point_proj_bytes_f32": (c_sz, [c_i64]),
    "sgn_point_project_f32": (c_i32, [ctypes.POINTER(PointTables), c_vp, c_vp, c_vp]),
    "sgn_point_project_f32_subset": (c_i32, [ctypes.POINTER(PointTables), c_vp, c_vp, c_vp, c_vp, c_vp]),
    "sgn_aggregate_workspace_bytes_f32": (c_sz, [c_i64]),
    "sgn_aggregate_f32": (c_i32, [c_i32, c_i32, c_vp, c_vp, ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i64, c_i32, c_vp,
                                  c_vp, c_vp, c_vp, c_vp, c_sz, c_i32, c_vp]),
    "sgn_aggregate_check_f32": (c_i32, [c_vp, c_sz, c_vp]),
    "sgn_mlp_packed_bytes_exact": (c_sz, [c_i32, c_i32]),
    "sgn_mlp_pack_exact": (c_i32, [c_i32, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_vp, c_vp]),
    "sgn_aggregate_exact": (c_i32, [c_i32, c_i32, c_vp, ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i64,
                                    c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "sgn_aggregate_flag_offset_f32": (c_sz, [c_sz]),
    "sgn_aggregate_fs_offset_f32": (c_i64, [c_sz, c_i64]),
    "sgn_aggregate_train_fwd_f32": (c_i32, [c_vp, ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i64, c_i32,
                                            c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "sgn_aggregate_train_fwd_f32_sg": (c_i32, [c_i32, c_i32, c_vp, c_vp, ctypes.POINTER(PointTables),
                                               ctypes.POINTER(QueryOut), c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp,
                                               c_vp, c_vp, c_vp, c_sz, c_vp]),
    "sgn_train_row_gather": (c_i32, [ctypes.POINTER(QueryOut), c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "sgn_x3_gemm": (c_i32, [ctypes.POINTER(X3GemmArgs), c_vp]),
    "sgn_x3_gemm_bpack_bytes": (c_sz, [ctypes.POINTER(X3GemmArgs)]),
    "sgn_f16_weight_grad": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "sgn_train_lists_workspace_bytes": (c_sz, [c_i64]),
    "sgn_train_lists": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "sgn_train_row_inputs": (c_i32, [ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i32, c_vp, c_vp, c_vp,
                                     c_vp, c_vp, c_vp, c_vp]),
    "sgn_train_colour_head": (c_i32, [ctypes.POINTER(QueryOut), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "sgn_train_head_partial_floats": (c_sz, [c_i32]),
    "sgn_train_colour_head_bwd": (c_i32, [ctypes.POINTER(QueryOut), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                          c_vp]),
    "sgn_train_row_head": (c_i32, [ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i32, c_vp, c_vp, c_vp,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "sgn_train_row_tail": (c_i32, [ctypes.POINTER(PointTables), ctypes.POINTER(QueryOut), c_i32, c_vp, c_vp, c_vp,
                                   c_vp, ctypes.POINTER(PointGrads), c_vp]),
    "sgn_reduce_partials": (c_i32, [c_i32, ctypes.POINTER(PartialSegment), c_vp]),
    "sgn_mlp_layout_f32": (c_i64, [c_i32]),
    "sgn_mlp_pack_index_f32": (c_i32, [c_i32, c_i32, c_i32, ctypes.POINTER(c_i32), c_i64]),
    "sgn_composite": (c_i32, [ctypes.POINTER(CompositeParams), c_vp, c_vp, c_vp, c_i64, c_vp, c_i32,
                              c_i32, ctypes.POINTER(QueryOut), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "sgn_loss_workspace_bytes": (c_sz, [c_i64, c_i32]),
    "sgn_loss_train": (c_i32, [ctypes.POINTER(LossParams), c_vp, c_vp, c_i64, ctypes.POINTER(QueryOut), c_vp, c_vp,
                               c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "sgn_ray_march_dense": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, ctypes.POINTER(c_f32), c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_vp]),
}


class SgnError(RuntimeError):
    pass


_LIB = None


def lib():
    """Load (once) and return the ctypes handle.  Raises if the .so is absent."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise SgnError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback for the hot path)")
        h = ctypes.CDLL(LIB_PATH)
        v = h.sgn_abi_version()
        if v != ABI_VERSION:
            raise SgnError(f"libsgn_hip.so ABI {v} != expected {ABI_VERSION}: rebuild it")
        missing = [name for name in SIGNATURES if getattr(h, name, None) is None]
        if missing:   # a stale build: fail before any GPU work, not at the first call of a missing symbol
            raise SgnError(f"libsgn_hip.so lacks {', '.join(missing)}: rebuild it")
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = h
    return _LIB


def check(rc, what):
    if rc != 0:
        msg = lib().sgn_last_error()
        raise SgnError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def copy_segments(pairs, stream=None):
    """One sgn_copy_segments launch: pairs of (src tensor or None = clear, dst tensor), byte counts
    from dst (the source must hold at least as many bytes)."""
    n = len(pairs)
    src = (c_vp * n)(*[None if s is None else s.data_ptr() for s, _ in pairs])
    dst = (c_vp * n)(*[d.data_ptr() for _, d in pairs])
    nb = (c_i64 * n)(*[d.numel() * d.element_size() for _, d in pairs])
    for s, d in pairs:
        assert d.is_contiguous() and (s is None or (s.is_contiguous() and s.numel() * s.element_size() >= d.numel() * d.element_size()))
    check(lib().sgn_copy_segments(n, src, dst, nb, stream_handle() if stream is None else stream), "sgn_copy_segments")


def ptr(t):
    """Device address of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
