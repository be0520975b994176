"""Aggregator MLP parameters: reference-layout init and MFMA packing.

Parameter names and shapes follow PointAggregator.viewmlp_init
(models/aggregators/point_aggregators.py:312-421) at the ScanNet config, i.e. the
keys of `aggregator.*` in `{iter}_net_ray_marching.pth`.  Initialisation follows
init_seq (models/helpers/networks.py:120-172): xavier-uniform with the LeakyReLU(0.01)
gain for layers followed by an activation, gain 1 for the last layer, zero bias.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib

# (name, out, in, followed_by_activation)
LAYERS = [
    ("block1.0", 256, 284, True),
    ("block1.2", 256, 256, True),
    ("block3.0", 256, 263, True),
    ("block3.2", 256, 256, True),
    ("alpha_branch.0", 1, 256, False),
    ("color_branch.0", 128, 280, True),
    ("color_branch.2", 128, 128, True),
    ("color_branch.4", 128, 128, True),
    ("color_branch.6", 3, 128, False),
]
N_PARAMS = sum(o * i + o for _, o, i, _ in LAYERS)  # 341,764
# SG-NeRF: block2_bpnet.0 = Linear(256 + bpnet_dim, 256) + LReLU (point_aggregators.py:345-354),
# bpnet_dim = 96 with predict_semantic = 1, else 0.  Only one such layer is supported.
BPNET = "block2_bpnet.0"


def layers_for(bpnet_layers=0, bpnet_dim=0):
    if bpnet_layers not in (0, 1) or bpnet_dim not in (0, 96):
        raise NotImplementedError("block2_bpnet: 0 layers, or 1 layer with bpnet_dim 0 or 96")
    return LAYERS + ([(BPNET, 256, 256 + bpnet_dim, True)] if bpnet_layers else [])


def mlp_variant(state):
    """(bpnet_layers, bpnet_dim) of a (prefix-stripped) aggregator state."""
    w = state.get(BPNET + ".weight")
    if w is None:
        return 0, 0
    if any(k.startswith("block2_bpnet.") and not k.startswith(BPNET + ".") for k in state):
        raise NotImplementedError("only one block2_bpnet layer is supported")
    return 1, int(w.shape[1]) - 256


def init_mlp(seed=0, bias_std=0.0, bpnet_layers=0, bpnet_dim=0):
    """Reference-style init (init_seq).  bias_std > 0 perturbs biases (fixtures).  The SG
    block2_bpnet layer (if any) is drawn after the base layers, so base draws do not move."""
    g = torch.Generator().manual_seed(seed)
    leaky_gain = math.sqrt(2.0 / (1 + 0.01 ** 2))  # nn.init.calculate_gain('leaky_relu', 0.01)
    state = {}
    for name, o, i, act in LAYERS + layers_for(bpnet_layers, bpnet_dim)[len(LAYERS):]:
        gain = leaky_gain if act else 1.0
        std = gain * math.sqrt(2.0 / (i + o))
        a = std * math.sqrt(3.0)
        state[name + ".weight"] = (torch.rand((o, i), generator=g) * 2 - 1) * a
        b = torch.zeros(o)
        if bias_std > 0:
            b = torch.randn(o, generator=g) * bias_std
        state[name + ".bias"] = b
    return state


def strip_prefix(state, prefix="aggregator."):
    """Accepts a full net_ray_marching state dict (keys `aggregator.*`, `module.aggregator.*`)."""
    out = {}
    names = {n + s for n, *_ in LAYERS for s in (".weight", ".bias")}
    for k, v in state.items():
        for p in ("module." + prefix, prefix, ""):
            if k.startswith(p) and (k[len(p):] in names or k[len(p):].startswith("block2_bpnet.")):
                out[k[len(p):]] = v
                break
    missing = [n + s for n, *_ in LAYERS for s in (".weight", ".bias") if n + s not in out]
    if missing:
        raise KeyError(f"aggregator parameters missing: {missing}")
    return out


def check_shapes(state):
    for name, o, i, _ in layers_for(*mlp_variant(state)):
        w, b = state[name + ".weight"], state[name + ".bias"]
        if tuple(w.shape) != (o, i) or tuple(b.shape) != (o,):
            raise ValueError(f"{name}: expected weight {(o, i)} bias {(o,)}, got {tuple(w.shape)} {tuple(b.shape)}")


def pack_mlp(state, device, precision="f16"):
    """fp32 state -> packed MFMA fragment blob on `device` (uint8 tensor).  precision "f16":
    fp16 fragments (mlp.hip); "f32": (hi, lo) fp16 fragment pairs of 2^s-scaled weights plus
    fp32 biases (mlp_x3.hip, the reference's fp32 arithmetic); "exact": plain fp32 W^T per layer
    (exact.hip, the f32 mode's range fallback)."""
    state = strip_prefix(state)
    check_shapes(state)
    nl, dim = mlp_variant(state)
    layers = layers_for(nl, dim)
    L = _lib.lib()
    nbytes = int(L.sgn_mlp_packed_bytes_f32(nl, dim) if precision == "f32" else
                 L.sgn_mlp_packed_bytes_exact(nl, dim) if precision == "exact" else L.sgn_mlp_packed_bytes_sg(nl, dim))
    out = torch.empty(nbytes, dtype=torch.uint8, device=device)
    ws = [np.ascontiguousarray(torch.as_tensor(state[n + ".weight"]).detach().cpu().float().numpy()) for n, *_ in layers]
    bs = [np.ascontiguousarray(torch.as_tensor(state[n + ".bias"]).detach().cpu().float().numpy()) for n, *_ in layers]
    wp = (ctypes.c_void_p * len(layers))(*[w.ctypes.data for w in ws])
    bp = (ctypes.c_void_p * len(layers))(*[b.ctypes.data for b in bs])
    if torch.device(device).type == "cpu":
        if precision != "f32":
            raise ValueError("host packing: precision 'f32' only")
        _lib.check(L.sgn_mlp_pack_f32_host(nl, dim, wp, bp, out.data_ptr()), "sgn_mlp_pack_f32_host")
        return out
    with torch.cuda.device(device):
        if precision == "f32":
            _lib.check(L.sgn_mlp_pack_f32(nl, dim, wp, bp, _lib.ptr(out), _lib.stream_handle()), "sgn_mlp_pack_f32")
        elif precision == "exact":   # plain fp32 W^T for the range fallback (sgn_aggregate_exact)
            _lib.check(L.sgn_mlp_pack_exact(nl, dim, wp, bp, _lib.ptr(out), _lib.stream_handle()), "sgn_mlp_pack_exact")
        else:
            _lib.check(L.sgn_mlp_pack_sg(nl, dim, wp, bp, _lib.ptr(out), _lib.stream_handle()), "sgn_mlp_pack_sg")
    return out
