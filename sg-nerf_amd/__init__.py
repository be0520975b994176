"""sgnerf_amd -- MI355X-native per-ray rendering hot path of SG-NeRF / Point-NeRF.

neural-point grid -> ray march + layered kNN -> aggregator MLP (MFMA) -> alpha
composite, as hand-written HIP kernels for gfx950 behind a C ABI
(include/sgn_hip.h, libsgn_hip.so), with host classes mirroring the
reference's operator API (NeuralPointsRayMarching.forward(inputs) -> dict).
"""
from .opts import HotPathOpts, SCANNET  # noqa: F401

__all__ = ["HotPathOpts", "SCANNET"]
