"""Candidate depths along each ray.

Restates near_far_linear_ray_generation
(models/rendering/diff_ray_marching.py:349-393), which the querier calls at
query_point_indices_worldcoords.py:103.  The reference materialises
raypos[B, R, D, 3]; the HIP march only needs the depth table t (the
reference's `middle_point_ts`) and recomputes raypos = campos + raydir * t with
the same two roundings.

Test mode (jitter 0) gives one table shared by every ray ([D], computed once on
the host with the reference's exact torch op sequence, so every consumer -- the
kernels and the oracle -- sees identical fp32 values).  Training mode (jitter
0.3) gives a per-ray table [R, D].
"""
import torch


def depth_table(near, far, D, jitter=0.0, R=1, device="cpu", generator=None):
    near = float(near)
    far = float(far)
    tvals = torch.linspace(0, 1, D + 1, device=device).view(1, -1)
    tvals = near * (1 - tvals) + far * tvals
    if jitter == 0.0:
        seg = (tvals[..., 1:] - tvals[..., :-1]).view(1, 1, D)
    else:
        rnd = torch.rand((1, R, D), device=device, generator=generator)
        seg = (tvals[..., 1:] - tvals[..., :-1]) * (1 + jitter * (rnd - 0.5))
    end = torch.cumsum(seg, dim=2)
    end = torch.cat([torch.zeros((end.shape[0], end.shape[1], 1), device=end.device), end], dim=2)
    end = near + end
    mid = (end[:, :, :-1] + end[:, :, 1:]) / 2
    return mid[0, 0].contiguous() if jitter == 0.0 else mid[0].contiguous()


_CACHE = {}


def shared_depth_table(near, far, D, device):
    """Cached test-mode table on `device` (built on CPU, then copied)."""
    key = (float(near), float(far), int(D), str(device))
    t = _CACHE.get(key)
    if t is None:
        t = depth_table(near, far, D).to(device)
        _CACHE[key] = t
    return t
