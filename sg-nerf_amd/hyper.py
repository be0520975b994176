"""Grid hyper-parameters, restating lighting_fast_querier.get_hyperparameters
(models/neural_points/query_point_indices_worldcoords.py:66-92) with the same
float32/float64 promotion chain, so the voxel origin, size, dims and radius are
bit-identical to the reference's.
"""
from dataclasses import dataclass

import numpy as np
import torch


@dataclass(frozen=True)
class GridHyper:
    ranges: np.ndarray        # float32[6]   ranges_np (:82)
    shift: np.ndarray         # float32[3]   d_coord_shift = ranges[:3] (:793)
    vsize: np.ndarray         # float64[3]   vsize_np (as passed in, :97)
    scaled_vsize: np.ndarray  # float32[3]   (:73)
    scaled_vdim: np.ndarray   # int32[3]     (:86)
    radius_limit: np.float32  # (:91)
    r2: np.float32            # np.float32(radius_limit ** 2) (:894)

    @property
    def volume(self):
        return int(np.prod(self.scaled_vdim.astype(np.int64)))


def grid_hyperparameters(opts, min_xyz, max_xyz):
    """min_xyz/max_xyz: float32 torch tensors [3] (per-axis point extent)."""
    vsize_np = list(opts.vsize)
    vscale_np = np.array(opts.vscale, dtype=np.int32)
    scaled_vsize_np = (vsize_np * vscale_np).astype(np.float32)
    min_xyz = min_xyz.detach().to("cpu", torch.float32)
    max_xyz = max_xyz.detach().to("cpu", torch.float32)
    if opts.ranges is not None:
        rg = list(opts.ranges)
        min_xyz = torch.max(torch.stack([min_xyz, torch.as_tensor(rg[:3], dtype=torch.float32)], dim=0), dim=0)[0]
        max_xyz = torch.min(torch.stack([max_xyz, torch.as_tensor(rg[3:], dtype=torch.float32)], dim=0), dim=0)[0]
    pad = torch.as_tensor(scaled_vsize_np * list(opts.kernel_size) / 2, dtype=torch.float32)
    min_xyz = min_xyz - pad
    max_xyz = max_xyz + pad
    ranges_np = torch.cat([min_xyz, max_xyz], dim=-1).numpy().astype(np.float32)
    vdim_np = (max_xyz - min_xyz).numpy() / vsize_np
    scaled_vdim_np = np.ceil(vdim_np / vscale_np).astype(np.int32)
    radius_limit_np = np.asarray(opts.radius_limit_scale * max(vsize_np[0], vsize_np[1])).astype(np.float32)
    r2 = np.float32(radius_limit_np ** 2)
    return GridHyper(ranges=ranges_np, shift=ranges_np[:3].copy(), vsize=np.asarray(vsize_np),
                     scaled_vsize=scaled_vsize_np, scaled_vdim=scaled_vdim_np,
                     radius_limit=np.float32(radius_limit_np), r2=r2)


def point_extent(xyz):
    """Per-axis min/max of a [N,3] (or [1,N,3]) tensor, as the reference's
    torch.min/max(dim=-2) (:71); one small device->host copy."""
    x = xyz.reshape(-1, 3)
    return torch.min(x, dim=0)[0].cpu(), torch.max(x, dim=0)[0].cpu()
