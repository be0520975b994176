"""The plane background of bgmodel '*plane' (DTU scenes): each ray's background colour is the
source images warped onto a known ground plane.  Setup-time work, once per view set, outside the
per-ray hot path, so it stays torch on the device like the reference's own helpers; the per-ray
hot path only consumes the result (`inputs['bg_ray']`, blended as T_bg * bg_ray in
ray_marching.NeuralPointsRayMarching.render, neural_points_volumetric_model.py:114-116).

Restates models/mvs/mvs_utils.py:299-331 (homo_warp_nongrid, homo_warp_fg_mask), :372-420
(id2mask, gen_bg_points, get_rayplane_cross, extract_from_2d_grid) and
models/mvs_points_volumetric_model.py:276-315 (set_bg)."""
import torch
import torch.nn.functional as F


def rayplane_cross(campos, raydir, plane_pnt, plane_normal, epsilon=1e-3):
    """get_rayplane_cross (mvs_utils.py:387-408): campos [1,3], raydir [1,R,3] -> [1,R,3] world points
    where the rays meet the plane; rays with normal . dir < epsilon get (0, 0, 0)."""
    p_co = plane_pnt.reshape(1, 1, 3)
    p_no = plane_normal.reshape(1, 1, 3)
    dot = torch.sum(p_no * raydir, dim=-1)                      # [1, R]
    board = dot >= epsilon
    w = campos.reshape(1, 1, 3) - p_co
    fac = -torch.sum(p_no * w, dim=-1) / torch.where(board, dot, torch.ones_like(dot))
    hit = campos.reshape(1, 1, 3) + raydir * fac[..., None]
    return torch.where(board[..., None], hit, torch.zeros_like(hit))


def gen_bg_points(batch):
    """gen_bg_points (mvs_utils.py:380-385): the plane crossings of batch['raydir'] from batch['campos']."""
    dev = batch["campos"].device
    pnt = torch.as_tensor(batch["plane_pnt"][0], dtype=torch.float32, device=dev)
    nrm = torch.as_tensor(batch["plane_normal"][0], dtype=torch.float32, device=dev)
    return rayplane_cross(batch["campos"].reshape(1, 3).float(), batch["raydir"].float(), pnt, nrm)


def _project(c2w, w2c, intrinsic, xyz):
    """[xyz, 1] c2w^T w2c^T, then the pinhole projection (mvs_utils.py:302-306); -> pixel xy [B,M,2]."""
    cam = torch.cat([xyz, torch.ones_like(xyz[..., :1])], dim=-1) @ c2w.transpose(1, 2) @ w2c.transpose(1, 2)
    return ((cam[..., :3] / cam[..., 2:3]) @ intrinsic.transpose(1, 2))[..., :2]


def _inside(grid, HD, WD):
    lo = grid >= 0
    hi = grid <= torch.tensor([[[WD - 1, HD - 1]]], dtype=grid.dtype, device=grid.device)
    return torch.all(torch.cat([lo, hi], dim=-1), dim=-1, keepdim=True)   # [B, M, 1]


def homo_warp_nongrid(c2w, w2c, intrinsic, xyz, HD, WD):
    """homo_warp_nongrid(filter=False) (mvs_utils.py:299-315): normalised sampling grid [B,M,2] (in
    [-1, 1] inside the image), in-image mask [B,M,1] and the ceil'd pixel ids [B,M,2]."""
    grid = _project(c2w, w2c, intrinsic, xyz).to(torch.float32)
    mask = _inside(grid, HD, WD)
    hard = torch.ceil(grid)
    norm = torch.stack([grid[..., 0] / ((WD - 1.0) / 2.0) - 1.0, grid[..., 1] / ((HD - 1.0) / 2.0) - 1.0], dim=-1)
    return norm, mask, hard


def homo_warp_fg_mask(c2w, w2c, intrinsic, xyz, HD, WD):
    """homo_warp_fg_mask + id2mask (mvs_utils.py:318-331, 372-376): int8 [HD, WD], 1 where a point of
    `xyz` [1,N,3] projects (ceil'd pixel ids)."""
    grid = _project(c2w, w2c, intrinsic, xyz).to(torch.float32)
    m = _inside(grid, HD, WD)[0, :, 0]
    hard = torch.ceil(grid)[0, m].long()
    out = torch.zeros(HD, WD, dtype=torch.int8, device=xyz.device)
    out[hard[:, 1], hard[:, 0]] = 1
    return out


def extract_from_2d_grid(src_feat, src_grid, mask):
    """extract_from_2d_grid (mvs_utils.py:411-420): bilinear samples of src_feat [1,C,H,W] at the
    normalised points src_grid [1,M,2] (zeros outside, align_corners=True), scattered into [1,N,C] at
    the rows `mask` [1,N,1] selects."""
    B, M, _ = src_grid.shape
    w = F.grid_sample(src_feat, src_grid[:, None], mode="bilinear", padding_mode="zeros", align_corners=True)
    w = w.permute(0, 2, 3, 1).reshape(B, M, src_feat.shape[1])
    full = torch.zeros(B, mask.shape[1], src_feat.shape[1], dtype=w.dtype, device=w.device)
    full[0, mask[0, :, 0]] = w
    return full


def plane_bg(xyz_world_sect_plane, img_lst, w2cs_lst, intrinsics_all, HDWD_lst, plane_color, points_xyz,
             fg_masks=None, thresh=0.03):
    """set_bg's computation (mvs_points_volumetric_model.py:276-315).  For each source view: the ray's
    plane point projected into it, kept where it lands inside the image on a pixel no neural point
    projects to (the view's foreground mask, from `points_xyz` unless `fg_masks` [1,V,HD,WD] is given),
    the image bilinearly sampled there; a view's sample counts only when every channel is within
    `thresh` of plane_color; the ray's background is the channel-wise max over the views that count
    (0 when none does).  Returns (bg_ray [1,R,3], fg_masks as given -- the reference returns its
    argument, mvs_points_volumetric_model.py:314)."""
    xyz = xyz_world_sect_plane.reshape(1, -1, 3).float()
    dev = xyz.device
    c2w = torch.eye(4, device=dev, dtype=torch.float32)[None]
    pc = torch.as_tensor(plane_color, dtype=torch.float32, device=dev).reshape(-1)
    warped = []
    for count, (imgs, w2c, intrinsics, HDWD) in enumerate(zip(img_lst, w2cs_lst, intrinsics_all, HDWD_lst)):
        HD, WD = int(HDWD[0]), int(HDWD[1])
        w2c = torch.as_tensor(w2c, dtype=torch.float32, device=dev)[:, 0]
        intrinsics = torch.as_tensor(intrinsics, dtype=torch.float32, device=dev)
        grid, mask, hard = homo_warp_nongrid(c2w, w2c, intrinsics, xyz, HD, WD)
        inside = mask[0, :, 0]
        hv = hard[0, inside].long()
        if fg_masks is None:
            fg = homo_warp_fg_mask(c2w, w2c, intrinsics, points_xyz.reshape(1, -1, 3).float(), HD, WD)
        else:
            fg = fg_masks[:, count]
            fg = fg.reshape(fg.shape[-2], fg.shape[-1])
        keep = inside.clone()
        keep[inside] = fg[hv[:, 1], hv[:, 0]] < 1
        mask = keep.reshape(1, -1, 1)
        src = torch.as_tensor(imgs, dtype=torch.float32, device=dev)[0:1]
        warped.append(extract_from_2d_grid(src, grid[:, keep], mask))
    w = torch.stack(warped, dim=-2)                                  # [1, R, V, 3]
    fit = torch.all((w >= pc - thresh) & (w <= pc + thresh), dim=-1, keepdim=True)
    w = torch.where(fit, w, torch.zeros_like(w))
    return torch.max(w, dim=-2)[0], fg_masks
