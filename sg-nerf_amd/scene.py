"""Seeded synthetic scenes and cameras (no datasets/checkpoints exist offline).

Scenes follow SURVEY.md §8(d):
  * synth-room: room [0,4]x[0,4]x[0,3] m, points uniform on the 6 faces plus 8
    axis-aligned boxes, jitter N(0, 0.002); per-point embedding U(-0.5,0.5)
    (matches `torch.rand - 0.5`, neural_points.py:386), colour U(0,1), dir random
    unit, conf U(0.5,1).
  * dense: points uniform in a 1 m cube in front of the camera.
  * lego stand-in: sphere shell + 3 boxes (no lego cloud in the container).
Cameras: ScanNet-style un-normalised ray directions (get_dtu_raydir,
data/data_utils.py:55-69, dir_norm=0) and Blender-style (get_blender_raydir
:41-53, pose_spherical data/load_blender.py:51-56).
"""
from dataclasses import dataclass

import numpy as np


@dataclass
class PointCloud:
    xyz: np.ndarray        # float32 [N,3]
    embedding: np.ndarray  # float32 [N,32]
    color: np.ndarray      # float32 [N,3]
    dir: np.ndarray        # float32 [N,3]
    conf: np.ndarray       # float32 [N,1]
    bpnet: np.ndarray = None   # float32 [N,96] SG BPNet point embedding (optional)
    labels: np.ndarray = None  # int32 [N] SG point labels (optional)

    @property
    def n(self):
        return self.xyz.shape[0]


def with_semantics(pc, seed=0, n_classes=20, bpnet_dim=96, cell=None):
    """Synthetic stand-ins for the BPNet outputs the SG variant consumes (set_bpnet_feats,
    neural_points.py:653-665): a 96-d per-point embedding and labels 0..n_classes-1.
    cell=None: labels random per point; cell=c: one label per c-metre cube (spatially
    coherent, as a segmentation is)."""
    rng = np.random.default_rng(seed)
    emb = (rng.standard_normal((pc.n, bpnet_dim)) * 0.5).astype(np.float32)
    if cell is None:
        lab = rng.integers(0, n_classes, pc.n).astype(np.int32)
    else:
        c = np.floor(pc.xyz / cell).astype(np.int64)
        h = (c[:, 0] * 73856093) ^ (c[:, 1] * 19349663) ^ (c[:, 2] * 83492791)
        lab = (np.abs(h) % n_classes).astype(np.int32)
    return PointCloud(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, emb, lab)


def _attributes(rng, n, feat_dim=32):
    emb = (rng.random((n, feat_dim), dtype=np.float32) - np.float32(0.5)).astype(np.float32)
    col = rng.random((n, 3), dtype=np.float32)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32) + np.float32(1e-12)
    conf = (np.float32(0.5) + np.float32(0.5) * rng.random((n, 1), dtype=np.float32)).astype(np.float32)
    return emb, col, d.astype(np.float32), conf


def _box_faces(lo, hi):
    """(origin, u, v, area) for the 6 faces of an axis-aligned box."""
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    ext = hi - lo
    faces = []
    for ax in range(3):
        a1, a2 = [a for a in range(3) if a != ax]
        for side in (lo[ax], hi[ax]):
            o = lo.copy()
            o[ax] = side
            u = np.zeros(3); u[a1] = ext[a1]
            v = np.zeros(3); v[a2] = ext[a2]
            faces.append((o, u, v, ext[a1] * ext[a2]))
    return faces


def _sample_faces(rng, faces, n):
    areas = np.array([f[3] for f in faces])
    counts = rng.multinomial(n, areas / areas.sum())
    out = []
    for (o, u, v, _), c in zip(faces, counts):
        st = rng.random((c, 2))
        out.append(o[None] + st[:, :1] * u[None] + st[:, 1:] * v[None])
    return np.concatenate(out, 0)


def synth_room(n_points=1_200_000, seed=0, jitter=0.002):
    rng = np.random.default_rng(seed)
    faces = _box_faces((0, 0, 0), (4, 4, 3))
    for _ in range(8):
        size = rng.uniform(0.3, 1.0, 3)
        lo = np.array([rng.uniform(0.2, 3.8 - size[0]), rng.uniform(0.2, 3.8 - size[1]), 0.0])
        faces += _box_faces(lo, lo + size)
    xyz = _sample_faces(rng, faces, n_points)
    xyz = xyz + rng.normal(0.0, jitter, xyz.shape)
    xyz = xyz[rng.permutation(len(xyz))].astype(np.float32)
    return PointCloud(xyz, *_attributes(rng, len(xyz)))


def room_corner(n_points=60_000, seed=0, jitter=0.002):
    """A 1.2 m room corner (floor and two walls) with two boxes in front of it, at the
    ScanNet-like surface density of synth_room(1.2M) (~14k points / m^2): a small scene whose
    rays cross several surfaces (about 6 samples per ray, 7 of 8 neighbours per sample)."""
    rng = np.random.default_rng(seed)
    lo, hi = np.array([1.0, 1.0, 0.0]), np.array([2.2, 2.2, 1.2])
    faces = []
    for ax in range(3):      # the three faces through `lo`
        a1, a2 = [a for a in range(3) if a != ax]
        u = np.zeros(3); u[a1] = hi[a1] - lo[a1]
        v = np.zeros(3); v[a2] = hi[a2] - lo[a2]
        faces.append((lo.copy(), u, v, u[a1] * v[a2]))
    faces += _box_faces((1.25, 1.3, 0.0), (1.6, 1.65, 0.35))
    faces += _box_faces((1.55, 1.75, 0.0), (1.8, 2.0, 0.5))
    xyz = _sample_faces(rng, faces, n_points)
    xyz = xyz + rng.normal(0.0, jitter, xyz.shape)
    xyz = xyz[rng.permutation(len(xyz))].astype(np.float32)
    return PointCloud(xyz, *_attributes(rng, len(xyz)))


def dense_cube(n_points=500_000, seed=0, center=(2.0, 2.0, 3.2), side=1.0):
    rng = np.random.default_rng(seed)
    xyz = (np.asarray(center)[None] + (rng.random((n_points, 3)) - 0.5) * side).astype(np.float32)
    return PointCloud(xyz, *_attributes(rng, n_points))


def dense_stress_view(h=800, w=800, shift=0.0):
    """SURVEY §8d's dense stress variant: the 1 m cube of dense_cube() (centre (2, 2, 3.2)) seen
    face-on from 1 m with fx = fy = w (every ray enters the cube, so each of the first SR
    candidates is occupied with >= K neighbours); `shift` slides the camera sideways (m)."""
    return room_view(h, w, yaw=90.0, pitch=0.0, campos=(2.0 + shift, 0.5, 3.2), focal=float(w))


def lego_standin(n_points=300_000, seed=0):
    rng = np.random.default_rng(seed)
    n_sph = n_points // 2
    d = rng.standard_normal((n_sph, 3))
    sph = d / np.linalg.norm(d, axis=1, keepdims=True)
    faces = []
    for lo, hi in [((-0.5, -0.5, -0.5), (0.0, 0.5, 0.2)), ((0.1, -0.3, -0.6), (0.5, 0.3, 0.0)),
                   ((-0.2, -0.6, 0.1), (0.3, -0.1, 0.6))]:
        faces += _box_faces(lo, hi)
    box = _sample_faces(rng, faces, n_points - n_sph)
    xyz = np.concatenate([sph, box], 0)
    xyz = (xyz + rng.normal(0, 0.002, xyz.shape))[rng.permutation(n_points)].astype(np.float32)
    return PointCloud(xyz, *_attributes(rng, n_points))


# ---- cameras -------------------------------------------------------------------

def look_rotation(yaw_deg, pitch_deg):
    """camrotc2w whose camera +z looks along (yaw, pitch); x right, y down (OpenCV)."""
    yaw, pitch = np.deg2rad(yaw_deg), np.deg2rad(pitch_deg)
    fwd = np.array([np.cos(pitch) * np.cos(yaw), np.cos(pitch) * np.sin(yaw), np.sin(pitch)])
    up = np.array([0.0, 0.0, 1.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    down = np.cross(fwd, right)
    return np.stack([right, down, fwd], axis=1).astype(np.float32)  # columns = camera axes


def intrinsic_matrix(fx, fy, cx, cy):
    return np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], dtype=np.float32)


def pixel_grid(h, w):
    px, py = np.meshgrid(np.arange(w).astype(np.float32), np.arange(h).astype(np.float32))
    return np.stack((px, py), axis=-1).astype(np.float32)  # H x W x 2


def dtu_raydir(pixelcoords, intrinsic, rot):
    """get_dtu_raydir (data/data_utils.py:55-69), dir_norm = 0."""
    x = (pixelcoords[..., 0] + 0.5 - intrinsic[0, 2]) / intrinsic[0, 0]
    y = (pixelcoords[..., 1] + 0.5 - intrinsic[1, 2]) / intrinsic[1, 1]
    z = np.ones_like(x)
    dirs = np.stack([x, y, z], axis=-1)
    return (dirs @ rot[:, :].T).astype(np.float32)


def blender_raydir(pixelcoords, height, width, focal, rot):
    """get_blender_raydir (data/data_utils.py:41-53), dir_norm = 0."""
    x = (pixelcoords[..., 0] + 0.5 - width / 2.0) / focal
    y = (pixelcoords[..., 1] + 0.5 - height / 2.0) / focal
    z = np.ones_like(x)
    dirs = np.stack([x, -y, -z], axis=-1)
    return np.sum(dirs[..., None, :] * rot[:, :], axis=-1).astype(np.float32)


def pose_spherical(theta, phi, radius):
    """data/load_blender.py:51-56."""
    trans_t = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, radius], [0, 0, 0, 1]], dtype=np.float32)
    ph, th = phi / 180.0 * np.pi, theta / 180.0 * np.pi
    rot_phi = np.array([[1, 0, 0, 0], [0, np.cos(ph), -np.sin(ph), 0], [0, np.sin(ph), np.cos(ph), 0],
                        [0, 0, 0, 1]], dtype=np.float32)
    rot_theta = np.array([[np.cos(th), 0, -np.sin(th), 0], [0, 1, 0, 0], [np.sin(th), 0, np.cos(th), 0],
                          [0, 0, 0, 1]], dtype=np.float32)
    c2w = rot_theta @ (rot_phi @ trans_t)
    return (np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]]) @ c2w).astype(np.float32)


@dataclass
class View:
    campos: np.ndarray     # float32 [3]
    camrotc2w: np.ndarray  # float32 [3,3]
    raydir: np.ndarray     # float32 [R,3]
    pixel_idx: np.ndarray  # float32 [R,2]
    intrinsic: np.ndarray  # float32 [3,3]
    h: int
    w: int
    near: float
    far: float


def room_view(h=800, w=800, yaw=30.0, pitch=-10.0, campos=(2.0, 2.0, 1.5), focal=None,
              near=0.1, far=8.0, pixels=None):
    """ScanNet-style view from inside synth-room (fx=fy=h/2, cx=cy=centre)."""
    f = float(h) / 2.0 if focal is None else float(focal)
    K = intrinsic_matrix(f, f, w / 2.0, h / 2.0)
    rot = look_rotation(yaw, pitch)
    pix = pixel_grid(h, w).reshape(-1, 2) if pixels is None else np.asarray(pixels, np.float32).reshape(-1, 2)
    rd = dtu_raydir(pix, K, rot)
    return View(np.asarray(campos, np.float32), rot, rd.reshape(-1, 3), pix, K, h, w, near, far)


def spiral_yaw_pitch(i, n=120):
    """Config C3 spiral: yaw 0->360 deg, pitch 10*sin(2 pi i / n) deg."""
    return 360.0 * i / n, 10.0 * np.sin(2 * np.pi * i / n)


def lego_view(theta=30.0, h=800, w=800, focal=1111.1111, near=2.0, far=6.0):
    c2w = pose_spherical(theta, -30.0, 4.0)
    rot, pos = c2w[:3, :3], c2w[:3, 3]
    pix = pixel_grid(h, w).reshape(-1, 2)
    rd = blender_raydir(pix, h, w, focal, rot)
    K = intrinsic_matrix(focal, focal, w / 2.0, h / 2.0)
    return View(pos.astype(np.float32), rot.astype(np.float32), rd.reshape(-1, 3), pix, K, h, w, near, far)
