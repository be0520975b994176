"""Model plugin for the reference's driver scripts (run/test_ft.py, run/render_vid.py).

The reference finds `models.<name>_model.<Name>Model` (models/__init__.py:5-27) and
drives it through the BaseModel surface (models/base_model.py:7-142,
models/base_rendering_model.py:387-533).  HipPointsVolumetricModel exposes that
surface for inference over the HIP hot path; INTEGRATION.md shows the three-line
shim `models/hip_points_volumetric_model.py` a maintainer adds to the reference.

Checkpoints use the reference layout: `{epoch}_net_ray_marching.pth` holding
`neural_points.{xyz,points_embeding,points_color,points_dir,points_conf}` and
`aggregator.*` (models/base_model.py:85-119), loaded with
torch.load(weights_only=True).

Training (run/train_ft.py:858-1051): optimize_parameters runs one HipTrainer step
(train_hip.py: HIP query, MFMA aggregator forward/backward, reference losses, two Adam
groups lr / plr with iter_exponential_decay, DP all-reduce when torch.distributed is up);
setup_optimizer / clean_optimizer / init_scheduler / prune_points / grow_points follow
models/mvs_points_volumetric_model.py:47-141,195-270 and neural_points.py:520-572.  The
trainable tensors are shared with `neural_points`, so test() renders the current state.

SG-NeRF's extra surface: the probe ranking (update_rank_ray_miss / rank_ray_miss /
reset_ray_miss_ranking, top_ray_miss_loss / top_ray_miss_ids, mvs_points_volumetric_model.py:
157-189) fed by the ray_miss_coarse_raycolor loss of every step; the semantic dumps
saveSemanticEmbedding / saveSemanticPoints / saveSemanticPoints_test
(neural_points_volumetric_model.py:337-362, 674-720); checkpoints carry
neural_points.points_feats / points_label / bpnet_points_embedding.  set_bg (plane background)
returns the rays' bg_ray, which test() blends as T_bg * bg_ray and optimize_parameters composites
into the loss the same way.  Pruning keeps the semantic
per-point arrays aligned with the points (the reference leaves them unpruned).
"""
import dataclasses
import os

import numpy as np
import torch

from .opts import HotPathOpts
from .ray_marching import NeuralPoints, NeuralPointsRayMarching
from .weights import strip_prefix

LOSS_NAMES = ["total", "ray_masked_coarse_raycolor", "ray_miss_coarse_raycolor", "coarse_raycolor",
              "conf_coefficient"]

# ScanNet-20 label colours of the reference's point dumps (neural_points_volumetric_model.py:35-57)
LABEL_RGB = {0: (174, 198, 232), 1: (151, 223, 137), 2: (31, 120, 180), 3: (255, 188, 120), 4: (188, 189, 35),
             5: (140, 86, 74), 6: (255, 152, 151), 7: (213, 39, 40), 8: (196, 176, 213), 9: (148, 103, 188),
             10: (196, 156, 148), 11: (23, 190, 208), 12: (247, 183, 210), 13: (218, 219, 141),
             14: (254, 127, 14), 15: (227, 119, 194), 16: (158, 218, 229), 17: (43, 160, 45),
             18: (112, 128, 144), 19: (82, 83, 163), 255: (255, 255, 170)}


def label_colours(labels):
    """[N] integer labels -> [N,3] RGB (0..255) through LABEL_RGB; an unknown label raises
    KeyError, as the reference's dict lookup does."""
    lab = np.asarray(labels).reshape(-1).astype(np.int64)
    lut = np.full((256, 3), -1, np.int64)
    for k, c in LABEL_RGB.items():
        lut[k] = c
    bad = (lab < 0) | (lab > 255)
    if bad.any() or (lut[np.clip(lab, 0, 255), 0] < 0).any():
        raise KeyError(f"label without a colour: {sorted(set(lab[bad | (lut[np.clip(lab, 0, 255), 0] < 0)].tolist()))[:8]}")
    return lut[lab].astype(np.float32)


class HipPointsVolumetricModel:
    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        parser.add_argument("--sgn_fix_occ0", type=int, default=0,
                            help="1: do not reproduce the voxel_idx>0 grid bug (worldcoords.py:395)")
        parser.add_argument("--sgn_reservoir_seed", type=int, default=0,
                            help="seed of the per-voxel reservoir (the reference uses the wall clock)")
        return parser

    def name(self):
        return self.__class__.__name__

    # -- BaseModel.initialize / setup -------------------------------------------------
    def initialize(self, opt):
        self.opt = opt
        gpu_ids = getattr(opt, "gpu_ids", [0]) or [0]
        self.device = torch.device("cuda", gpu_ids[0])
        self.is_train = bool(getattr(opt, "is_train", False))
        self.save_dir = os.path.join(getattr(opt, "checkpoints_dir", "."), getattr(opt, "name", "sgn"))
        extra = {}
        if hasattr(opt, "sgn_fix_occ0"):
            extra["fix_occ0"] = int(opt.sgn_fix_occ0)
        if hasattr(opt, "sgn_reservoir_seed"):
            extra["reservoir_seed"] = int(opt.sgn_reservoir_seed)
        # rendering (test / probe) runs the test-mode depth table; the trainer jitters (is_train)
        self.opts = HotPathOpts.from_opt(opt, **extra, is_train=0).check_supported()
        self.model_names = ["ray_marching"]
        self.visual_names = ["coarse_raycolor", "ray_mask", "coarse_is_background"]
        self.loss_names = []
        self.neural_points = None
        self.net_ray_marching = None
        self.output = {}

    def setup(self, opt, train_len=None):
        resume = getattr(opt, "resume_iter", None)
        if resume is not None and getattr(opt, "resume_dir", None):
            self.load_networks(resume)
        if self.is_train and self.neural_points is not None:
            self.setup_optimizer(opt)
            self.init_scheduler(int(getattr(opt, "resume_step", 0) or 0), opt)
        # probe ranking buffers (mvs_points_volumetric_model.py:178-184)
        prob_freq = int(getattr(opt, "prob_freq", 0) or 0)
        nstep = int(getattr(opt, "prob_num_step", 100) or 0)
        if prob_freq > 0 and train_len is not None and nstep > 1:
            self.num_probe = train_len // nstep
            self.reset_ray_miss_ranking()
        elif prob_freq > 0 and train_len is not None and nstep == 1:
            self.top_ray_miss_loss = torch.zeros([1], dtype=torch.float32, device=self.device)

    def set_points(self, points_xyz, points_feats=None, points_embedding=None, points_label=None, points_color=None,
                   points_dir=None, points_conf=None, points_semantic=None, Rw2c=None, eulers=None, editing=False,
                   aggregator_state=None):
        """mvs_points_volumetric_model.py:191-199 -> neural_points.py:575-600 (same argument names
        and order); also takes the aggregator weights when no checkpoint is loaded.  In training
        the optimizers are rebuilt over the new points."""
        if editing:
            raise NotImplementedError("set_points(editing=True) (point-cloud editing) is outside the HIP hot path")
        if points_embedding is None:
            raise ValueError("set_points: points_embedding is required")
        if points_conf is None:
            points_conf = torch.ones(points_embedding.shape[:-1] + (1,), dtype=torch.float32)
        for name, t in (("points_color", points_color), ("points_dir", points_dir)):
            if t is None:
                raise NotImplementedError(f"set_points without {name}: the MFMA aggregator's inputs include it")
        self.neural_points = NeuralPoints(points_xyz, points_embedding, points_color, points_dir, points_conf,
                                          self.device, points_feats=points_feats, points_label=points_label)
        if aggregator_state is not None or self.net_ray_marching is None:
            if aggregator_state is None:
                raise ValueError("set_points: aggregator_state required before the first render")
            self.net_ray_marching = NeuralPointsRayMarching(self.neural_points, aggregator_state, self.opts,
                                                            self.device)
        else:
            self._sync_weights()
            self.net_ray_marching.neural_points = self.neural_points
        if self.is_train:
            self.setup_optimizer(self.opt)

    # -- training (mvs_points_volumetric_model.py:47-141, base_model.py:138-160) -----------------
    def setup_optimizer(self, opt):
        """Two Adam groups, aggregator (lr) and neural points (plr), as the reference builds them."""
        from .train import PointParams
        from .train_hip import HipTrainer
        if self.neural_points is None or self.net_ray_marching is None:
            raise RuntimeError("setup_optimizer: no neural points / aggregator weights yet")
        self._sync_weights()
        npnt = self.neural_points
        params = PointParams(npnt.xyz, npnt.points_embeding, npnt.points_color, npnt.points_dir, npnt.points_conf,
                             self.device)
        g = lambda k, d: float(getattr(opt, k, d) if getattr(opt, k, None) is not None else d)  # noqa: E731
        bp = npnt.bpnet_points_embedding if self.opts.bpnet_variant[1] else None
        if self.opts.bpnet_variant[1] and bp is None:
            # SG: BPNet's embedding arrives later (neural_points.set_bpnet_feats); the trainer is
            # built by setup() / the first optimize_parameters once it is there
            self.trainer = None
            return
        # the step at the model's arithmetic: precision "f32" (the reference's) trains through the
        # fp32-faithful forward and the fp32 backward (base viewmlp and SG's block2_bpnet alike)
        prec = "f16" if self.opts.precision == "f16" else "f32"
        self.trainer = HipTrainer(params, self.net_ray_marching.renderer.mlp_state,
                                  dataclasses.replace(self.opts, is_train=1), self.device,
                                  lr=g("lr", 5e-4), plr=g("plr", 2e-3), lr_decay_exp=g("lr_decay_exp", 0.1),
                                  lr_decay_iters=g("lr_decay_iters", 1_000_000), bpnet=bp, precision=prec)
        # the renderer reads the trained tensors in place (views; the table cache follows their versions)
        n = params.xyz.shape[0]
        npnt.points_embeding = params.points_embeding.detach().view(1, n, -1)
        npnt.points_color = params.points_color.detach().view(1, n, 3)
        npnt.points_dir = params.points_dir.detach().view(1, n, 3)
        npnt.points_conf = params.points_conf.detach().view(1, n, 1)
        self.optimizers = [self.trainer.opt_net, self.trainer.opt_pts]
        self.schedulers = []
        self.loss_names = list(LOSS_NAMES)

    def init_scheduler(self, total_steps, opt):
        """iter_exponential_decay resumed at total_steps (the reference steps its schedulers that often)."""
        if getattr(self, "trainer", None) is not None:
            self.trainer.step_count = int(total_steps)
            self.trainer._set_lr()

    reset_scheduler = init_scheduler

    def clean_optimizer(self):
        self._sync_weights()
        self.trainer = None
        self.optimizers = []

    def clean_scheduler(self):
        self.schedulers = []

    def clean_optimizer_scheduler(self):
        self.clean_optimizer()
        self.clean_scheduler()

    def reset_optimizer(self, opt):
        self.clean_optimizer()
        self.setup_optimizer(opt)

    def _sync_weights(self):
        """Trained aggregator weights -> the renderer's packed blob (once per change); every point
        row brought to the optimizer's step (the row-sparse point Adam defers untouched rows)."""
        tr = getattr(self, "trainer", None)
        if tr is not None:
            tr.sync_points()
        if tr is not None and getattr(self, "_weights_dirty", False):
            self.net_ray_marching.set_aggregator_state(tr.mlp_state())
        self._weights_dirty = False

    def prune_points(self, thresh):
        """neural_points.py:520-543: keep points with conf >= thresh."""
        self._sync_weights()
        p = self.neural_points
        mask = p.points_conf[0, :, 0] >= thresh
        keep = lambda t: None if t is None or t.shape[-2 if t.dim() == 3 else 0] != mask.shape[0] else (  # noqa: E731
            t[:, mask] if t.dim() == 3 else t[mask])
        self.neural_points = NeuralPoints(p.xyz[mask], p.points_embeding[:, mask], p.points_color[:, mask],
                                          p.points_dir[:, mask], p.points_conf[:, mask], self.device,
                                          points_feats=keep(p.points_feats), points_label=keep(p.points_label),
                                          bpnet_points_embedding=keep(p.bpnet_points_embedding))
        self.net_ray_marching.neural_points = self.neural_points
        return int((~mask).sum())

    def grow_points(self, add_xyz, add_embedding, add_color, add_dir, add_conf, add_label=None, **unused):
        """neural_points.py:546-572: append points (embedding/colour/dir/conf given as [M, C]).
        Labels are appended when both sides have them (:550); points_feats is kept as it is,
        as the reference keeps it.  The BPNet embedding gets zero rows for the new points (the
        reference leaves it at the old length, which its index_select at neural_points.py:972
        would then overrun)."""
        self._sync_weights()
        p = self.neural_points
        f = lambda t, c: torch.as_tensor(t).to(self.device, torch.float32).reshape(1, -1, c)  # noqa: E731
        label = p.points_label
        bp = p.bpnet_points_embedding
        if bp is not None:
            m = torch.as_tensor(add_xyz).reshape(-1, 3).shape[0]
            bp = torch.cat([bp, bp.new_zeros(1, m, bp.shape[-1])], 1)
        if label is not None and add_label is not None:
            label = torch.cat([label, torch.as_tensor(add_label).to(label.device, label.dtype).reshape(-1, 1)], 0)
        elif label is not None:
            label = None   # the reference's cat would fail; an unlabelled tail invalidates the labels
        self.neural_points = NeuralPoints(
            torch.cat([p.xyz, f(add_xyz, 3)[0]], 0),
            torch.cat([p.points_embeding, f(add_embedding, p.points_embeding.shape[-1])], 1),
            torch.cat([p.points_color, f(add_color, 3)], 1), torch.cat([p.points_dir, f(add_dir, 3)], 1),
            torch.cat([p.points_conf, f(add_conf, 1)], 1), self.device, points_feats=p.points_feats,
            points_label=label, bpnet_points_embedding=bp)
        self.net_ray_marching.neural_points = self.neural_points
        if self.is_train and getattr(self, "trainer", None) is not None:
            self.setup_optimizer(self.opt)

    # -- per-batch surface -----------------------------------------------------------------
    def set_input(self, input):
        self.input = {k: (v.to(self.device) if torch.is_tensor(v) else v) for k, v in input.items()}
        self.gt_image = self.input.get("gt_image")

    def forward(self):
        if self.net_ray_marching is None:
            raise RuntimeError("no neural points / weights: call load_networks() or set_points() first")
        self._sync_weights()
        self.output = self.net_ray_marching.render(self.input)  # == fill_invalid(forward(input))
        for k in self.visual_names:
            setattr(self, k, self.output[k])

    def test(self):
        with torch.no_grad():
            self.forward()
        return self.output

    def get_current_visuals(self, data=None):
        return {k: getattr(self, k) for k in self.visual_names}

    def get_current_losses(self):
        return {k: getattr(self, "loss_" + k) for k in self.loss_names if hasattr(self, "loss_" + k)}

    def eval(self):
        return self

    def train(self):
        return self

    def optimize_parameters(self, backward=True, total_steps=0):
        """neural_points_volumetric_model.py:320-331: forward, losses, backward, both Adam steps."""
        if getattr(self, "trainer", None) is None:
            self.setup_optimizer(self.opt)
        if self.trainer is None:  # SG with predict_semantic: setup_optimizer waits for the embedding
            raise ValueError("optimize_parameters: the SG-NeRF aggregator (predict_semantic = 1) needs the points' "
                             "BPNet embedding first (neural_points.set_bpnet_feats / bpnet_points_embedding)")
        inp = self.input
        tr = self.trainer
        near = inp["near"] if "near" in inp else self.opts.near_plane
        far = inp["far"] if "far" in inp else self.opts.far_plane
        near, far = (float(torch.as_tensor(x).reshape(-1)[0]) for x in (near, far))
        gt = inp["gt_image"].reshape(-1, 3).to(self.device, torch.float32)
        args = (inp["campos"], inp["camrotc2w"], inp["raydir"], near, far, gt)
        labels = None
        if self.opts.semantic_guidance == 1:  # neural_points.py:771-785, as the renderer passes them
            pl = self.neural_points.points_label
            if pl is None or inp.get("pixel_label") is None:
                raise ValueError("semantic_guidance = 1 needs neural_points.points_label and inputs['pixel_label']")
            labels = (pl.reshape(-1).to(self.device, torch.int32).contiguous(),
                      torch.as_tensor(inp["pixel_label"]).reshape(-1).to(self.device, torch.int32).contiguous(),
                      inp.get("seconds"))
        tr.step_count = int(total_steps)
        # the plane background model's per-ray colour (set_bg -> inputs['bg_ray'], run/train_ft.py:209-218):
        # the loss composites T_bg * bg_ray + colour (neural_points_volumetric_model.py:175-177)
        bg_ray = inp.get("bg_ray")
        if backward:
            parts, full, ray_mask = tr.step(*args, labels=labels, bg_ray=bg_ray)
            self._weights_dirty = True
        else:
            parts, full, ray_mask = tr.backward(*args, labels=labels, bg_ray=bg_ray)
        for k, v in parts.items():
            setattr(self, "loss_" + k, v)
        self.output = {"coarse_raycolor": full[None], "ray_mask": ray_mask[None].to(torch.int8)}
        self.coarse_raycolor = self.output["coarse_raycolor"]
        self.ray_mask = self.output["ray_mask"]
        self.update_rank_ray_miss(total_steps)   # neural_points_volumetric_model.py:328-330
        return parts

    # -- probe ranking (mvs_points_volumetric_model.py:157-184) ------------------------------
    def update_rank_ray_miss(self, total_steps):
        """Rank this frame by its ray_miss_coarse_raycolor loss among the top frames the next
        probe visits (prob_num_step > 1), or keep the running maximum (prob_num_step == 1)."""
        opt = self.opt
        if getattr(self, "top_ray_miss_loss", None) is None or not hasattr(self, "loss_ray_miss_coarse_raycolor"):
            return
        ks = getattr(opt, "prob_kernel_size", None)
        tiers = getattr(opt, "prob_tiers", 250000)
        if ks is not None and np.sum(np.asarray(tiers) < total_steps) >= len(ks) // 3:
            return
        prob_freq = int(getattr(opt, "prob_freq", 0) or 0)
        nstep = int(getattr(opt, "prob_num_step", 100) or 0)
        loss = self.loss_ray_miss_coarse_raycolor.reshape(()).to(self.top_ray_miss_loss.device)
        if prob_freq > 0 and nstep > 1:
            self.top_ray_miss_loss, self.top_ray_miss_ids = self.rank_ray_miss(
                self.input["id"][0], loss, self.top_ray_miss_ids, self.top_ray_miss_loss)
        elif prob_freq > 0 and nstep == 1:
            self.top_ray_miss_loss[0] = torch.maximum(loss, self.top_ray_miss_loss[0])

    def rank_ray_miss(self, new_id, newloss, inds, losses):
        """mvs_points_volumetric_model.py:166-176: a frame already ranked keeps its largest loss,
        a new frame replaces the last entry; then sort by loss, descending.  Branch-free on the
        device (the reference's `if torch.sum(mask) > 0` is a host sync per step)."""
        with torch.no_grad():
            new_id = torch.as_tensor(new_id, device=inds.device).reshape(()).to(inds.dtype)
            newloss = torch.as_tensor(newloss, device=losses.device).reshape(()).to(losses.dtype)
            mask = inds == new_id
            hit = mask.any()
            last = torch.zeros_like(mask)
            last[-1] = True
            losses = torch.where(hit, torch.where(mask, torch.maximum(losses, newloss), losses),
                                 torch.where(last, newloss, losses))
            inds = torch.where(hit, inds, torch.where(last, new_id, inds))
            losses, order = torch.sort(losses, descending=True)
            return losses, inds[order]

    def reset_ray_miss_ranking(self):
        """mvs_points_volumetric_model.py:187-189."""
        self.top_ray_miss_loss = torch.zeros([self.num_probe + 1], dtype=torch.float32, device=self.device)
        self.top_ray_miss_ids = torch.arange(self.num_probe + 1, dtype=torch.int32, device=self.device)

    def set_bg(self, xyz_world_sect_plane, img_lst, c2ws_lst, w2cs_lst, intrinsics_all, HDWD_lst, plane_color,
               fg_masks=None, **kwargs):
        """mvs_points_volumetric_model.py:276-315 (bgmodel '*plane'): the rays' background colours from
        the source images warped onto the plane (sgnerf_amd.plane_bg).  Returns (bg_ray [1,R,3],
        fg_masks); the drivers put bg_ray into the input dict as 'bg_ray' (run/train_ft.py:209-218),
        which the renderer blends as T_bg * bg_ray."""
        from .plane_bg import plane_bg
        if self.neural_points is None:
            raise RuntimeError("set_bg: no neural points (its foreground masks project them)")
        return plane_bg(xyz_world_sect_plane, img_lst, w2cs_lst, intrinsics_all, HDWD_lst, plane_color,
                        self.neural_points.xyz, fg_masks=fg_masks)

    # -- semantic dumps (neural_points_volumetric_model.py:337-362, 674-720) ------------------
    def _semantic_dir(self):
        return os.path.join(getattr(self.opt, "checkpoints_dir", "."), getattr(self.opt, "name", "sgn"))

    def saveSemanticEmbedding(self, epoch):
        """`{epoch}_semanticEmbedding.pth`: the BPNet per-point embedding [N,96] on the CPU
        (None when BPNet never ran, as in the reference)."""
        e = self.neural_points.bpnet_points_embedding if self.neural_points is not None else None
        e = None if e is None else e.detach().reshape(e.shape[-2], e.shape[-1]).cpu()
        path = os.path.join(self._semantic_dir(), f"{epoch}_semanticEmbedding.pth")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        torch.save(e, path)
        return path

    def _save_label_points(self, path):
        p = self.neural_points
        if p is None or p.points_label is None:
            raise RuntimeError("saveSemanticPoints: no per-point labels (set_points(points_label=...) or "
                               "neural_points.set_bpnet_feats)")
        lab = p.points_label.reshape(-1).cpu().numpy()
        xyz = p.xyz.detach().cpu().numpy()
        if lab.shape[0] != xyz.shape[0]:
            raise RuntimeError(f"saveSemanticPoints: {lab.shape[0]} labels for {xyz.shape[0]} points")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        np.savetxt(path, np.concatenate([xyz.astype(np.float32), label_colours(lab)], 1), fmt="%f")
        print("savepoints:", path)
        return path

    def saveSemanticPoints(self, train_steps):
        """`predict_points_{train_steps}.txt`: x y z r g b per point, the label's colour."""
        return self._save_label_points(os.path.join(self._semantic_dir(), f"predict_points_{train_steps}.txt"))

    def saveSemanticPoints_test(self, totalIter, imgNum):
        """`test_{totalIter}/test_predict_points_iter{totalIter}_imgNum{imgNum}.txt`."""
        return self._save_label_points(os.path.join(self._semantic_dir(), f"test_{totalIter}",
                                                    f"test_predict_points_iter{totalIter}_imgNum{imgNum}.txt"))

    def update_learning_rate(self, opt=None, total_steps=None, **k):
        """Schedulers are the trainer's iter_exponential_decay, applied at every step."""
        if getattr(self, "trainer", None) is not None and total_steps is not None:
            self.init_scheduler(total_steps + 1, opt)
        return [g["lr"] for o in getattr(self, "optimizers", []) for g in o.param_groups]

    # -- checkpoints (models/base_model.py:85-119) -------------------------------------------
    def state_dict(self):
        self._sync_weights()
        sd = dict(self.neural_points.state_dict())
        for k, v in self.net_ray_marching.renderer.mlp_state.items():
            sd["aggregator." + k] = v
        return sd

    def save_networks(self, epoch, other_states={}, back_gpu=True):
        os.makedirs(self.save_dir, exist_ok=True)
        sd = {k: v.detach().cpu() for k, v in self.state_dict().items()}
        torch.save(sd, os.path.join(self.save_dir, f"{epoch}_net_ray_marching.pth"))
        torch.save(dict(other_states), os.path.join(self.save_dir, f"{epoch}_states.pth"))

    def load_networks(self, epoch, directory=None):
        directory = directory or getattr(self.opt, "resume_dir", None) or self.save_dir
        path = os.path.join(directory, f"{epoch}_net_ray_marching.pth")
        sd = torch.load(path, map_location="cpu", weights_only=True)
        self.neural_points = NeuralPoints.from_state_dict(sd, self.device)
        self.net_ray_marching = NeuralPointsRayMarching(self.neural_points, strip_prefix(sd), self.opts, self.device)
        return path
