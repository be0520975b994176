"""Model plugin for the reference's driver scripts (run/test_ft.py, run/render_vid.py).

The reference finds `models.<name>_model.<Name>Model` (models/__init__.py:5-27) and
drives it through the BaseModel surface (models/base_model.py:7-142,
models/base_rendering_model.py:387-533).  HipPointsVolumetricModel exposes that
surface for inference over the HIP hot path; INTEGRATION.md shows the three-line
shim `models/hip_points_volumetric_model.py` a maintainer adds to the reference.

Checkpoints use the reference layout: `{epoch}_net_ray_marching.pth` holding
`neural_points.{xyz,points_embeding,points_color,points_dir,points_conf}` and
`aggregator.*` (models/base_model.py:85-119), loaded with
torch.load(weights_only=True).  Training (optimize_parameters and friends) is
SURVEY.md §8 row f1 and raises NotImplementedError until it lands.
"""
import os

import torch

from .opts import HotPathOpts
from .ray_marching import NeuralPoints, NeuralPointsRayMarching
from .weights import strip_prefix


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
        self.opts = HotPathOpts.from_opt(opt, **extra).check_supported()
        self.model_names = ["ray_marching"]
        self.visual_names = ["coarse_raycolor", "ray_mask", "coarse_is_background"]
        self.loss_names = []
        self.neural_points = None
        self.net_ray_marching = None
        self.output = {}

    def setup(self, opt, train_len=None):
        if self.is_train:
            raise NotImplementedError("training on the HIP path is SURVEY.md §8 row f1 (not built yet)")
        resume = getattr(opt, "resume_iter", None)
        if resume is not None and getattr(opt, "resume_dir", None):
            self.load_networks(resume)

    def set_points(self, xyz, points_embeding, points_conf=None, points_dir=None, points_color=None,
                   aggregator_state=None, Rw2c=None, **unused):
        """neural_points.py:520-572; also takes the aggregator weights when no checkpoint is loaded."""
        self.neural_points = NeuralPoints(xyz, points_embeding, points_color, points_dir, points_conf, self.device)
        if aggregator_state is not None or self.net_ray_marching is None:
            if aggregator_state is None:
                raise ValueError("set_points: aggregator_state required before the first render")
            self.net_ray_marching = NeuralPointsRayMarching(self.neural_points, aggregator_state, self.opts,
                                                            self.device)
        else:
            self.net_ray_marching.neural_points = self.neural_points

    # -- per-batch surface -----------------------------------------------------------------
    def set_input(self, input):
        self.input = {k: (v.to(self.device) if torch.is_tensor(v) else v) for k, v in input.items()}
        self.gt_image = self.input.get("gt_image")

    def forward(self):
        if self.net_ray_marching is None:
            raise RuntimeError("no neural points / weights: call load_networks() or set_points() first")
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
        return {}

    def eval(self):
        return self

    def train(self):
        raise NotImplementedError("training on the HIP path is SURVEY.md §8 row f1 (not built yet)")

    def optimize_parameters(self, *a, **k):
        raise NotImplementedError("training on the HIP path is SURVEY.md §8 row f1 (not built yet)")

    def update_learning_rate(self, *a, **k):
        raise NotImplementedError("training on the HIP path is SURVEY.md §8 row f1 (not built yet)")

    # -- checkpoints (models/base_model.py:85-119) -------------------------------------------
    def state_dict(self):
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
