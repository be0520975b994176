"""The training losses on the HIP loss stage (csrc/loss.hip, sgn_loss_train).

`LossStage(...)` has the signature and results of train.composite_losses (ray_dist +
ray_march + fill_invalid + ray_masked_coarse_raycolor + zero_one_loss on conf_coefficient, with
ray_miss / coarse colour logged; neural_points_volumetric_model.py:569-631,
diff_ray_marching.py:509-555, base_rendering_model.py:534-664, mvs_points_volumetric_model.py:607-614)
but runs as three HIP launches that compute the losses AND their gradients w.r.t. the per-sample
features and the points' conf in one pass, with no host synchronisation (graph-capturable).
Autograd sees one node: its backward scales the kernel's gradients by the incoming ones.
"""
import ctypes

import torch

from . import _lib
from .opts import HotPathOpts

_N_LOSS = 8


class _HipLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, conf, run):
        losses, full, mask, dfeat, dconf = run(feat, conf)
        ctx.save_for_backward(dfeat, dconf)
        ctx.mark_non_differentiable(full, mask)
        return losses, full, mask

    @staticmethod
    def backward(ctx, g_losses, g_full, g_mask):
        dfeat, dconf = ctx.saved_tensors
        # losses[0] = ray_masked_coarse_raycolor (d/d feat in dfeat), losses[1] = zero-one (d/d conf in dconf)
        return dfeat * g_losses[0], dconf * g_losses[1], None


class LossStage:
    """The loss stage with its reusable workspace."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._key = None

    def _buffers(self, R, SR):
        """The workspace grows, never moves to a smaller one (a captured graph keeps the pointer it
        was captured with: HipTrainer gives every captured loss stage its own LossStage)."""
        need = max(int(_lib.lib().sgn_loss_workspace_bytes(R, SR)), 16)
        if self._key is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
            self._key = (R, SR)
        return self.ws

    def __call__(self, points, q_abi, feat, campos, rot, gt, opts: HotPathOpts, R, bg=(1.0, 1.0, 1.0),
                 zero_one_weight=1e-4, zero_eps=1e-3, bg_ray=None):
        """feat [S_cap, 4] fp32 per sample (alpha, r, g, b; zeros for samples without neighbours),
        q_abi: the query's sgn_query_out; bg_ray: the rays' background [R, 3] (device, replaces bg).
        Returns (total, parts, full [R, 3], ray_mask [R] bool) as train.composite_losses."""
        dev = self.device
        conf = points.points_conf
        n_points = conf.shape[0]
        feat = feat.contiguous()
        if feat.shape[0] == 0:   # a batch without samples: one zero row keeps the pointers valid
            feat = torch.cat([feat, feat.new_zeros(1, 4)])
        ws = self._buffers(R, opts.SR)
        campos = campos.reshape(3).to(dev, torch.float32).contiguous()
        rot = rot.reshape(3, 3).to(dev, torch.float32).contiguous()
        gt = gt.reshape(-1, 3).to(dev, torch.float32).contiguous()
        lp = _lib.LossParams()
        lp.SR, lp.K = opts.SR, opts.K
        lp.vsize_z, lp.raydist_mode_unit = float(opts.vsize[2]), int(opts.raydist_mode_unit)
        for i in range(3):
            lp.bg[i] = float(bg[i])
        lp.zero_one_weight, lp.zero_one_eps = 1.0, float(zero_eps)   # dconf = d zero-one / d conf
        if bg_ray is not None:
            bg_ray = bg_ray.reshape(R, 3).to(dev, torch.float32).contiguous()
            lp.bg_ray = bg_ray.data_ptr()

        def run(feat_t, conf_t):
            losses = torch.empty(_N_LOSS, dtype=torch.float32, device=dev)
            full = torch.empty(R, 3, dtype=torch.float32, device=dev)
            mask = torch.empty(R, dtype=torch.int8, device=dev)
            dfeat = torch.zeros_like(feat_t)   # entries past the rays' samples (capacity padding) stay 0
            dconf = torch.zeros(n_points, dtype=torch.float32, device=dev)
            _lib.check(_lib.lib().sgn_loss_train(ctypes.byref(lp), _lib.ptr(campos), _lib.ptr(rot), R,
                                                 ctypes.byref(q_abi), _lib.ptr(feat_t.detach()), _lib.ptr(gt),
                                                 _lib.ptr(conf_t.detach()), _lib.ptr(full), _lib.ptr(mask),
                                                 _lib.ptr(losses), _lib.ptr(dfeat), _lib.ptr(dconf), _lib.ptr(ws),
                                                 ws.numel(), _lib.stream_handle()), "sgn_loss_train")
            return losses, full, mask, dfeat, dconf.view(conf_t.shape)

        losses, full, mask = _HipLoss.apply(feat, conf, run)
        l_col, l_zo = losses[0], losses[1]
        total = l_col + 3e-6 + zero_one_weight * l_zo
        parts = {"ray_masked_coarse_raycolor": l_col.detach(), "ray_miss_coarse_raycolor": losses[2].detach(),
                 "coarse_raycolor": losses[3].detach(), "conf_coefficient": l_zo.detach()}
        return total, parts, full, mask.bool()
