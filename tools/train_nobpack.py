"""Experiment (NOT product): bench.py --train with the rows-mode GEMMs' weight images (bpack) switched off,
so the rows kernels convert their weight block in every workgroup.  Same-box A/B against a plain
`python bench.py --train ...` run.  Usage: python tools/train_nobpack.py <bench.py args>"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import sgnerf_amd.train_f32 as tf  # noqa: E402


def _no_bpack(gemms, device):
    for g in gemms:
        g.bpack = None
    return torch.empty(16, dtype=torch.uint8, device=device)


tf._attach_bpack = _no_bpack
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
