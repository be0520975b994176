"""GPU test of sgn_f16_weight_grad (csrc/dw_f16.hip), the f16 training step's row-layer weight
and bias gradients: split-K partials of d^T x over fp16 rows against float64 torch on the same fp16 values, at
the step's column counts (256, 272, 288, SG's 352), ragged row counts and empty runs."""
import pytest
import torch

import sgnerf_amd  # noqa: F401
from sgnerf_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("ncols,rows,splits", [(256, 0, 8), (256, 31, 128), (272, 5000, 85), (288, 20011, 85),
                                               (352, 147456, 85), (256, 147000, 128)])
def test_f16_weight_grad_matches_float64(ncols, rows, splits):
    g = torch.Generator().manual_seed(ncols + rows)
    cap = max(rows, 1) + 77   # rows past n_rows hold garbage the kernel must not read
    d = (torch.randn(cap, 256, generator=g) * 3).to(torch.float16).to(DEV)
    x = torch.randn(cap, ncols, generator=g).to(torch.float16).to(DEV)
    d[rows:] = float("nan")
    x[rows:] = float("nan")
    part = torch.full((splits, 256, ncols), float("nan"), device=DEV)
    pb = torch.full((splits, 256), float("nan"), device=DEV)
    _lib.check(_lib.lib().sgn_f16_weight_grad(_lib.ptr(d), 256, _lib.ptr(x), ncols, ncols, rows, splits,
                                              _lib.ptr(part), _lib.ptr(pb), _lib.stream_handle()), "sgn_f16_weight_grad")
    torch.cuda.synchronize()
    assert bool(torch.isfinite(part).all()) and bool(torch.isfinite(pb).all())
    # the bias partials: column sums of d (fp32 accumulation of exact fp16 values)
    refb = d[:rows].double().sum(0)
    magb = d[:rows].double().abs().sum(0)
    assert float(((pb.double().sum(0) - refb).abs() / magb.clamp(min=1e-30)).max()) < 3e-5
    ref = d[:rows].double().t() @ x[:rows].double()
    got = part.double().sum(0)
    if rows == 0:
        assert bool((part == 0).all())
        return
    # exact fp16 products, fp32 accumulation over a run's rows (<= 1760 here: n u <= 1.1e-4 at worst, a
    # random walk's ~1e-6 typically), then the runs summed in float64: relative to sum |d x|
    mag = d[:rows].double().abs().t() @ x[:rows].double().abs()
    assert float(((got - ref).abs() / mag.clamp(min=1e-30)).max()) < 3e-5
    # the runs are the fixed 32-aligned row ranges: run s holds exactly its rows' sum
    per = ((rows + splits - 1) // splits + 31) // 32 * 32
    s = min(rows // per, splits - 1) if per else 0
    r0, r1 = s * per, min(rows, (s + 1) * per)
    if r1 > r0:
        refs = d[r0:r1].double().t() @ x[r0:r1].double()
        mags = d[r0:r1].double().abs().t() @ x[r0:r1].double().abs()
        assert float(((part[s].double() - refs).abs() / mags.clamp(min=1e-30)).max()) < 3e-5
