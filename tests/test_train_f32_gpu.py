"""GPU unit tests of the fp32 training step's kernels (csrc/train_x3.hip) through the C ABI:
sgn_x3_gemm in both modes against float64 torch on the same fp32 operands, the deterministic
work list / compact row offsets of sgn_train_lists, and the fixed-order partial reduction."""
import ctypes

import pytest
import torch

import sgnerf_amd  # noqa: F401
from sgnerf_amd import _lib
from sgnerf_amd.train_f32 import _operand, _rows_gemm, _splitk_gemm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
# the 3-product split carries 22 significant bits per factor with fp32 accumulation: every output
# within a few fp32 ulps of sum |a b| (relative to the output's scale), the bar the f32 mode holds
REL = 2e-6


def _gemm(g):
    _lib.check(_lib.lib().sgn_x3_gemm(ctypes.byref(g), _lib.stream_handle()), "sgn_x3_gemm")


def _gemm_both(g, outs, amax=None):
    """sgn_x3_gemm in rows mode with the in-workgroup weight conversion, then with the weight images
    (bpack, ABI 13) into re-filled outputs: bit-identical results (the same split of the same values)."""
    _gemm(g)
    first = [o.clone() for o in outs]
    am = amax.clone() if amax is not None else None
    nb = int(_lib.lib().sgn_x3_gemm_bpack_bytes(ctypes.byref(g)))
    assert nb > 0
    ws = torch.full((nb // 4 + 4,), float("nan"), device=DEV)
    g2 = type(g).from_buffer_copy(g)
    g2.bpack = ws.data_ptr()
    for o in outs:
        o.fill_(-5.0)
    if amax is not None:
        amax.zero_()
    _gemm(g2)
    torch.cuda.synchronize()
    for a, b in zip(first, outs):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    if amax is not None:
        assert torch.equal(am, amax)


def _rel(x, ref):
    return float((x.double() - ref).abs().max() / ref.abs().max().clamp(min=1e-30))


def _lrelu(x):
    return torch.where(x > 0, x, x * 0.01)


@pytest.mark.parametrize("scale", [1.0, 1e-7, 3e3])
def test_x3_gemm_rows_mode_matches_float64(scale):
    """Y = (dY W) * LReLU'(mask) with a bias / column split, and X W^T + b with LeakyReLU on the
    operand and the output: rows beyond the device count untouched, the amax word written."""
    g = torch.Generator().manual_seed(1)
    rows_cap, rows, K, N = 700, 613, 256, 263
    dy = (torch.randn(rows_cap, K, generator=g) * scale).to(DEV)
    W = (torch.randn(K, N, generator=g) * 0.06).to(DEV)          # [K][N] row-major: the NN (kmajor) form
    mask = torch.randn(rows_cap, 256, generator=g).to(DEV)
    shift = torch.tensor([14 - int(torch.frexp(W.abs().max().cpu())[1])], dtype=torch.int32, device=DEV)
    amax_in = torch.tensor([dy[:rows].abs().max().item()], dtype=torch.float32, device=DEV).view(torch.int32)
    nrows = torch.tensor([rows], dtype=torch.int32, device=DEV)
    out = torch.full((rows_cap, 256), -5.0, device=DEV)
    out2 = torch.full((rows_cap, 8), -5.0, device=DEV)
    amax = torch.zeros(2, dtype=torch.int32, device=DEV)
    a = _operand(dy.data_ptr(), K, K, 0, amax=amax_in.data_ptr())
    b = _operand(W.data_ptr(), N, N, 1, shift=shift.data_ptr())
    _gemm_both(_rows_gemm(a, b, rows_cap, N, K, nrows.data_ptr(), out.data_ptr(), 256, mask=mask.data_ptr(), ldm=256,
                          out_cols=256, out2=out2.data_ptr(), ldo2=8, amax_out=amax.data_ptr(),
                          amax_out2=amax[1:].data_ptr()), [out, out2], amax)
    torch.cuda.synchronize()
    ref = dy[:rows].double() @ W.double()
    ref1 = torch.where(mask[:rows] > 0, ref[:, :256], ref[:, :256] * 0.01)
    assert _rel(out[:rows], ref1) < REL
    assert _rel(out2[:rows, :7], ref[:, 256:263]) < REL
    assert bool((out[rows:] == -5.0).all()) and bool((out2[:, 7:] == -5.0).all())
    assert abs(amax[:1].view(torch.float32).item() - out[:rows].abs().max().item()) == 0.0
    # forward form: LReLU(LReLU(x) W^T + b), x with a second source past column 256
    Wf = (torch.randn(128, 280, generator=g) * 0.05).to(DEV)
    bf = torch.randn(128, generator=g).to(DEV)
    x1 = (torch.randn(rows_cap, 256, generator=g) * scale).to(DEV)
    x2 = torch.randn(rows_cap, 32, generator=g).to(DEV)
    sf = torch.tensor([14 - int(torch.frexp(Wf.abs().max().cpu())[1])], dtype=torch.int32, device=DEV)
    y = torch.full((rows_cap, 128), -5.0, device=DEV)
    _gemm_both(_rows_gemm(_operand(x1.data_ptr(), 256, 280, 0, p2=x2.data_ptr(), ld2=32, csplit=256, act=1),
                          _operand(Wf.data_ptr(), 280, 280, 0, shift=sf.data_ptr()), rows_cap, 128, 280, nrows.data_ptr(),
                          y.data_ptr(), 128, bias=bf.data_ptr(), act=1), [y])
    torch.cuda.synchronize()
    xin = torch.cat([_lrelu(x1[:rows].double()), x2[:rows, :24].double()], 1)
    reff = _lrelu(xin @ Wf.double().t() + bf.double())
    assert _rel(y[:rows], reff) < REL
    assert bool((y[rows:] == -5.0).all())


@pytest.mark.parametrize("rows,splits", [(0, 8), (31, 8), (5000, 64), (20011, 128)])
def test_x3_gemm_splitk_mode_matches_float64(rows, splits):
    """dW = dY^T [LReLU(z) | ext | 1] as split-K partials, reduced in order into a flat gradient
    (sgn_reduce_partials): weights, the bias through the ones column, nothing else touched."""
    g = torch.Generator().manual_seed(2)
    cap, M = 20480, 256
    dy = (torch.randn(cap, M, generator=g) * 1e-5).to(DEV)
    z = torch.randn(cap, 256, generator=g).to(DEV)
    ext = torch.randn(cap, 8, generator=g).to(DEV)
    ext[:, 7] = 1.0
    nrows = torch.tensor([rows], dtype=torch.int32, device=DEV)
    amax_in = torch.tensor([max(dy[:rows].abs().max().item(), 1e-30) if rows else 0.0], device=DEV).view(torch.int32)
    N = 264
    part = torch.full((splits, M, N), float("nan"), device=DEV)
    _gemm(_splitk_gemm(_operand(dy.data_ptr(), 256, 256, 1, amax=amax_in.data_ptr()),
                       _operand(z.data_ptr(), 256, 264, 1, p2=ext.data_ptr(), ld2=8, csplit=256, act=1),
                       M, N, cap, nrows.data_ptr(), part.data_ptr(), splits))
    flat = torch.zeros(M * 263 + M + 5, device=DEV)
    seg = _lib.PartialSegment()
    seg.part, seg.splits, seg.M, seg.N, seg.n_in, seg.bias_col, seg.ldw = part.data_ptr(), splits, M, N, 263, 263, 263
    seg.dst_w, seg.dst_b = flat.data_ptr(), flat.data_ptr() + 4 * M * 263
    _lib.check(_lib.lib().sgn_reduce_partials(1, ctypes.byref(seg), _lib.stream_handle()), "sgn_reduce_partials")
    torch.cuda.synchronize()
    x = torch.cat([_lrelu(z[:rows].double()), ext[:rows, :7].double()], 1)
    refw = dy[:rows].double().t() @ x
    refb = dy[:rows].double().sum(0)
    if rows == 0:
        assert bool((flat == 0).all())
        return
    assert _rel(flat[:M * 263].view(M, 263), refw) < REL
    assert _rel(flat[M * 263:M * 264], refb) < REL
    assert bool((flat[M * 264:] == 0).all())


def test_train_lists_deterministic_order():
    """sgn_train_lists: the samples with neighbours in ascending order, compact row offsets = the
    exclusive prefix sum of samp_nnb, totals, feat cleared for s < S (over several blocks)."""
    g = torch.Generator().manual_seed(3)
    cap, S = 5000, 4321
    nnb = torch.randint(0, 9, (cap,), generator=g, dtype=torch.int32)
    nnb[torch.rand(cap, generator=g) < 0.3] = 0
    counters = torch.tensor([S, int((nnb[:S] > 0).sum()), 0, 0], dtype=torch.int32, device=DEV)
    work = torch.full((cap,), -1, dtype=torch.int32, device=DEV)
    row_off = torch.full((cap,), -1, dtype=torch.int32, device=DEV)
    feat = torch.full((cap, 4), 3.0, device=DEV)
    counts = torch.zeros(4, dtype=torch.int32, device=DEV)
    L = _lib.lib()
    ws = torch.empty(int(L.sgn_train_lists_workspace_bytes(cap)), dtype=torch.uint8, device=DEV)
    nd = nnb.to(DEV)
    _lib.check(L.sgn_train_lists(_lib.ptr(counters), _lib.ptr(nd), cap, _lib.ptr(work), _lib.ptr(row_off),
                                 _lib.ptr(feat), _lib.ptr(counts), _lib.ptr(ws), _lib.stream_handle()), "sgn_train_lists")
    torch.cuda.synchronize()
    items = torch.nonzero(nnb[:S] > 0).reshape(-1).to(torch.int32)
    assert int(counts[0]) == items.numel() and int(counts[1]) == int(nnb[:S].sum())
    assert torch.equal(work[:items.numel()].cpu(), items)
    exp_off = torch.cumsum(nnb[:S], 0) - nnb[:S]
    assert torch.equal(row_off[:S].cpu(), exp_off.to(torch.int32))
    assert bool((feat[:S] == 0).all()) and bool((feat[S:] == 3.0).all())
