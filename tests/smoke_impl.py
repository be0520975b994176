"""__graft_entry__.smoke(): one small query on cuda:0 checked against the oracle."""
import numpy as np
import torch


def run_smoke():
    import oracle_query as oq
    from helpers import hyper_for, make_view, opts, small_room, t_table
    from sgnerf_amd.querier import HipGrid, QueryWorkspace, run_query

    assert torch.cuda.is_available(), "smoke() needs the GPU"
    dev = "cuda:0"
    pc = small_room(100_000)
    o = opts()
    hy = hyper_for(pc, o)
    view = make_view(24, 32)
    g = HipGrid(torch.from_numpy(pc.xyz).to(dev), o, hyper=hy)
    t = t_table(o)
    ws = QueryWorkspace(view.raydir.shape[0], o.SR, o.K, dev, dense=True)
    res = run_query(g, o, torch.from_numpy(view.campos).to(dev), torch.from_numpy(view.raydir).to(dev),
                    t.to(dev), 0, ws, dense=True)
    R = view.raydir.shape[0]
    pidx = res.pidx[: R * o.SR * o.K].view(R, o.SR, o.K).cpu().numpy()
    ref = oq.OracleGrid(pc.xyz, hy, o).query(view.campos, view.raydir, t.numpy())
    assert np.array_equal(pidx, ref["pidx"]), "smoke: neighbour indices differ from the oracle"
    assert (pidx >= 0).sum() > 0
    print(f"smoke OK: {R} rays, {int((pidx >= 0).sum())} neighbour indices bit-exact")

    # full hot path through the reference operator API (query -> MFMA aggregator ->
    # composite) against the oracle's torch restatement
    import agg_ref
    from sgnerf_amd.ray_marching import NeuralPoints, NeuralPointsRayMarching
    from sgnerf_amd.weights import init_mlp
    mlp = init_mlp(0, bias_std=0.01)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 100.0
    net = NeuralPointsRayMarching(NeuralPoints.from_cloud(pc, dev), mlp, o, dev)
    d = lambda a: torch.from_numpy(a).to(dev)[None]  # noqa: E731
    out = net.render({"campos": d(view.campos), "raydir": d(view.raydir), "camrotc2w": d(view.camrotc2w),
                      "near": 0.1, "far": 8.0})
    qs = oq.OracleGrid(pc.xyz, hy, o).query(view.campos, view.raydir, t.numpy())
    tp = {k: torch.from_numpy(getattr(pc, k)) for k in ("xyz", "embedding", "color", "dir", "conf")}
    with torch.no_grad():
        full, mask, _, _, _ = agg_ref.render(tp, mlp, torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w),
                                             torch.from_numpy(view.raydir), qs, o.SR)
    rgb = out["coarse_raycolor"][0].cpu()
    assert torch.equal(out["ray_mask"][0].cpu().bool(), mask), "smoke: ray_mask differs from the oracle"
    err = float((rgb - full).abs().max())
    assert err <= 1e-3, f"smoke: rgb differs from the oracle by {err:.3e}"
    print(f"smoke OK: rendered {R} rays, {int(mask.sum())} valid, max |rgb - oracle| = {err:.2e}")
