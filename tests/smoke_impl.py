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
