"""Debug probe (not product): run the fp32 training step's forward on one config-5 batch (no
jitter) repeatedly and report which buffers differ from the first run (bitwise)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import sgnerf_amd  # noqa: E402,F401
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.train import PointParams  # noqa: E402
from sgnerf_amd.train_hip import HipTrainer  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

DEV = torch.device("cuda", 0)
O = HotPathOpts(SR=24)
pc = scene.synth_room(1_200_000, seed=0)
yaw, pitch = scene.spiral_yaw_pitch(37, 120)
view = scene.room_view(800, 800, yaw=yaw + 15.0, pitch=pitch - 5.0)
g = torch.Generator().manual_seed(2)
idx = torch.randint(0, 800 * 800, (4096,), generator=g).numpy()
raydir = torch.from_numpy(np.ascontiguousarray(view.raydir[idx])).to(DEV)
gt = torch.rand(4096, 3, generator=g).to(DEV)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
campos, rot = torch.from_numpy(view.campos).to(DEV), torch.from_numpy(view.camrotc2w).to(DEV)
points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
tr = HipTrainer(points, mlp, O, DEV, precision="f32")
first = None
n_runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
for it in range(n_runs):
    parts, full, mask = tr.backward(campos, rot, raydir, 0.1, 8.0, gt)
    torch.cuda.synchronize()
    st = tr._f32step
    n, rows = [int(x) for x in st.counts[:2].tolist()]
    S = int(st.q.counters[0])
    ws = st.ws32
    ws_items = (ws.numel() - 2048) // (1024 + 48)
    rows_t = ws[ws_items * 1024:ws_items * 1024 + ws_items * 32].view(torch.int32).view(-1, 8)
    slots_t = ws[ws_items * 1056:ws_items * 1056 + ws_items * 16].view(torch.int32).view(-1, 4)
    nslot = int(ws[ws_items * 1072:ws_items * 1072 + 4].view(torch.int32)[0])
    snap = {"rows_tab": rows_t[:nslot].clone(), "slots_tab": slots_t[:nslot].clone(), "full": full.clone(), "feat": st.feat[:S].clone(), "fs": st.fs[:n].clone(), "h3": st.h[2][:n].clone(),
            "z1": st.z[0][:rows].clone(), "z3": st.z[2][:rows].clone(), "work": st.q.work[:n].clone(),
            "pidx": st.q.pidx[:S * 8].clone(), "grad": tr.mlp.flat.grad.clone(),
            "g_emb": points.points_embeding.grad.clone()}
    if first is None:
        first = snap
        print("run 0: S", S, "items", n, "rows", rows, flush=True)
        continue
    diff = {k: float((v.double() - first[k].double()).abs().max()) for k, v in snap.items()
            if k not in ("rows_tab", "slots_tab")}
    bad = {k: v for k, v in diff.items() if v != 0.0}
    print(f"run {it}: differs in {bad}" if bad else f"run {it}: identical", flush=True)
    if "feat" in bad:
        dd = (snap["feat"] - first["feat"]).abs().max(1).values
        ss = torch.nonzero(dd).reshape(-1)
        print("  samples differing:", ss.numel(), ss[:10].tolist(), "items?",
              [int((first["work"] == s).any()) for s in ss[:10].tolist()])
        for s in ss[:4].tolist():
            print("   ", s, first["feat"][s].tolist(), snap["feat"][s].tolist())
            for tag, sn in (("good", first), ("bad", snap)):
                hit = torch.nonzero(((sn["rows_tab"] >> 3) == s).any(1)).reshape(-1).tolist()
                for sl in hit:
                    t0 = sl // 8 * 8
                    print(f"      {tag}: slot {sl} (tile {sl // 8}, wave {(sl % 8) // 2}, half {sl % 2}) rows "
                          f"{sn['rows_tab'][sl].tolist()} entry {[hex(x & 0xffffffff) for x in sn['slots_tab'][sl].tolist()]}")
                    print(f"        tile rows: {[[(v >> 3, v & 7) if v >= 0 else -1 for v in sn['rows_tab'][t].tolist()] for t in range(t0, min(t0 + 8, sn['rows_tab'].shape[0]))]}")
