"""Rank script for tests/test_dist_cpu.py::test_launch_ranks_gloo (not a test module): every
rank joins a gloo group from the torch.distributed.run environment, all-reduces rank + 1 and
rank 0 prints one JSON line, the way bench.py reports under its own launcher."""
import json
import os
import sys

import torch
import torch.distributed as dist

if __name__ == "__main__":
    dist.init_process_group("gloo")
    x = torch.tensor([float(dist.get_rank() + 1)])
    dist.all_reduce(x)
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), "sum": float(x), "argv": sys.argv[1:],
                          "master": os.environ.get("MASTER_ADDR")}), flush=True)
    dist.destroy_process_group()
