"""Helper for test_dist_cpu.py: a rank process as bench.launch_ranks starts it (gloo only,
no GPU).  Rank 0 prints one JSON line with what every rank saw."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if os.environ.get("PROBE_DIE_EARLY_RANK") == os.environ["RANK"]:
    sys.exit(5)          # dies before the rendezvous: the other ranks would block in it
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
el = bench.timed_region(lambda: None, steps=2, warmup=1, sync=lambda: None, dist=dist)
seen = [None] * world
dist.all_gather_object(seen, {"rank": rank, "local": int(os.environ["LOCAL_RANK"]),
                              "argv": sys.argv[1:], "el": el})
if rank == 0:
    print(json.dumps({"world": world, "ranks": seen}), flush=True)
dist.destroy_process_group()
sys.exit(int(os.environ.get("PROBE_EXIT_RANK", "-1")) == rank and 3 or 0)
