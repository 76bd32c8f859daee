"""world_size-2 gloo tests on CPU for the multi-GPU coordination: the timed
region's barrier + max-over-ranks timing used by bench.py, and the shard arithmetic."""
import os
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import time
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.02 * (rank + 1))  # rank 1 is the slow one

    el = bench.timed_region(step, steps=3, warmup=1, sync=lambda: None, dist=dist)
    q.put((rank, el, len(calls)))
    dist.destroy_process_group()


def test_timed_region_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (_, e0, c0), (_, e1, c1) = res
    assert c0 == c1 == 4                    # warmup + exactly K timed steps
    assert e0 == e1                          # every rank reports the same (max) time
    assert e0 >= 3 * 0.04                    # dominated by the slow rank


def test_shard_ranges(sdr):
    from sdrgpu.shard import channel_range, time_range
    for nch, world in [(8192, 8), (1024, 3), (5, 8)]:
        rs = [channel_range(nch, world, r) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == nch
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    for n, world, align in [(1 << 28, 8, 4), (1000, 3, 4)]:
        rs = [time_range(n, world, r, align) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(lo % align == 0 for lo, _ in rs)


def test_launch_ranks_spawns_world(capsys):
    """`bench.py --gpus N` without torchrun starts N rank processes itself (the driver's
    N-GPU invocation shape) and relays rank 0's JSON line."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    probe = os.path.join(ROOT, "tests", "_rank_probe.py")
    rc = bench.launch_ranks(3, ["--steps", "2"], script=probe, timeout=120)
    out = capsys.readouterr().out.strip().splitlines()[-1]
    d = json.loads(out)
    assert rc == 0 and d["world"] == 3
    assert sorted(r["rank"] for r in d["ranks"]) == [0, 1, 2]
    assert [r["local"] for r in sorted(d["ranks"], key=lambda r: r["rank"])] == [0, 1, 2]
    assert all(r["argv"] == ["--steps", "2"] for r in d["ranks"])
    assert len({r["el"] for r in d["ranks"]}) == 1   # max-over-ranks time on every rank


def test_launch_ranks_propagates_failure(capsys):
    sys.path.insert(0, ROOT)
    import bench
    probe = os.path.join(ROOT, "tests", "_rank_probe.py")
    os.environ["PROBE_EXIT_RANK"] = "1"
    try:
        rc = bench.launch_ranks(2, [], script=probe, timeout=120)
    finally:
        del os.environ["PROBE_EXIT_RANK"]
    assert rc == 3


def test_launch_ranks_kills_blocked_ranks_when_one_dies_early(capsys):
    """A rank that exits before the rendezvous leaves the others waiting in it: the launcher
    kills them and returns the dead rank's status instead of hanging (advisor finding)."""
    sys.path.insert(0, ROOT)
    import time
    import bench
    probe = os.path.join(ROOT, "tests", "_rank_probe.py")
    os.environ["PROBE_DIE_EARLY_RANK"] = "1"
    try:
        t0 = time.monotonic()
        rc = bench.launch_ranks(3, [], script=probe, timeout=120)
        el = time.monotonic() - t0
    finally:
        del os.environ["PROBE_DIE_EARLY_RANK"]
    assert rc == 5 and el < 60


def test_launch_ranks_timeout_kills_all(capsys):
    sys.path.insert(0, ROOT)
    import bench
    probe = os.path.join(ROOT, "tests", "_rank_probe.py")
    os.environ["PROBE_DIE_EARLY_RANK"] = "1"   # ranks 0 and 2 then wait for rank 1 forever
    try:
        rc = bench.launch_ranks(3, [], script=probe, timeout=0.5)
    finally:
        del os.environ["PROBE_DIE_EARLY_RANK"]
    assert rc in (5, 124)


def test_bench_rejects_world_mismatch():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
