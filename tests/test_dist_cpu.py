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


@pytest.mark.parametrize("nch,world", [(8192, 8), (8192, 3), (1024, 3), (5, 8), (1, 4)])
def test_channel_range_uneven_and_empty(sdr, nch, world):
    """Balanced split: sizes differ by at most one, the first ranks take the remainder, and
    with nch < world the last ranks get an empty block (5 channels over 8 ranks)."""
    from sdrgpu.shard import channel_range
    sizes = [b - a for a, b in (channel_range(nch, world, r) for r in range(world))]
    assert sum(sizes) == nch and max(sizes) - min(sizes) <= 1
    assert sizes == sorted(sizes, reverse=True)
    if nch < world:
        assert sizes.count(0) == world - nch


@pytest.mark.parametrize("nch,world", [(8192, 8), (8192, 3), (5, 8), (1, 4), (3, 2)])
@pytest.mark.parametrize("root", ["first", "last"])
@pytest.mark.parametrize("gather", [False, True], ids=["scatterv", "gatherv"])
def test_comm_plan_v_splits(sdr, nch, world, root, gather):
    """sdrgpu_comm_plan_v -- the ops sdrgpu_comm_scatterv / gatherv issue (abi_comm.cpp) --
    for uneven and zero-channel ranks, on every rank: each non-empty rank pairs one op with
    the root at its displacement, an empty rank takes part in nothing, and the root's blocks
    tile its packed buffer exactly (no gap, no overlap)."""
    sys.path.insert(0, ROOT)
    import bench
    from sdrgpu.shard import COPY, RECV, SEND, channel_range, counts_displs, plan_v
    n = 1 << 10
    root = 0 if root == "first" else world - 1
    sizes = bench.channel_block_bytes(nch, world, n)
    _, displs = counts_displs(sizes)
    plans = [plan_v(world, r, root, gather, sizes) for r in range(world)]
    mine, theirs = (RECV, SEND) if gather else (SEND, RECV)
    for r in range(world):
        if r == root:
            continue
        if sizes[r] == 0:
            assert plans[r] == [], (r, plans[r])   # the empty-rank path: no send / recv
            continue
        assert plans[r] == [(theirs, root, 0, sizes[r])]
        assert (mine, r, displs[r], sizes[r]) in plans[root]
    spans = sorted((off, off + nb) for k, p, off, nb in plans[root])
    assert all(nb > 0 for *_, nb in plans[root])
    assert len(plans[root]) == sum(1 for v in sizes if v)
    assert [k for k, p, *_ in plans[root] if p == root] == ([COPY] if sizes[root] else [])
    assert spans[0][0] == 0 and spans[-1][1] == sum(sizes)
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    # bench.py's post-gather spot check reads channel c at channel_offset_bytes(c, n): that
    # must be inside rank r's block at its scatterv displacement
    for r in range(world):
        lo, hi = channel_range(nch, world, r)
        for c in {lo, (lo + hi) // 2, hi - 1} if hi > lo else ():
            off = bench.channel_offset_bytes(c, n)
            assert off == displs[r] + 8 * n * (c - lo)
            assert displs[r] <= off and off + 8 * n <= displs[r] + sizes[r]


def test_comm_plan_v_rejects_bad_args(sdr):
    from sdrgpu._lib import SdrGpuError
    from sdrgpu.shard import plan_v
    with pytest.raises(SdrGpuError):
        plan_v(4, 0, 4, False, [8, 8, 8, 8])    # root out of range
    with pytest.raises(SdrGpuError):
        plan_v(4, 4, 0, True, [8, 8, 8, 8])     # rank out of range


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
