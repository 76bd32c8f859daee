"""CPU tests of bench.py's JSON line (the driver contract) and its evidence fields: the
fp16x2 arithmetic label, the PMC traffic figure tied to the kernel source it was measured
on, and the channel-sharded leg's record shape (the leg itself runs on the GPU:
tests/test_bench_gpu.py)."""
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")


def test_headline_record_contract_and_labels():
    n = 1 << 28
    r = bench.headline_record(5.1e5, 1, 20, 3, 20 * 0.53e-3, n, 4, 0.525, 2.75e9,
                              {"status": "matches this kernel source"}, "auto")
    assert all(k in r for k in CONTRACT)
    assert r["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert r["config"]["workload"].startswith("configs[1]")
    assert "fp16x2" in r["config"]["arith"] and "f32 accumulate" in r["config"]["arith"]
    rf = r["roofline"]
    assert rf["bound"] == "hbm" and rf["peak"] == 8000.0 and rf["unit"] == "GB/s"
    assert abs(rf["achieved"] - 10 * n / 0.525e-3 / 1e9) < 0.1
    assert abs(rf["frac"] - rf["achieved"] / 8000.0) < 1e-4
    assert rf["traffic"] == 2.75e9 and rf["traffic_source"]["status"].startswith("matches")
    json.dumps(r)


def test_pmc_traffic_tied_to_kernel_source(tmp_path):
    sha = bench.kernel_source_sha16()
    good = {"log2n": 28, "algo": "auto", "hbm_bytes_per_launch": 2.7e9,
            "kernel_source_sha16": sha, "commit": "abc1234", "method": "m"}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(good))
    t, src = bench.pmc_traffic(str(p), 28, "auto")
    assert t == 2.7e9 and src["status"] == "matches this kernel source"
    assert src["commit"] == "abc1234" and src["kernel_source_sha16"] == sha
    p.write_text(json.dumps(dict(good, kernel_source_sha16="0" * 16)))
    t, src = bench.pmc_traffic(str(p), 28, "auto")
    assert t is None and src["status"].startswith("stale")
    p.write_text(json.dumps(dict(good, log2n=20)))
    assert bench.pmc_traffic(str(p), 28, "auto")[0] is None
    t, src = bench.pmc_traffic(str(tmp_path / "none.json"), 28, "auto")
    assert t is None and src["status"] == "missing"


def test_committed_pmc_file_matches_the_shipped_kernel():
    """profiles/pmc_fir_c2.json is the figure bench.py reports as roofline.traffic: it must
    have been measured on the fir_mxh source in this tree (re-measure after a kernel change:
    tools/gpu/final.sh's FETCH / WRITE passes -> tools/pmc_to_json.py)."""
    t, src = bench.pmc_traffic(os.path.join(ROOT, "profiles", "pmc_fir_c2.json"), 28, "auto")
    assert t is not None, src
    assert 1.0 <= t / (10 * (1 << 28)) <= 1.1


def test_channel_sharded_leg_guard_exception_and_hang():
    """bench.run_guarded: a failing leg becomes an "error" entry; a hung leg (a peer that died
    inside an RCCL collective) fires the watchdog, which emits the line and exits NON-zero
    (bench.LEG_HUNG_EXIT), so the hang is reported as a failed run, not a clean one."""
    import subprocess
    import sys
    import bench
    out = bench.run_guarded(lambda: 1 / 0, 30.0, 0, lambda: None)
    assert "ZeroDivisionError" in out["error"]
    assert bench.run_guarded(lambda: {"ok": 1}, 30.0, 0, lambda: None) == {"ok": 1}
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.run_guarded(lambda: time.sleep(60), 0.5, 0, lambda: print('LINE', flush=True)); "
            "print('NOT REACHED')") % bench.ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=30)
    assert p.returncode == bench.LEG_HUNG_EXIT != 0, (p.returncode, p.stderr)
    assert "LINE" in p.stdout and "NOT REACHED" not in p.stdout
    assert "abandoning" in p.stderr


def test_gloo_init_keeps_stdout_clean(tmp_path):
    """bench.init_gloo_quiet: a 2-rank gloo rendezvous prints nothing on stdout (the driver
    reads rank 0's stdout for its one JSON line); gloo's connect message goes to stderr."""
    import subprocess
    import sys
    import bench
    code = ("import os, sys; sys.path.insert(0, %r); import bench; import torch.distributed as dist; "
            "bench.init_gloo_quiet(dist); dist.barrier(); print('OK', flush=True); "
            "dist.destroy_process_group()") % bench.ROOT
    port = bench._free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 0, err
        assert out.strip() == "OK", out
