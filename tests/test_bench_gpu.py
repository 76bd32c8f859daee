"""bench.py's configs[4] channel-sharded leg on one GPU (the N = 1 point of the driver's
scaling runs): the resident bank rate record and the float64 spot check of the outputs."""
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, ROOT)


def test_channel_sharded_leg_single_rank():
    import bench
    r = bench.channel_sharded_leg(steps=2, warmup=1, world=1, rank=0, local=0, dist=None,
                                  nch_total=300, log2n=13)
    assert r["channels_per_rank"] == [300]
    assert r["resident"]["value"] > 0 and r["resident"]["ms_per_step"] > 0
    assert "rccl" not in r                       # one rank: nothing to fan out
    assert len(r["spot_check_max_over_rms"]) == 1
    assert max(r["spot_check_max_over_rms"].values()) <= 1e-5
