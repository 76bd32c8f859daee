"""RCCL channel fan-out / gather (sdrgpu_comm_*) on one GPU: a single-rank communicator
exercises the scatter / gather and the grouped scatterv / gatherv entry points end to end
(the N-rank rendezvous itself is covered by the gloo tests; a 1-GPU box cannot host two
RCCL ranks on one device)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_comm_single_rank_roundtrip(sdr):
    from sdrgpu.device import DeviceBuffer
    from sdrgpu.shard import Comm, unique_id
    c = Comm(0, 1, 0, unique_id())
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    src = DeviceBuffer.from_numpy(a)
    mid = DeviceBuffer(a.nbytes)
    back = DeviceBuffer(a.nbytes)
    c.scatter(src.ptr, mid.ptr, a.nbytes, 0)
    c.gather(mid.ptr, back.ptr, a.nbytes, 0)
    c.barrier()
    assert np.array_equal(back.download(dtype=np.uint8), a)
    mid.fill_zero()
    back.fill_zero()
    c.scatterv(src.ptr, mid.ptr, [a.nbytes], 0)
    c.gatherv(mid.ptr, back.ptr, [a.nbytes], 0)
    c.barrier()
    assert np.array_equal(mid.download(dtype=np.uint8), a)
    assert np.array_equal(back.download(dtype=np.uint8), a)
    c.close()
