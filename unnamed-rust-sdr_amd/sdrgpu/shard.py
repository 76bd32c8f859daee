"""Channel / time sharding across the GPUs of one node.

Channels of a FIR bank or PLL batch are independent, and a single stream shards by time
with a (K-1)-sample halo, so the data path needs no reduction.  `Comm` wraps the RCCL
fan-out / gather in libsdrgpu (sdrgpu_comm_*), used only to move channel blocks between a
root and the other ranks; the 128-byte RCCL id is exchanged out of band by the caller
(bench_configs.py uses torch.distributed over gloo).
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib

ID_BYTES = 128


def channel_range(nch: int, world: int, rank: int):
    """Contiguous channel block of `rank` (balanced, first ranks take the remainder)."""
    base, rem = divmod(nch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def time_range(n: int, world: int, rank: int, align: int = 1):
    """Contiguous time shard of a single stream, boundaries aligned to `align` samples
    (the decimation factor, so every shard starts on a kept-output phase)."""
    units = n // align
    lo, hi = channel_range(units, world, rank)
    return lo * align, (hi * align if rank < world - 1 else n)


SEND, RECV, COPY = 0, 1, 2  # sdrgpu_comm_op kinds (include/sdrgpu.h)


class CommOp(ctypes.Structure):
    """sdrgpu_comm_op: one transfer of a scatterv / gatherv plan."""
    _fields_ = [("kind", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("offset", ctypes.c_size_t), ("bytes", ctypes.c_size_t)]


def counts_displs(bytes_per_rank):
    """(bytes, displs): rank r's block size and its offset in the root's packed buffer
    (blocks in rank order, as channel_range lays the channels out)."""
    b = [int(v) for v in bytes_per_rank]
    return b, [sum(b[:r]) for r in range(len(b))]


def _c_counts(bytes_per_rank):
    b, d = counts_displs(bytes_per_rank)
    n = len(b)
    return (ctypes.c_size_t * n)(*b), (ctypes.c_size_t * n)(*d)


def plan_v(nranks: int, rank: int, root: int, gather: bool, bytes_per_rank):
    """The ops sdrgpu_comm_scatterv (gather False) / gatherv (True) issue on `rank`, as
    (kind, peer, offset in the root's buffer, bytes) tuples -- sdrgpu_comm_plan_v, host-only
    (no GPU needed), so every split, including zero-byte ranks, is testable on the CPU."""
    assert len(bytes_per_rank) == nranks
    b, d = _c_counts(bytes_per_rank)
    n = ctypes.c_int()
    check(lib().sdrgpu_comm_plan_v(nranks, rank, root, int(gather), b, d, None, 0,
                                   ctypes.byref(n)), "sdrgpu_comm_plan_v")
    ops = (CommOp * max(1, n.value))()
    check(lib().sdrgpu_comm_plan_v(nranks, rank, root, int(gather), b, d, ops, n.value,
                                   ctypes.byref(n)), "sdrgpu_comm_plan_v")
    return [(o.kind, o.peer, o.offset, o.bytes) for o in ops[:n.value]]


def unique_id() -> bytes:
    buf = (ctypes.c_char * ID_BYTES)()
    check(lib().sdrgpu_comm_unique_id(buf), "sdrgpu_comm_unique_id")
    return bytes(buf)


class Comm:
    def __init__(self, device: int, nranks: int, rank: int, uid: bytes):
        assert len(uid) == ID_BYTES
        self.nranks, self.rank, self.device = nranks, rank, device
        self._h = ctypes.c_void_p()
        buf = (ctypes.c_char * ID_BYTES).from_buffer_copy(uid)
        check(lib().sdrgpu_comm_init(device, nranks, rank, buf, ctypes.byref(self._h)),
              "sdrgpu_comm_init")

    def scatter(self, d_send: int, d_recv: int, bytes_per_rank: int, root: int = 0, stream=None):
        check(lib().sdrgpu_comm_scatter(self._h, d_send, d_recv, bytes_per_rank, root, stream),
              "sdrgpu_comm_scatter")

    def gather(self, d_send: int, d_recv: int, bytes_per_rank: int, root: int = 0, stream=None):
        check(lib().sdrgpu_comm_gather(self._h, d_send, d_recv, bytes_per_rank, root, stream),
              "sdrgpu_comm_gather")

    def _counts(self, bytes_per_rank):
        assert len(bytes_per_rank) == self.nranks
        return _c_counts(bytes_per_rank)

    def scatterv(self, d_send: int, d_recv: int, bytes_per_rank, root: int = 0, stream=None):
        """Uneven blocks: rank r receives bytes_per_rank[r] bytes, packed in rank order in
        the root's buffer."""
        b, d = self._counts(bytes_per_rank)
        check(lib().sdrgpu_comm_scatterv(self._h, d_send, b, d, d_recv, root, stream),
              "sdrgpu_comm_scatterv")

    def gatherv(self, d_send: int, d_recv: int, bytes_per_rank, root: int = 0, stream=None):
        b, d = self._counts(bytes_per_rank)
        check(lib().sdrgpu_comm_gatherv(self._h, d_send, d_recv, b, d, root, stream),
              "sdrgpu_comm_gatherv")

    def barrier(self, stream=None):
        check(lib().sdrgpu_comm_barrier(self._h, stream), "sdrgpu_comm_barrier")

    def close(self):
        if self._h:
            lib().sdrgpu_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
