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
        n = self.nranks
        assert len(bytes_per_rank) == n
        b = (ctypes.c_size_t * n)(*bytes_per_rank)
        d = (ctypes.c_size_t * n)(*[sum(bytes_per_rank[:r]) for r in range(n)])
        return b, d

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
