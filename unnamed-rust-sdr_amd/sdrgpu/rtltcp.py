"""rtl_tcp client mirror (reference src/rtltcp.rs) feeding raw I/Q bytes to the GPU path.

`RtlTcp` keeps the reference builder (new / address / rate / frequency / gain / rtlagc /
listen, src/rtltcp.rs:7-77) and the connection protocol (12-byte dongle id, then 5-byte
commands: 1-byte opcode + u32 big-endian argument, :84-135).  Where the reference's
`RtlTcpSignal::next` converts every byte pair to Complex<f32> on the CPU (:156-164),
`listen()` here yields the BYTES in blocks with sample kind CU8, so `.filter(taps)` and a
PLL stage consume them directly on the GPU ((v - 128) / 128 is done in the kernel load).
Networking is host plumbing (out of the hot path); this module exists so the
u8 ingest can be driven end to end.
"""
from __future__ import annotations

import math
import socket
import struct

import numpy as np

from . import _lib
from .signal import Signal

SET_FREQUENCY, SET_SAMPLE_RATE, SET_TUNER_GAIN_MODE, SET_TUNER_GAIN, SET_RTL_AGC = (
    0x01, 0x02, 0x03, 0x04, 0x08)


class RtlTcpConnection:
    """RtlTcpConnection (src/rtltcp.rs:79-149)."""

    def __init__(self, rate: int, addr):
        self.sock = socket.create_connection(addr)
        self.id = self._read_exact(12)
        self.rate = 0
        self.command(SET_SAMPLE_RATE, rate)

    def _read_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("rtl_tcp: connection closed during read")
            buf += chunk
        return bytes(buf)

    def command(self, op: int, arg: int):
        self.sock.sendall(struct.pack(">BI", op, arg & 0xFFFFFFFF))
        if op == SET_SAMPLE_RATE:
            if not (225001 <= arg <= 300000) and not (900001 <= arg <= 3200000):
                raise ValueError(f"bad sample rate for rtltcp: {arg}")  # the reference panics
            self.rate = arg

    def read_block(self, nbytes: int) -> bytes:
        """Up to nbytes (even), b'' at end of stream."""
        buf = bytearray()
        while len(buf) < nbytes:
            chunk = self.sock.recv(nbytes - len(buf))
            if not chunk:
                break
            buf += chunk
        return bytes(buf[:len(buf) // 2 * 2])

    def close(self):
        self.sock.close()


class RtlTcp:
    """RtlTcp builder (src/rtltcp.rs:7-77)."""

    def __init__(self):
        self._addr = ("127.0.0.1", 1234)
        self._rate = 1800000
        self._frequency = 100000000
        self._gain = None
        self._rtlagc = False

    def address(self, addr):
        self._addr = addr
        return self

    def rate(self, rate: int):
        self._rate = int(rate)
        return self

    def frequency(self, frequency: int):
        self._frequency = int(frequency)
        return self

    def gain(self, gain):
        """dB, None = automatic"""
        self._gain = gain
        return self

    def rtlagc(self, on: bool):
        self._rtlagc = bool(on)
        return self

    def connect(self) -> RtlTcpConnection:
        """RtlTcp::listen's command sequence (:54-76)."""
        conn = RtlTcpConnection(self._rate, self._addr)
        conn.command(SET_FREQUENCY, self._frequency)
        if self._gain is not None:
            conn.command(SET_TUNER_GAIN_MODE, 1)
            g10 = float(np.float32(self._gain) * np.float32(10.0))
            # f32::round: half away from zero (gain > 0 here)
            conn.command(SET_TUNER_GAIN, int(math.floor(g10 + 0.5)) if g10 > 0 else 0)
        else:
            conn.command(SET_TUNER_GAIN_MODE, 0)
        conn.command(SET_RTL_AGC, int(self._rtlagc))
        return conn

    def listen(self, block_seconds: float = 0.1) -> Signal:
        """A Signal of raw interleaved I/Q byte blocks (sample kind CU8, 2 bytes/sample)."""
        me = self
        nbytes = 2 * max(1, int(round(block_seconds * self._rate)))

        def gen():
            conn = me.connect()
            try:
                while True:
                    b = conn.read_block(nbytes)
                    if not b:
                        return
                    yield np.frombuffer(b, dtype=np.uint8)
            finally:
                conn.close()
        return Signal(float(self._rate), gen, _lib.CU8)
