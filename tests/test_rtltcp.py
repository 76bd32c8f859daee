"""rtl_tcp ingest end to end: a fake rtl_tcp server speaks the protocol of
reference src/rtltcp.rs (12-byte id, 5-byte big-endian commands, then interleaved u8 I/Q);
the sdrgpu.rtltcp client mirrors RtlTcp::listen's command sequence (:54-76) and hands the
raw bytes to the GPU FIR / PLL (CU8 sample kind), which must equal the oracle applied to
RtlTcpSignal::next's (v - 128) / 128 samples (:156-164)."""
import socket
import struct
import threading

import numpy as np
import pytest
import scipy.signal as ss


class FakeRtlTcp:
    def __init__(self, payload: bytes):
        self.payload = payload
        self.commands = []
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(1)
        self.port = self.srv.getsockname()[1]
        self.t = threading.Thread(target=self.run, daemon=True)
        self.t.start()

    def run(self):
        c, _ = self.srv.accept()
        c.sendall(b"RTL0" + struct.pack(">II", 5, 29))  # dongle id: magic, tuner, gains
        c.settimeout(0.5)
        buf = b""
        try:  # commands until the client goes quiet
            while True:
                d = c.recv(64)
                if not d:
                    break
                buf += d
                if len(buf) >= 25:
                    break
        except socket.timeout:
            pass
        self.commands = [struct.unpack(">BI", buf[i:i + 5]) for i in range(0, len(buf) // 5 * 5, 5)]
        c.sendall(self.payload)
        c.close()
        self.srv.close()


def make_iq(n, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 1.8e6
    x = np.exp(2j * np.pi * 50e3 * t) * 0.6 + 0.05 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    iq = np.empty(2 * n, np.uint8)
    iq[0::2] = np.clip(np.round(x.real * 127 + 128), 0, 255)
    iq[1::2] = np.clip(np.round(x.imag * 127 + 128), 0, 255)
    return iq


def test_rtltcp_protocol_and_bytes(sdr):
    from sdrgpu import rtltcp
    iq = make_iq(50000)
    srv = FakeRtlTcp(iq.tobytes())
    sig = (rtltcp.RtlTcp().address(("127.0.0.1", srv.port)).rate(1800000)
           .frequency(96300000).gain(None).rtlagc(True).listen(0.01))
    assert sig.rate() == 1800000.0 and sig.sample_kind == sdr.CU8
    got = np.concatenate(list(sig.blocks()))
    assert np.array_equal(got, iq)
    # RtlTcpConnection::connect + RtlTcp::listen (src/rtltcp.rs:54-76, 93-108)
    assert srv.commands == [(0x02, 1800000), (0x01, 96300000), (0x03, 0), (0x08, 1)]


def test_rtltcp_manual_gain_and_bad_rate(sdr):
    from sdrgpu import rtltcp
    srv = FakeRtlTcp(b"")
    conn = rtltcp.RtlTcp().address(("127.0.0.1", srv.port)).gain(2.25).connect()
    conn.close()
    srv.t.join(2)
    assert (0x03, 1) in srv.commands and (0x04, 23) in srv.commands  # round half away
    srv2 = FakeRtlTcp(b"")
    with pytest.raises(ValueError):
        rtltcp.RtlTcp().address(("127.0.0.1", srv2.port)).rate(500000).connect()


@pytest.mark.gpu
def test_rtltcp_into_gpu_fir_and_pll(sdr, oracle):
    from sdrgpu import rtltcp
    f = sdr.filter
    iq = make_iq(120000, seed=3)
    taps = ss.firwin(255, 0.2).astype(np.float32)
    x = oracle.u8_to_c64(iq)
    # FIR + decimate on the raw bytes (examples/live.rs:29-31 shape)
    srv = FakeRtlTcp(iq.tobytes())
    y = (rtltcp.RtlTcp().address(("127.0.0.1", srv.port)).listen(0.013)
         .filter(taps).decimate(1.8e6 / 4).collect())
    ref = oracle.Fir(taps, decim=4, sample_kind=oracle.C64).process(x)
    from conftest import assert_parity
    assert_parity(y, ref, what="rtl_tcp -> FIR")
    # PLL FM demod on the raw bytes (src/main.rs:48-49), bit-exact
    srv = FakeRtlTcp(iq.tobytes())
    pllf = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                       f.BiquadD.LowPass(20000.0, 0.7))
    blocks = list(rtltcp.RtlTcp().address(("127.0.0.1", srv.port)).listen(0.01)
                  .filter(pllf).blocks())
    out = np.concatenate([b["value"] for b in blocks])
    lk = np.concatenate([b["locked"] for b in blocks])
    ro, rl = oracle.pll_batch(oracle.pll_params(0.0, 0.035, 1.8e6, (1, 80000.0, 0.7),
                                                (0, 0.0, 0.0), (1, 20000.0, 0.7)), x)
    assert np.array_equal(out, ro[0]) and np.array_equal(lk, rl[0].astype(bool))
