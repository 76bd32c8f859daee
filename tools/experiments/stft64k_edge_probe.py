import sys, numpy as np
sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo/unnamed-rust-sdr_amd'); sys.path.insert(0, '/root/repo/oracle')
import conftest
from conftest import rms_rel_err
import sdrgpu
from sdrgpu.device import DeviceBuffer
from test_fft_gpu import _c3_frame_span, cplx
n, hop, nfr = 65536, 32768, 12
total = hop * nfr
rng = np.random.default_rng(64)
t = np.arange(total)
for noise in (1e-6, 0.0, 1.0):
    base = (np.exp(2j * np.pi * 0.1234567 * t) + noise * cplx(rng, total)).astype(np.complex64)
    base[4 * hop:6 * hop] = 0
    for scale in (1e-30, 1e-20, 1e-10, 1.0, 1e30):
        x = (base * np.float32(scale)).astype(np.complex64)
        s = sdrgpu.fft.Stft(n, hop)
        dx = DeviceBuffer.from_numpy(x); dy = DeviceBuffer.empty(nfr * n)
        s.process_dev(dx.ptr, total, dy.ptr, nfr); s.sync()
        y = dy.download(nfr * n).reshape(nfr, n)
        errs = []
        for j in (0, 3, 4, 6, nfr - 1):
            span = _c3_frame_span(x, j, n, hop).astype(np.complex128)
            ref = np.fft.fftshift(np.fft.fft(span)) / np.sqrt(n)
            errs.append("%.1e" % rms_rel_err(y[j], ref)[0])
        # also the generic small-N plan on frame 0 as a cross-check
        print(f"noise {noise} scale {scale}: frames 0,3,4,6,11 max/rms", errs, flush=True)
