# STFT throughput per frame size (hop N/2, 2^28 c64 zeros resident): python tools/stft_sizes.py [N ...]
import sys, os, json, time
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"] + "/unnamed-rust-sdr_amd")
import numpy as np, sdrgpu
from sdrgpu.device import DeviceBuffer, Event, synchronize
n_in = 1 << 28
x = DeviceBuffer.empty(n_in)
x.fill_zero()
SIZES = [int(v) for v in sys.argv[1:]] or [8192, 16384, 32768, 65536]
for N in SIZES:
    st = sdrgpu.fft.Stft(N, N // 2)
    nf = st.output_len(n_in)
    y = DeviceBuffer.empty(nf * N)
    for _ in range(2):
        st.reset(); st.process_dev(x.ptr, n_in, y.ptr, nf)
    st.sync()
    e0, e1 = Event(), Event()
    e0.record(st.stream())
    for _ in range(5):
        st.reset(); st.process_dev(x.ptr, n_in, y.ptr, nf)
    e1.record(st.stream()); st.sync()
    ms = e0.elapsed_ms(e1) / 5
    print(json.dumps({"N": N, "ms": round(ms, 4), "frac": round(24 * n_in / (ms * 1e-3) / 8e12, 4)}), flush=True)
    del y
