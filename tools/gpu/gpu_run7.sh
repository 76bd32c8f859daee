#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_pll_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_pll.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_pll.log
cat > /tmp/pllbench.py <<'PY'
import sys, time, numpy as np
sys.path.insert(0, 'unnamed-rust-sdr_amd')
import sdrgpu
from sdrgpu.device import DeviceBuffer, Event
f = sdrgpu.filter
nch, n = 1024, 1 << 16
rng = np.random.default_rng(0)
x = (np.exp(1j * rng.uniform(0, 6.28, (nch, n))) ).astype(np.complex64)
pll = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity, f.BiquadD.LowPass(20000.0, 0.7)).design(1.8e6, nch=nch)
dx = DeviceBuffer.from_numpy(x); dy = DeviceBuffer.empty(nch * n, np.float32); dl = DeviceBuffer.empty(nch * n, np.uint8)
pll.process_dev(dx.ptr, n, n, dy.ptr, dl.ptr, n); pll.sync()
e0, e1 = Event(), Event()
e0.record(pll.stream()); pll.process_dev(dx.ptr, n, n, dy.ptr, dl.ptr, n); e1.record(pll.stream()); pll.sync()
ms = e0.elapsed_ms(e1)
print(f"PLL {nch} ch x {n}: {ms:.2f} ms -> {nch*n/ms/1e3:.1f} Msamples/s, {ms*1e6/n:.1f} ns/sample/channel-chain")
PY
timeout -k 10 300 python /tmp/pllbench.py > gpurun_out/pllbench.log 2>&1
echo done
