#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fft
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fft_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "65536 or stft" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench_configs.py --config c3 --no-cpu-baseline > $O/c3_$n.log 2>&1 || { tail -5 $O/c3_$n.log; exit 2; }
  python -c "
import json; d=json.loads(open('$O/c3_$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
run nt0_s128 SDRGPU_FFT64K_NT=0
run nt1_s128 SDRGPU_FFT64K_NT=1
run nt1_s64 SDRGPU_FFT64K_NT=1 SDRGPU_FFT_SLAB_MIB=64
run nt1_s192 SDRGPU_FFT64K_NT=1 SDRGPU_FFT_SLAB_MIB=192
run nt1_s256 SDRGPU_FFT64K_NT=1 SDRGPU_FFT_SLAB_MIB=256
run nt1_s512 SDRGPU_FFT64K_NT=1 SDRGPU_FFT_SLAB_MIB=512
