#!/bin/bash
# 64K STFT: two-stream batch overlap (SDRGPU_FFT64K_STREAMS=2) -- parity, then c3 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fft2s
mkdir -p $O
cd $R
SDRGPU_FFT64K_STREAMS=2 timeout -k 10 300 python -u -m pytest tests/test_fft_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for cfg in "2 256" "2 128" "2 192" "2 64"; do
set -- $cfg
SDRGPU_FFT64K_STREAMS=$1 SDRGPU_FFT_SLAB_MIB=$2 timeout -k 10 200 python bench_configs.py --config c3 --no-cpu-baseline --steps 5 > $O/c3_$1_$2_$rep.log 2>&1 || { tail -5 $O/c3_$1_$2_$rep.log; exit 2; }
echo "streams=$1 slab=$2 rep=$rep $(tail -1 $O/c3_$1_$2_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
done
