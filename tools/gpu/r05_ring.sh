set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_fir_gpu.py tests/test_firbank_gpu.py tests/test_ingest_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ring_tests.log 2>&1 || { tail -30 gpurun_out/ring_tests.log; exit 1; }
tail -1 gpurun_out/ring_tests.log
OUT=${OUT:-ab_ring} KINDS="${KINDS:-c64 bank}" REPS=${REPS:-3} bash tools/gpu/ab.sh
