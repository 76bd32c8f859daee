#!/bin/bash
# configs[2] STFT with the two-stream default: kernel trace + FETCH/WRITE PMC passes; resampler PMC.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c3prof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench_configs.py --config c3 --no-cpu-baseline --steps 5 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
tail -1 $O/trace.log | cut -c1-300
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python $R/bench_configs.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 2; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python $R/bench_configs.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/sfetch -o run -- python $R/bench_configs.py --config src --steps 3 --warmup 1 > $O/sfetch.log 2>&1 || { tail -5 $O/sfetch.log; exit 4; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/swrite -o run -- python $R/bench_configs.py --config src --steps 3 --warmup 1 > $O/swrite.log 2>&1 || { tail -5 $O/swrite.log; exit 5; }
echo pmc done
