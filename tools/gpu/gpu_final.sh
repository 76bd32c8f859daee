#!/bin/bash
# Round-end GPU pass: full GPU tests, smoke, default bench, kernel-trace profile of the
# same bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes (no trace domains).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest died rc=$rc"; tail -20 $O/pytest_gpu.log; exit 1;; esac
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 2; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 4; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 5; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 6; }
echo pmc done
cd $R
timeout -k 10 600 python bench_configs.py --config all > $O/configs.log 2>&1 || { tail -5 $O/configs.log; exit 7; }
grep '^{' $O/configs.log > $O/configs.jsonl
echo configs done
