#!/bin/bash
# configs[2] timing under env variants, one line of VAR=value assignments per variant ($VFILE).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_c3v}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
timeout -k 10 300 python -u -m pytest tests/test_fft_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "64k or c3 or 65536" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  env $line timeout -k 10 120 python -u bench_configs.py --config c3 --no-cpu-baseline $EXTRA --steps 10 --warmup 2 > $O/v$i.jsonl 2> $O/v$i.err
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "variant $i ($line) failed rc=$rc"; tail -3 $O/v$i.err
    case $rc in 124|134|137|139) exit 2;; esac
    continue
  fi
  python -c "import json; d=json.loads(open('$O/v$i.jsonl').read().splitlines()[-1]); r=d['roofline']; print('$line |', r['kernel_ms'], r['frac'], d['spot_check_max_over_rms'])"
done < $VFILE
