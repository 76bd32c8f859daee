#!/bin/bash
# Evidence pass for a tree (outputs under gpurun_out/$OUT): the driver's GPU suite, smoke, the
# driver's bench command plus a rocprofv3 kernel trace / stats of that same command, FETCH and
# WRITE PMC passes of the headline launch (-> pmc_fir_c2.json via tools/pmc_to_json.py),
# every bench_configs line, and the 2-rank rehearsals (one GPU shared).  SKIP_TESTS / SKIP_HEAD
# / SKIP_CONFIGS skip a part; U8PROF=1 adds the rtl_tcp u8 launch's trace and PMC.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-final}
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
if [ -z "$SKIP_HEAD" ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
cut -c1-400 $O/bench.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.jsonl 2> $O/prof.log || { tail -20 $O/prof.log; exit 4; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-channel-sharded > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 5; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-channel-sharded > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 6; }
cd $R
python3 tools/pmc_to_json.py $O/pmc $O/pmc_fir_c2.json fir_mxh && head -8 $O/pmc_fir_c2.json
fi
if [ -z "$SKIP_CONFIGS" ]; then
timeout -k 10 900 python -u bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 7; }
cut -c1-300 $O/configs.jsonl
timeout -k 10 300 python -u bench_configs.py --config c5 --gpus 2 --no-cpu-baseline > $O/c5_2rank.jsonl 2> $O/c5_2rank.err || { tail -20 $O/c5_2rank.err; exit 8; }
cut -c1-500 $O/c5_2rank.jsonl
timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_2rank.jsonl 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 9; }
cut -c1-300 $O/bench_2rank.jsonl
fi
if [ -n "$U8PROF" ]; then
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_u8 -o run -- python3 $R/bench_configs.py --config c2u8 --steps 20 --warmup 5 > $O/prof_u8.jsonl 2> $O/prof_u8.log || { tail -20 $O/prof_u8.log; exit 10; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_u8/pmc_fetch -o run -- python3 $R/bench_configs.py --config c2u8 --steps 3 --warmup 1 > $O/pmc_u8_fetch.log 2>&1 || { tail -5 $O/pmc_u8_fetch.log; exit 11; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_u8/pmc_write -o run -- python3 $R/bench_configs.py --config c2u8 --steps 3 --warmup 1 > $O/pmc_u8_write.log 2>&1 || { tail -5 $O/pmc_u8_write.log; exit 12; }
cd $R
python3 tools/pmc_to_json.py $O/pmc_u8 $O/pmc_u8.json fir_mxi && head -8 $O/pmc_u8.json
cut -c1-400 $O/prof_u8.jsonl
fi
