#!/bin/bash
# bench.py self-launched ranks (2 ranks sharing the box's one GPU), comm test, c4/c5 lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_multi}
mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest tests/test_comm_gpu.py -m gpu -x -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/pytest_comm.log 2>&1 || { tail -30 $O/pytest_comm.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 2; }
tail -1 $O/bench2.log
timeout -k 10 500 python bench_configs.py --config c4 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 3; }
tail -1 $O/c4.log
timeout -k 10 300 python bench_configs.py --config c5 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 4; }
tail -1 $O/c5.log
