#!/bin/bash
# Async pinned host streaming: parity test, then PCIe-inclusive rates (pageable sync vs pinned async).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pinned
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stream_gpu.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench_configs.py --config c2pinned > $O/pinned.log 2>&1 || { tail -20 $O/pinned.log; exit 2; }
tail -1 $O/pinned.log
timeout -k 10 300 python bench_configs.py --config c2host --steps 5 > $O/host.log 2>&1 || { tail -20 $O/host.log; exit 3; }
tail -1 $O/host.log
