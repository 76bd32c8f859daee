#!/bin/bash
# PLL parity tests, c4 line, PMC instruction counts of the PLL kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_pll}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_pll_gpu.py tests/test_stream_gpu.py tests/test_firbank_gpu.py tests/test_rtltcp.py tests/test_signal.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench_configs.py --config c4 --no-cpu-baseline --c4-log2n 18 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 2; }
tail -1 $O/c4.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc -o run -- python3 $R/bench_configs.py --config c4 --no-cpu-baseline --c4-log2n 16 --steps 2 --warmup 1 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 3; }
mkdir -p $O/pmcd/p1 && cp -r $O/pmc/* $O/pmcd/p1/ && python3 $R/tools/pmc_summary.py $O/pmcd pll_kernel
