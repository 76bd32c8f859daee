#!/bin/bash
# Round 6: fir_mxi's digit combination as VOP3 (no packed-f32 pairs) -- u8 tests, outputs of the
# u8 shapes bitwise against the previous build (tools/diag/var_build/lib_head.so), A/Bs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_mxi_vop3}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_ingest_gpu.py tests/test_fir_gpu.py -k "cu8 or u8 or silent" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 200 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_head.so tools/diag/determinism.py > $O/det_head.txt 2>&1 &&
timeout -k 10 200 python -u tools/diag/determinism.py > $O/det_new.txt 2>&1 || exit 2
paste -d'|' <(cut -c1-90 $O/det_head.txt) <(cut -c40-200 $O/det_new.txt)
OUT=${OUT:-r06_mxi_vop3}/ab REPS=${REPS:-3} KINDS=${KINDS:-"u8 u8d1 u8d8"} ARMS="head=tools/diag/var_build/lib_head.so new=product" bash tools/gpu/ab.sh
