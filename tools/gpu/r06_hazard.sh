#!/bin/bash
# Round 6: the configs[3] chain reproducer (tools/diag/c4_snap_diag.py: 1024-channel ONE bank
# block beside the pre-fix split PLL) over the packed-f32 wait-state arms of
# tools/diag/hazard_build.sh (prebuilt in tools/diag/probe_build/).  One process per arm.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_hazard}
mkdir -p $O
cd $R
i=0
for v in ${ARMS:-ctl after12 before12 rt after0 after12 ctl}; do
  i=$((i + 1))
  f=$O/${i}_$v.txt
  timeout -k 10 180 python -u tools/experiments/run_with_lib.py tools/diag/probe_build/lib_haz_$v.so tools/diag/c4_snap_diag.py ${CUT:-3000} 0 split > $f 2>&1 || { tail -20 $f; exit 2; }
  echo "== $i $v"; grep -h "PLL\|bad channels" $f | cut -c1-220
done
