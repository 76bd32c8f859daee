#!/bin/bash
# Round 5: configs[3] chain discriminator over PLL register footprints (tools/diag/pll_vgpr_build.sh,
# prebuilt here): which (bank build, PLL kernel, PLL VGPRs) pairs mismatch the oracle?  Then
# the PLL's ns per sample-chain for the candidate fixes (bench_configs c4, 2^18 samples).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_vgpr_disc}
mkdir -p $O
cd $R
for v in ${VARS:-one_orig one_scalar96 one_split80 one_splitx one_scalarx prod_split80 prod_scalar80 prod_orig}; do
  f=$O/$v.txt
  timeout -k 10 180 python -u tools/experiments/run_with_lib.py tools/diag/probe_build/lib_$v.so tools/diag/c4_snap_diag.py ${CUT:-3000} 0 split > $f 2>&1 || { tail -20 $f; exit 2; }
  echo "== $v"; grep -h "PLL\|^  " $f | cut -c1-300
done
for v in ${TVARS:-prod_orig prod_splitx prod_scalarx prod_orig}; do
  f=$O/c4_$v.jsonl
  timeout -k 10 240 python -u tools/experiments/run_with_lib.py tools/diag/probe_build/lib_$v.so bench_configs.py --config c4 --no-cpu-baseline --c4-log2n 18 > $f 2> $O/c4_$v.err || { tail -20 $O/c4_$v.err; exit 3; }
  echo "== c4 $v"; python3 -c "import json,sys; d=json.loads(open('$f').readline()); print(d.get('pll_ns_per_sample_chain'), d.get('fir_ms'), d.get('pll_ms'))"
done
