#!/bin/bash
# Rehearse bench.py's multi-rank path (gloo barrier, max-over-ranks) with 2 ranks on the box's GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dist2
mkdir -p $O
cd $R
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
grep '^{' $O/bench2.log | cut -c1-400
