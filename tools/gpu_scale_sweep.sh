#!/bin/bash
# Sweep-engine scaling with pairs per launch (census8): is it latency-bound?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/scale_sweep; mkdir -p $OUT
for P in 1 2 4 8 12; do
  echo "== pairs $P"
  timeout -k 10 120 python tools/ablate.py --pairs $P --rounds 3 --flags 0,16384,$((16384|(1<<24))) > $OUT/p$P.log 2>&1 || { cat $OUT/p$P.log; exit 1; }
  cat $OUT/p$P.log
done
