#!/bin/bash
# census8: per-direction (0, horizontal census on the fly 2048), k_sweep, k_sweep2 nw=3 / nw=4 at 8 and 16 pairs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sw4; mkdir -p $OUT
for P in 8 16; do
  timeout -k 10 150 python tools/ablate.py --mode census8 --pairs $P --rounds 3 --flags 0,16384,$((16384|128)),$((16384|(1<<27))) > $OUT/census8_p$P.log 2>&1 || { cat $OUT/census8_p$P.log; exit 1; }
  echo "== census8 P=$P"; cat $OUT/census8_p$P.log
done
