#!/bin/bash
# fused sweeps (default, wide strips) vs the per-direction engine (4096) at small launch groups
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/minpairs; mkdir -p $OUT
for m in census8 sgbm5 sgbm8; do
  for P in 3 4 6; do
    timeout -k 10 120 python tools/ablate.py --mode $m --pairs $P --rounds 3 --flags 16384,4096 > $OUT/${m}_p$P.log 2>&1 || { cat $OUT/${m}_p$P.log; exit 1; }
    echo "== $m P=$P"; grep '^{' $OUT/${m}_p$P.log | cut -c1-200
  done
done
