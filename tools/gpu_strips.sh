#!/bin/bash
# strip-width choice of the fused sweeps: default (model) vs narrow (1 << 19) vs wide (1 << 21),
# per-direction (4096) for reference, at several launch-group sizes; then the census8 bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/strips; mkdir -p $OUT
for m in census8 sgbm5 sgbm8; do
  for P in ${PAIRS:-3 7 8}; do
    timeout -k 10 150 python tools/ablate.py --mode $m --pairs $P --rounds 3 \
      --flags 0,$((16384|(1<<19))),$((16384|(1<<21))),4096 > $OUT/${m}_p$P.log 2>&1 || { cat $OUT/${m}_p$P.log; exit 1; }
    echo "== $m P=$P"; grep '^{' $OUT/${m}_p$P.log | cut -c1-220
  done
done
timeout -k 10 300 python -u bench.py --cpu-baseline-pairs 0 --host-surface-calls 0 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-400
