#!/bin/bash
# census8 per-direction engine: Infinity-Cache-sized launch groups (default) vs one 8-pair group (1 << 30)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mall; mkdir -p $OUT
timeout -k 10 200 python tools/ablate.py --mode census8 --pairs 8 --rounds 5 --flags 0,$((1<<30)) > $OUT/census8_p8.log 2>&1 || { cat $OUT/census8_p8.log; exit 1; }
cat $OUT/census8_p8.log
timeout -k 10 200 python tools/ablate.py --mode census8 --pairs 16 --rounds 3 --flags 0,$((1<<30)) > $OUT/census8_p16.log 2>&1 || { cat $OUT/census8_p16.log; exit 1; }
cat $OUT/census8_p16.log
timeout -k 10 200 python -u bench.py --cpu-baseline-pairs 0 --host-surface-calls 0 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-300
