#!/bin/bash
# census8 / sgbm5 sweeps: upper bound of removing the per-row workgroup barrier (results wrong)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/nobar; mkdir -p $OUT
timeout -k 10 150 python tools/ablate.py --mode census8 --pairs 8 --rounds 3 --flags 16384,$((16384|(1<<24))),$((16384|(1<<26))),$((16384|(3<<25))) > $OUT/census8.log 2>&1 || { cat $OUT/census8.log; exit 1; }
cat $OUT/census8.log
timeout -k 10 150 python tools/ablate.py --mode sgbm5 --pairs 8 --rounds 3 --flags 0,$((1<<26)) > $OUT/sgbm5.log 2>&1 || { cat $OUT/sgbm5.log; exit 1; }
cat $OUT/sgbm5.log
