#!/bin/bash
# Single-pair surface + sgbm5 (sweeps, per-direction) per library: main and var/lib_<name>.so.
#   bash tools/gpu_libs.sh TAG name1 name2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in main "$@"; do
  if [ $v = main ]; then L=""; else L="$PWD/var/lib_$v.so"; fi
  STEREO_MATCH_AMD_LIB=$L timeout -k 10 120 python tools/single_pair.py --flags 0 --calls 30 > $OUT/single_$v.log 2>&1 || exit $?
  echo "$v single: $(grep flags $OUT/single_$v.log)"
  for e in auto perdir; do
    STEREO_MATCH_AMD_LIB=$L timeout -k 10 200 python bench.py --mode sgbm5 --engine $e --steps 100 --warmup 10 --cpu-baseline-pairs 0 --host-surface-calls 0 > $OUT/sgbm5_${e}_$v.jsonl 2> $OUT/sgbm5_${e}_$v.err || exit $?
    python3 -c "import json; d=json.loads(open('$OUT/sgbm5_${e}_$v.jsonl').read().strip().splitlines()[-1]); print('$v sgbm5 $e', round(d['value'],1), 'pairs/s', {k: round(v,1) for k,v in d['stage_us_per_pair'].items() if v})"
  done
done
