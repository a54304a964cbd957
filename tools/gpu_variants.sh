#!/bin/bash
# census8 (or MODE) bench of the main library and each var/lib_<name>.so given, same box.
# Usage: bash tools/gpu_variants.sh TAG MODE name1 name2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; MODE=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in main "$@" main; do
  if [ $v = main ]; then L=""; else L="$PWD/var/lib_$v.so"; fi
  STEREO_MATCH_AMD_LIB=$L timeout -k 10 240 python bench.py --mode $MODE --steps 200 --warmup 10 --cpu-baseline-pairs 0 --host-surface-calls 0 > $OUT/var_${MODE}_$v.jsonl 2> $OUT/var_${MODE}_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 $OUT/var_${MODE}_$v.err; exit $rc; fi
  python3 -c "import json; d=json.loads(open('$OUT/var_${MODE}_$v.jsonl').read().strip().splitlines()[-1]); print('$v', '$MODE', round(d['value'],1), 'pairs/s', 'pipe', round(d['pipeline_roofline']['frac'],3), {k: round(v,1) for k,v in d['stage_us_per_pair'].items() if v})"
done
