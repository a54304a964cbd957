#!/bin/bash
# cost-stage launch-shape variants (tools/build_api_variant.sh builds): per-stage device us per
# pair for sgbm5 and census8, 8 KITTI pairs, and a digest of each build's maps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/costvar; mkdir -p $OUT
for v in "$@"; do
  for m in ${MODES:-sgbm5 census8}; do
    STEREO_MATCH_AMD_LIB=$PWD/var/lib_$v.so timeout -k 10 120 python3 tools/ablate.py --mode $m --flags 0 --rounds 5 > $OUT/${v}_$m.log 2>&1 || { echo "FAIL $v $m"; exit 1; }
    echo "$v $m $(tail -2 $OUT/${v}_$m.log | tr '\n' ' ')"
  done
done
