#!/bin/bash
# Single-pair (one compute_disparity per call, settings.ini D=160) timing of the main library
# and each var/lib_<name>.so given, interleaved on one box.
# Usage: bash tools/gpu_single_ab.sh TAG name1 name2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in main "$@" main; do
  if [ $v = main ]; then L=""; else L="$PWD/var/lib_$v.so"; fi
  STEREO_MATCH_AMD_LIB=$L timeout -k 10 240 python3 tools/single_pair.py --flags 0 --calls 40 > $OUT/single_$v.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 $OUT/single_$v.log; exit $rc; fi
  echo "$v $(tail -1 $OUT/single_$v.log)"
done
