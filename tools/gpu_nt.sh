#!/bin/bash
# A/B: default path-volume stores vs nt (stereo_match_amd/libsm_nt.so, -DPATHS_STORE_AUX=2),
# census8 per-direction engine at 8 and 2 pairs per launch group (cap bits 2 << 16)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/nt; mkdir -p $OUT
for lib in default nt; do
  if [ $lib = nt ]; then export STEREO_MATCH_AMD_LIB=$PWD/stereo_match_amd/libsm_nt.so; fi
  timeout -k 10 150 python tools/ablate.py --mode census8 --pairs 8 --rounds 3 --flags 0,$((3<<16)),$((4<<16)),$((5<<16)),$((6<<16)) > $OUT/$lib.log 2>&1 || { cat $OUT/$lib.log; exit 1; }
  echo "== $lib"; cat $OUT/$lib.log
done
