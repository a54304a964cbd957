#!/bin/bash
# fused sweeps vs compute waves per strip (SWEEP_NCW builds in var/, tools/build_variant.sh):
# census8 sweeps (16384; flag 0 = per-direction reference), sgbm5 / sgbm8 (flag 4096 = per-direction)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ncw; mkdir -p $OUT
for v in default ${VARIANTS:-ncw9 ncw11 ncw13 ncw15}; do
  if [ $v = default ]; then unset STEREO_MATCH_AMD_LIB; else export STEREO_MATCH_AMD_LIB=$PWD/var/lib_$v.so; fi
  for m in census8 sgbm5 sgbm8; do
    fl=0,4096; [ $m = census8 ] && fl=0,16384
    timeout -k 10 150 python tools/ablate.py --mode $m --pairs ${PAIRS:-8} --rounds 3 --flags $fl > $OUT/${m}_${v}_p${PAIRS:-8}.log 2>&1 || { cat $OUT/${m}_${v}_p${PAIRS:-8}.log; exit 1; }
    echo "== $v $m P=${PAIRS:-8}"; cat $OUT/${m}_${v}_p${PAIRS:-8}.log
  done
done
