#!/bin/bash
# Horizontal-family prefetch depth: default library vs tools/exp/*.so, sgbm5 (E/W before
# the WTA sweep), census8 sweeps (16384) and the census8 per-direction headline (0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for so in default tools/exp/*.so; do
  [ "$so" = default ] || [ -e "$so" ] || continue
  n=$(basename $so .so)
  if [ "$so" = default ]; then unset STEREO_MATCH_AMD_LIB; else export STEREO_MATCH_AMD_LIB=$PWD/$so; fi
  timeout -k 10 300 python -u tools/ablate.py --mode sgbm5 --flags 0 --pairs 8 --rounds 3 > gpurun_out/pf_$n.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/ablate.py --flags 0,16384 --pairs 8 --rounds 3 >> gpurun_out/pf_$n.log 2>&1 || exit $?
  echo $n; grep -o '"flags.*' gpurun_out/pf_$n.log | cut -c1-200
done
