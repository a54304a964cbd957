#!/bin/bash
# Quick sweep-engine timing: default library and tools/exp/*.so variants (census8 sweeps, sgbm5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for so in default tools/exp/*.so; do
  [ "$so" = default ] || [ -e "$so" ] || continue
  n=$(basename $so .so)
  if [ "$so" = default ]; then unset STEREO_MATCH_AMD_LIB; else export STEREO_MATCH_AMD_LIB=$PWD/$so; fi
  timeout -k 10 300 python -u tools/ablate.py --flags ${FLAGS:-16384,33570816} --pairs ${PAIRS:-8} --rounds 3 > gpurun_out/abl_$n.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/ablate.py --mode sgbm5 --flags 0 --pairs ${PAIRS:-8} --rounds 3 >> gpurun_out/abl_$n.log 2>&1 || exit $?
  echo $n; grep flags gpurun_out/abl_$n.log
done
