#!/bin/bash
# Quick sweep-engine timing: default library and (if present) tools/exp/*.so variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ablate.py --flags ${FLAGS:-0,4096} --pairs ${PAIRS:-8} --rounds 3 > gpurun_out/abl_def.log 2>&1 || exit $?
echo default; grep flags gpurun_out/abl_def.log
for so in tools/exp/*.so; do
  [ -e "$so" ] || continue
  n=$(basename $so .so)
  STEREO_MATCH_AMD_LIB=$PWD/$so timeout -k 10 300 python -u tools/ablate.py --flags 0 --pairs ${PAIRS:-8} --rounds 3 > gpurun_out/abl_$n.log 2>&1 || exit $?
  echo $n; grep flags gpurun_out/abl_$n.log
done
