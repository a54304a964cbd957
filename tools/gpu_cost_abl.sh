#!/bin/bash
# SGBM cost kernel timing: default library and tools/exp/*.so variants (sgbm5), then a PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for so in default tools/exp/*.so; do
  [ "$so" = default ] || [ -e "$so" ] || continue
  n=$(basename $so .so)
  if [ "$so" = default ]; then unset STEREO_MATCH_AMD_LIB; else export STEREO_MATCH_AMD_LIB=$PWD/$so; fi
  timeout -k 10 300 python -u tools/ablate.py --mode sgbm5 --flags ${FLAGS:-0,8388608} --pairs 8 --rounds 3 > gpurun_out/cabl_$n.log 2>&1 || exit $?
  echo $n; grep -o '"flags.*"cost": [0-9.]*' gpurun_out/cabl_$n.log
done
unset STEREO_MATCH_AMD_LIB
[ -n "${PMC:-}" ] && MODE=sgbm5 KF="cost2|prefilter|tail" bash tools/pmc.sh cost2 ${PMCFLAGS:-0} \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
exit 0
