#!/bin/bash
# PMC passes over the census8 fused sweeps on wide strips (default, 8 pairs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export KF="sweep|k_ew"
C1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS"
C2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
bash tools/pmc.sh wide 0 "$C1" "$C2"
