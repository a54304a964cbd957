#!/bin/bash
# VALU issue of each kernel from SQ counters (one rocprofv3 --pmc pass, kernel trace
# only), over bench.py: what roofline.valu in the bench line reads back
# (profiles/valu_latest.json, stamped like the traffic file).
# Usage: bash tools/valu.sh [config] [mode]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/valu; mkdir -p $OUT
CONFIG=${1:-kitti}; MODE=${2:-census8}
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d $OUT/pmc -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --cpu-baseline-pairs 0 --host-surface-calls 0 --config $CONFIG --mode $MODE ${BENCH_EXTRA:-} > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/pmc.log; exit $rc; fi
python3 tools/valu_summary.py $OUT $CONFIG $MODE
