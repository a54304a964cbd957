#!/bin/bash
# GPU tests (optional -k expression), then sweep-engine timing ablations:
# census8 per-direction engine (0) vs sweeps (16384) and their no-wait / no-poll
# variants (| 1<<24, | 2<<24); sgbm5 sweeps (0) vs per-direction (4096).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pt_sw.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_sw.log 2>&1
fi
rc=$?; tail -4 gpurun_out/pt_sw.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ablate.py --flags 0,16384,16793600,33570816 --pairs ${PAIRS:-8} --rounds 3 > gpurun_out/abl8.log 2>&1 && \
timeout -k 10 300 python -u tools/ablate.py --mode sgbm5 --flags 0,4096 --pairs ${PAIRS:-8} --rounds 3 > gpurun_out/abl_sgbm.log 2>&1
rc2=$?
cat gpurun_out/abl8.log gpurun_out/abl_sgbm.log | grep flags
exit $rc2
