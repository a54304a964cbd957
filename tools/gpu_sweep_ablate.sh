#!/bin/bash
# GPU tests (-k expression optional), then sweep-engine timing ablations.
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
timeout -k 10 300 python -u tools/ablate.py --flags 0,16777216,4096 --pairs 8 --rounds 3 > gpurun_out/abl8.log 2>&1 && \
timeout -k 10 300 python -u tools/ablate.py --flags 0 --pairs 14 --rounds 3 > gpurun_out/abl14.log 2>&1 && \
timeout -k 10 300 python -u tools/ablate.py --mode sgbm5 --flags 0,4096 --pairs 8 --rounds 3 > gpurun_out/abl_sgbm.log 2>&1
rc=$?
cat gpurun_out/abl8.log gpurun_out/abl14.log gpurun_out/abl_sgbm.log | grep flags
exit $rc
