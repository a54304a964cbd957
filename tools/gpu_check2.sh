#!/bin/bash
# GPU suite (new round-2 tests first) + headline bench; each step time-limited, stop on failure
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-c2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_round2.py -x -v --timeout 300 --timeout-method thread > $O/pt_r2.log 2>&1; rc=$?
tail -25 $O/pt_r2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt_all.log 2>&1; rc=$?
tail -5 $O/pt_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -c 300 $O/bench.log
