#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wide; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 300 --timeout-method thread > $O/pt.log 2>&1; rc=$?
tail -40 $O/pt.log; exit $rc
