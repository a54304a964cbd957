#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/single; mkdir -p $O
timeout -k 10 300 python -u tools/single_pair.py --flags 0,4096,16384 > $O/single.log 2>&1 || exit $?
cat $O/single.log | grep flags
