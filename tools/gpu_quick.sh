#!/bin/bash
# Quick GPU iteration: GPU parity tests, then path-kernel ablations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pt_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pt_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop rc=$rc"; exit $rc; fi
timeout -k 10 300 python tools/ablate.py ${ABLATE_ARGS:-} > gpurun_out/ablate_$TAG.log 2>&1; rc2=$?; grep flags gpurun_out/ablate_$TAG.log; tail -2 gpurun_out/ablate_$TAG.log
exit $rc2
