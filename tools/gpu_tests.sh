#!/bin/bash
# GPU test subset: bash tools/gpu_tests.sh <tag> <pytest args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -m pytest -q -x "$@" > gpurun_out/pt_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/pt_$TAG.log
exit $rc
