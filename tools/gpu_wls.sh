#!/bin/bash
# WLS parity tests + compute_disparity bench (each step time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -m pytest tests/test_gpu_wls.py -q -x > gpurun_out/ptw_$TAG.log 2>&1; rc=$?; tail -5 gpurun_out/ptw_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop rc=$rc"; exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --mode disparity5 --cpu-baseline-pairs 0 > gpurun_out/bench_disp_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_disp_$TAG.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_us_per_pair'])"
