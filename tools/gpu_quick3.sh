#!/bin/bash
# GPU parity tests + benches of the three modes (each step time-limited; stop on fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pt_$TAG.log 2>&1; rc=$?; tail -5 gpurun_out/pt_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop rc=$rc"; exit $rc; fi
for m in census8 sgbm5 volume8 disparity5; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 3 --mode $m > gpurun_out/bench_${m}_$TAG.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_${m}_$TAG.log
done
