#!/bin/bash
# GPU parity tests + ablations for both modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pt_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pt_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop rc=$rc"; exit $rc; fi
timeout -k 10 200 python tools/ablate.py --flags 0,64 --rounds 3 > gpurun_out/ab_c_$TAG.log 2>&1 || exit $?
grep flags gpurun_out/ab_c_$TAG.log
timeout -k 10 200 python tools/ablate.py --mode sgbm5 --flags 0,4 --rounds 3 > gpurun_out/ab_s_$TAG.log 2>&1 || exit $?
grep flags gpurun_out/ab_s_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline-pairs 0 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline-pairs 0 --mode sgbm5 > gpurun_out/bench_s_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_s_$TAG.log
