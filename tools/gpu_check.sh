#!/bin/bash
# One GPU round-trip: the GPU test suite, then bench lines of every mode (short), each step
# under its own time limit; stops at the first failure.  Usage: bash tools/gpu_check.sh TAG [tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r3}; TESTS=${2:-tests/}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
for m in census8 sgbm5 sgbm8 disparity5; do
  timeout -k 10 240 python bench.py --mode $m --steps 100 --warmup 10 --cpu-baseline-pairs 0 --host-surface-calls 0 > $OUT/bench_$m.jsonl 2> $OUT/bench_$m.err
  rc=$?; if [ $rc -ne 0 ]; then echo "bench $m rc=$rc"; tail -5 $OUT/bench_$m.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$m.jsonl').read().strip().splitlines()[-1]); print('$m', round(d['value'],1), 'pairs/s', 'pipe', round(d['pipeline_roofline']['frac'],3), {k: round(v,1) for k,v in d['stage_us_per_pair'].items() if v})"
done
