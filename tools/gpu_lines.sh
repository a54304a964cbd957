#!/bin/bash
# In-sweep E/W lines: their GPU tests, then census8 / sgbm5 benches (optionally another library:
# LIB=var/lib_x.so).  bash tools/gpu_lines.sh <tag> [pytest -k expr]
set -u
TAG=${1:-lines}; K=${2:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
[ -n "${LIB:-}" ] && export STEREO_MATCH_AMD_LIB=$PWD/$LIB
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_round5.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider ${K:+-k "$K"} > "$OUT/t.log" 2>&1; rc=$?; tail -3 "$OUT/t.log"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
for m in ${MODES:-census8 sgbm5}; do
  timeout -k 10 200 python -u bench.py --mode $m --cpu-baseline-pairs 0 --host-surface-calls 0 --steps ${STEPS:-200} \
    ${BENCH_EXTRA:-} > "$OUT/$m.log" 2>&1 || exit $?
done
python tools/bsum.py "$OUT"/*.log
