#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprof kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
# Usage: bash tools/gpu_check.sh [tag] [pytest-args...]
set -u
TAG=${1:-r01}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>  (stdout/stderr -> $OUT/<name>.log)
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! stopping: $name rc=$rc"; exit $rc; fi
    return 0
}
rocminfo 2>/dev/null | grep -m1 -E "gfx9" ; nproc
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-}
step bench 600 python bench.py --steps 20 --warmup 3
step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-baseline-pairs 0
find "$OUT/prof" -name "*stats*.csv" -exec cp {} "$OUT/" \; 2>/dev/null
echo done
