#!/bin/bash
# Verify the tree on one GPU box: smoke -> GPU tests -> headline bench -> sgbm5 bench.
# Each step time-limited; a failure other than pytest's rc 1 stops the script.
#   bash tools/gpu_verify.sh <tag> [pytest -k expression]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v}
KEXPR=${2:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
if [ -n "$KEXPR" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR"
else
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
step bench 600 python -u bench.py
step bench_sgbm5 600 python -u bench.py --mode sgbm5
echo done
