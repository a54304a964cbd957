#!/bin/bash
# Round-2 evidence, part A: smoke -> GPU tests -> headline bench.  Each GPU step
# time-limited; a failure other than pytest's rc 1 stops the script.
set -u
TAG=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 780 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider
step bench 300 python -u bench.py
echo done
