#!/bin/bash
# GPU test suite + smoke (one process each, time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tests; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 780 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; fi; exit $rc
