#!/bin/bash
# Packed E/W lines: GPU parity suite, then census8 / sgbm5 / sgbm8 timings of the E/W variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ew; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; fi
for m in census8 sgbm5 sgbm8; do
  F=$([ $m = census8 ] && echo "16384,$((16384|256)),$((16384|128)),$((16384|384))" || echo "0,256,128,384")
  timeout -k 10 120 python tools/ablate.py --mode $m --pairs 8 --rounds 3 --flags $F > $OUT/$m.log 2>&1 || { cat $OUT/$m.log; exit 1; }
  echo "== $m"; cat $OUT/$m.log
done
