#!/bin/bash
# k_sweep2: GPU parity suite, then census8 sweep timings (k_sweep2 nw=4 / nw=2 / k_sweep) at 4 and 8 pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sw3; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; fi
for P in 4 8; do
  timeout -k 10 120 python tools/ablate.py --mode census8 --pairs $P --rounds 3 --flags 0,16384,$((16384|(1<<27))),$((16384|128)) > $OUT/census8_p$P.log 2>&1 || { cat $OUT/census8_p$P.log; exit 1; }
  echo "== census8 P=$P"; cat $OUT/census8_p$P.log
done
