#!/bin/bash
# Sweep-engine changes: GPU parity suite, then per-stage timings (census8 sweeps at
# 2/4/8 pairs per launch, sgbm5, sgbm8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sw2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; fi
for P in 2 4 8; do
  timeout -k 10 120 python tools/ablate.py --mode census8 --pairs $P --rounds 3 --flags 0,16384 > $OUT/census8_p$P.log 2>&1 || { cat $OUT/census8_p$P.log; exit 1; }
  echo "== census8 P=$P"; cat $OUT/census8_p$P.log
done
for m in sgbm5 sgbm8; do
  timeout -k 10 120 python tools/ablate.py --mode $m --pairs 8 --rounds 3 --flags 0,4096 > $OUT/$m.log 2>&1 || { cat $OUT/$m.log; exit 1; }
  echo "== $m"; cat $OUT/$m.log
done
