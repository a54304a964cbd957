#!/bin/bash
# WLS smoother: exact fast pivot reciprocal; rows in registers (default build) vs LDS tiles
# (libsm_lds.so, -DWLS_ROWS_LDS=1): WLS parity tests, then single-pair and batched timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wls2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wls.py tests/test_gpu_round2.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -k "wls or compute_disparity or valid_result" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in default lds; do
  if [ $lib != default ]; then export STEREO_MATCH_AMD_LIB=$PWD/stereo_match_amd/libsm_lds.so; fi
  echo "== $lib"
  timeout -k 10 120 python tools/single_pair.py --flags 0 --calls 20 || exit 1
  timeout -k 10 200 python -u bench.py --mode disparity5 --steps 100 --warmup 5 --cpu-baseline-pairs 0 --host-surface-calls 0 > $OUT/b_$lib.log 2>&1 || exit 1
  grep '^{' $OUT/b_$lib.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('disparity5', round(d['value'],1), {k:round(v,1) for k,v in d['stage_us_per_pair'].items() if v})"
done
