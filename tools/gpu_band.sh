#!/bin/bash
# Row bands: the round-6 tests, then the one-pair call's kernels under rocprofv3
# (kernel stats) and its stage timing for band settings.  bash tools/gpu_band.sh <tag> [runs]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/band_${1:-x}; mkdir -p "$OUT"
RUNS=${2:-"0/bands=1;0"}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_round6.py ${TESTS:-} > "$OUT/t.log" 2>&1; rc=$?
tail -n 3 "$OUT/t.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 tools/single_pair.py --runs 0 --calls 30 > "$OUT/prof.log" 2>&1 || exit $?
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -20
timeout -k 10 300 python3 tools/single_pair.py --calls 20 --runs "$RUNS" > "$OUT/sp.log" 2>&1 || exit $?
grep "^{" "$OUT/sp.log"
