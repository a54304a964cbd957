#!/bin/bash
# rocprofv3 kernel stats of one bench mode: bash tools/prof.sh <mode> <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODE=${1:-census8}; TAG=${2:-p}
OUT=gpurun_out/prof_${MODE}_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 bench.py --mode "$MODE" --steps 10 --warmup 2 --cpu-baseline-pairs 0 > "$OUT/bench.log" 2>&1 || exit $?
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
python3 tools/kstats.py "$OUT/kernel_stats.csv" 2>/dev/null || head -20 "$OUT/kernel_stats.csv"
