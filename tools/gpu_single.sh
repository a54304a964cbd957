#!/bin/bash
# Single-pair latency evidence (the reference's one-pair-per-call surface):
# kernel trace + stats of tools/single_pair.py, its stage timing under engine flags,
# and the sgbm5 launch-group overlap ablation.  bash tools/gpu_single.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/single_${1:-x}; mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 tools/single_pair.py --flags 0 --calls 30 > "$OUT/prof.log" 2>&1 || exit $?
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/prof" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/prof"
timeout -k 10 240 python3 tools/single_pair.py --flags ${FLAGS:-0,16384,64} --calls 30 > "$OUT/flags.log" 2>&1 || exit $?
[ -n "${ABL:-}" ] && { timeout -k 10 300 python3 tools/ablate.py $ABL > "$OUT/ablate.log" 2>&1 || exit $?; }
echo done
