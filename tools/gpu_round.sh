#!/bin/bash
# Round-end evidence on one GPU box: smoke -> GPU tests -> bench (census8) ->
# rocprofv3 kernel stats -> PMC traffic (separate FETCH/WRITE passes) -> bench
# again (now carrying roofline.traffic).  Each GPU step time-limited; a
# failure (other than pytest's rc 1) stops the script.
set -u
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench 600 python bench.py
step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline-pairs 0
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
step traffic 700 bash tools/traffic.sh kitti census8
cp gpurun_out/traffic/summary.json "$OUT/traffic.json"
cp gpurun_out/traffic/summary.json profiles/traffic_latest.json
step bench2 600 python bench.py
for m in sgbm5 volume8 disparity5; do step bench_$m 600 python bench.py --mode $m; done
echo done
