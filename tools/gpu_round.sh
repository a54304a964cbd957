#!/bin/bash
# Round-end evidence on one GPU box: smoke -> GPU tests -> headline bench ->
# rocprofv3 kernel stats + PMC traffic (separate FETCH/WRITE passes) for the
# headline (census8) and the parity mode (sgbm5, fused sweeps) -> the other
# bench modes.  Each GPU step time-limited; a failure (other than pytest's
# rc 1) stops the script.   bash tools/gpu_round.sh <tag>
set -u
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
for m in census8 sgbm5; do
  step prof_$m 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$m" -o run --output-format csv -- python3 bench.py --mode $m --steps 10 --warmup 2 --cpu-baseline-pairs 0
  find "$OUT/prof_$m" -name "*kernel_stats.csv" -exec cp {} "$OUT/${m}_kernel_stats.csv" \;
  step traffic_$m 500 bash tools/traffic.sh kitti $m
  cp gpurun_out/traffic/summary.json "$OUT/${m}_traffic.json"
  rm -rf gpurun_out/traffic
done
cp "$OUT/census8_traffic.json" profiles/traffic_latest.json
step bench 400 python -u bench.py --traffic-file "$OUT/census8_traffic.json"
step bench_sgbm5 400 python -u bench.py --mode sgbm5 --traffic-file "$OUT/sgbm5_traffic.json"
step bench_census8_sweep 300 python -u bench.py --engine sweep --cpu-baseline-pairs 0
step bench_sgbm5_perdir 300 python -u bench.py --mode sgbm5 --engine perdir --cpu-baseline-pairs 0
for m in sgbm8 volume8 disparity5 bm; do step bench_$m 400 python -u bench.py --mode $m; done
step bench_middlebury 400 python -u bench.py --config middlebury --pairs-per-gpu 4 --cpu-baseline-pairs 0
echo done
