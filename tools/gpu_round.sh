#!/bin/bash
# Round-end evidence on one GPU box, in two calls (each under gpurun's 20-minute cap):
#   bash tools/gpu_round.sh <tag> A : smoke -> GPU tests -> rocprofv3 kernel stats + PMC
#       traffic (separate FETCH/WRITE passes) + SQ counters for the headline (census8), the
#       parity mode (sgbm5) and Middlebury -> their benches with those files
#   bash tools/gpu_round.sh <tag> T : part A without smoke, tests and kernel stats
#   bash tools/gpu_round.sh <tag> P : part A without smoke, tests, valu_rate and the single-pair run
#   bash tools/gpu_round.sh <tag> B : the other bench modes / engines / configs
# Each GPU step is time-limited; a failure (other than pytest's rc 1) stops the script.
set -u
TAG=${1:-r04}; PART=${2:-A}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
if [ "$PART" = A ] || [ "$PART" = T ] || [ "$PART" = P ]; then
  if [ "$PART" = A ]; then
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider
  fi
  # (name, config, mode, extra bench arguments): the headline, the parity mode, Middlebury
  for spec in "census8 kitti census8" "sgbm5 kitti sgbm5" "middlebury middlebury census8 --pairs-per-gpu 4"; do
    set -- $spec; m=$1; cfg=$2; md=$3; shift 3; X="$*"
    [ "$PART" = T ] || step prof_$m 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$m" -o run --output-format csv -- python3 bench.py --config $cfg --mode $md $X --steps 10 --warmup 2 --cpu-baseline-pairs 0 --host-surface-calls 0
    [ "$PART" = T ] || find "$OUT/prof_$m" -name "*kernel_stats.csv" -exec cp {} "$OUT/${m}_kernel_stats.csv" \;
    BENCH_EXTRA="$X" step traffic_$m 300 bash tools/traffic.sh $cfg $md
    cp gpurun_out/traffic/summary.json "$OUT/${m}_traffic.json"
    BENCH_EXTRA="$X" step valu_$m 300 bash tools/valu.sh $cfg $md
    cp gpurun_out/valu/summary.json "$OUT/${m}_valu.json"
    rm -rf gpurun_out/traffic gpurun_out/valu "$OUT/prof_$m"
  done
  cp "$OUT/census8_traffic.json" profiles/traffic_latest.json
  cp "$OUT/census8_valu.json" profiles/valu_latest.json
  [ "$PART" = A ] && step valu_rate 120 ./tools/ubench/valu_rate
  [ "$PART" = A ] && FLAGS=0 step single 400 bash tools/gpu_single.sh $TAG
  step bench 400 python -u bench.py --traffic-file "$OUT/census8_traffic.json"
  step bench_sgbm5 400 python -u bench.py --mode sgbm5 --traffic-file "$OUT/sgbm5_traffic.json" --valu-file "$OUT/sgbm5_valu.json"
  step bench_middlebury 400 python -u bench.py --config middlebury --pairs-per-gpu 4 --steps 40 --warmup 4 --cpu-baseline-pairs 0 --host-surface-calls 0 --traffic-file "$OUT/middlebury_traffic.json" --valu-file "$OUT/middlebury_valu.json"
else
  step bench_census8_perdir 300 python -u bench.py --engine perdir --cpu-baseline-pairs 0 --host-surface-calls 0
  step bench_sgbm5_perdir 300 python -u bench.py --mode sgbm5 --engine perdir --cpu-baseline-pairs 0 --host-surface-calls 0
  for m in sgbm8 volume8 disparity5 bm; do step bench_$m 300 python -u bench.py --mode $m --host-surface-calls 0; done
  step bench_tsukuba 300 python -u bench.py --config tsukuba --mode sgbm5 --host-surface-calls 0
fi
echo done
