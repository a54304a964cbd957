# A/B of library variants on one box: bash tools/ab_ds.sh <tag> <variant|full>...
set -u
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for r in 1 2; do for v in "$@"; do
  if [ $v = full ]; then L=""; else L="STEREO_MATCH_AMD_LIB=$PWD/var/lib_$v.so"; fi
  env $L timeout -k 10 120 python -u bench.py --steps 200 --warmup 10 --cpu-baseline-pairs 0 --host-surface-calls 0 ${BENCH_ARGS:-} > gpurun_out/$TAG/$v.$r.log 2>&1 || exit 3
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/$TAG/$v.$r.log') if x.startswith('{')][-1]; d=json.loads(l); s=d['stage_us_per_pair']; print('$v', round(d['value']), {k: round(x,1) for k,x in s.items() if x and k not in ('total','paths','wta')})"
done; done
