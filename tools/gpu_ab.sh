# bench A/B over --tune strings: bash tools/gpu_ab.sh <mode> "<tune1>" "<tune2>" ...  ("-" = none)
set -u
mode=$1; shift
mkdir -p gpurun_out/ab
i=0
for t in "$@"; do
  i=$((i+1)); arg=""; [ "$t" != "-" ] && arg="--tune $t"
  timeout -k 10 200 python -u bench.py --mode $mode --steps 300 --warmup 10 --cpu-baseline-pairs 0 --host-surface-calls 0 $arg > gpurun_out/ab/${mode}_$i.log 2>&1 || exit 3
  python3 -c "
import json; l=[x for x in open('gpurun_out/ab/${mode}_$i.log') if x.startswith('{')][-1]; d=json.loads(l); s=d['stage_us_per_pair']
print('$mode', '$t', round(d['value']), {k: round(v,1) for k,v in s.items() if v and k not in ('total','paths','wta','median')})"
done
