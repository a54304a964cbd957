# quick A/B numbers on one box: census8 and sgbm5 benches (stage split) and the one-pair call
set -u
mkdir -p gpurun_out/q
for m in census8 sgbm5; do
  timeout -k 10 200 python -u bench.py --mode $m --steps 200 --warmup 10 --cpu-baseline-pairs 0 --host-surface-calls 0 ${BENCH_ARGS:-} > gpurun_out/q/$m.log 2>&1 || exit 3
  python3 -c "
import json; l=[x for x in open('gpurun_out/q/$m.log') if x.startswith('{')][-1]; d=json.loads(l); s=d['stage_us_per_pair']
print('$m', round(d['value']), {k: round(v,1) for k,v in s.items() if v and k not in ('total','paths','wta')}, d['counters'].get('ew_repairs_per_pair'))"
done
timeout -k 10 300 python3 tools/single_pair.py --calls 30 --stages call --runs "0" > gpurun_out/q/sp.log 2>&1 || exit 3
grep "^{" gpurun_out/q/sp.log | cut -c1-40,200-300
