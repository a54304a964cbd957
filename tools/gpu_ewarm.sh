# E/W segment warmup A/B (SM_TUNE_EW_WARMUP) for the 8-pair sgbm5 and census8 benches
set -u
mkdir -p gpurun_out/ew
run() { timeout -k 10 200 python -u bench.py --mode $1 --steps 300 --warmup 10 --cpu-baseline-pairs 0 --host-surface-calls 0 --tune ew_warmup=$2 > gpurun_out/ew/$1_$2.log 2>&1 || exit 3
  python3 -c "
import json; l=[x for x in open('gpurun_out/ew/$1_$2.log') if x.startswith('{')][-1]; d=json.loads(l); s=d['stage_us_per_pair']
print('$1 warm=$2', round(d['value']), {k: round(v,1) for k,v in s.items() if v and k in ('sweep','horizontal','sweep_wta')}, d['counters'].get('ew_repairs_per_pair'))"; }
for w in ${SG_W:-24 16 32 40 48 24}; do run sgbm5 $w; done
for w in ${CE_W:-16 8 24 32 16}; do run census8 $w; done
