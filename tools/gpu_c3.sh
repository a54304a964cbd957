#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-c3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt_all.log 2>&1; rc=$?
tail -5 $O/pt_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/single_pair.py --flags 0,4096,16384 > $O/single.log 2>&1 || exit $?
grep flags $O/single.log
timeout -k 10 300 python -u bench.py --cpu-baseline-pairs 0 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --mode disparity5 --cpu-baseline-pairs 0 --host-surface-calls 0 > $O/bench_d5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --mode sgbm5 --cpu-baseline-pairs 0 --host-surface-calls 0 > $O/bench_s5.log 2>&1 || exit $?
for f in bench bench_d5 bench_s5; do python3 -c "
import json,sys; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), {k:round(v,1) for k,v in d['stage_us_per_pair'].items() if v>0}, d.get('host_surface',{}).get('value'))"; done
