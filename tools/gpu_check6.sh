set -u
mkdir -p gpurun_out/c1
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_round6.py tests/test_gpu_round2.py tests/test_gpu_wls.py tests/test_gpu_parity.py tests/test_gpu_round5.py tests/test_gpu_wta.py > gpurun_out/c1/t.log 2>&1; rc=$?
tail -2 gpurun_out/c1/t.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python3 tools/single_pair.py --calls 30 --stages call --runs "0;0" > gpurun_out/c1/sp1.log 2>&1 || exit 3
timeout -k 10 300 python3 tools/single_pair.py --calls 30 --stages call,h2d,d2h --runs "0;0" > gpurun_out/c1/sp2.log 2>&1 || exit 3
grep -h "^{" gpurun_out/c1/sp1.log gpurun_out/c1/sp2.log | cut -c1-60,200-400
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --cpu-baseline-pairs 0 > gpurun_out/c1/b.log 2>&1 || exit 3
python3 -c "
import json; l=[x for x in open('gpurun_out/c1/b.log') if x.startswith('{')][-1]; d=json.loads(l); hs=d['host_surface']; s=d['stage_us_per_pair']
print(d['value'], {k: round(v,1) for k,v in s.items() if v}); print(hs['value'], hs['ms_per_call_median'], hs['device_ms_per_call'], hs['one_call_abi']['device_ms_per_call'], hs['one_call_abi']['value'])"
