# GPU tests of the round-5/6/2 suites, then the one-pair call A/B: current library vs var/lib_<v>.so
set -u
mkdir -p gpurun_out/f gpurun_out/q
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_round6.py tests/test_gpu_round2.py > gpurun_out/f/t5.log 2>&1
rc=$?; tail -2 gpurun_out/f/t5.log; [ $rc -eq 0 ] || exit $rc
for v in full $1 full $1; do
  if [ $v = full ]; then L=""; else L="STEREO_MATCH_AMD_LIB=$PWD/var/lib_$v.so"; fi
  env $L timeout -k 10 200 python3 tools/single_pair.py --calls 40 --stages call --runs "0" > gpurun_out/q/sp_$v.log 2>&1 || exit 3
  python3 -c "
import json
for l in open('gpurun_out/q/sp_$v.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', d['ms_per_call'], d.get('stage_us_per_call',{}).get('call'))"
done
