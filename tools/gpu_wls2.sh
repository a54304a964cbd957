set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -m pytest tests/test_gpu_wls.py -q -x > gpurun_out/ptw.log 2>&1; rc=$?; tail -3 gpurun_out/ptw.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/wls_ablate.py
