# full GPU suite, then the quick benches (census8, sgbm5 stage split, one-pair call)
set -u
mkdir -p gpurun_out/f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f/t.log 2>&1
rc=$?; tail -3 gpurun_out/f/t.log; if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/f/t.log | head -20; exit $rc; fi
bash tools/gpu_quick.sh
