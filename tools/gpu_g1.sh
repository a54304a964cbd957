set -u
mkdir -p gpurun_out/g1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/g1/bench.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1; echo pytest rc=$?
tail -3 gpurun_out/g1/pytest.log
