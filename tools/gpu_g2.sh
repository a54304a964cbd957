#!/bin/bash
# round-2 check: new bench line + launch-group-size ablation (MALL residency of the cost volume)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g2; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -c 600 $O/bench.log
timeout -k 10 300 python -u tools/ablate.py --flags 0,65536,131072,196608,262144,524288 --rounds 3 > $O/abl_perdir.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ablate.py --flags 16384,81920,147456,212992,278528,540672 --rounds 3 > $O/abl_sweep.log 2>&1 || exit $?
tail -20 $O/abl_perdir.log $O/abl_sweep.log
