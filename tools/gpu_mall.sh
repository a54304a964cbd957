#!/bin/bash
# MALL-residency probe: vertical-only / horizontal-only per-direction launches at group caps 1, 2, 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mall; mkdir -p $O
timeout -k 10 300 python -u tools/ablate.py --flags 4096,4097,69633,135169,266241,4098,69634,135170 --rounds 3 > $O/c8.log 2>&1 || exit $?
grep -h flags $O/*.log
