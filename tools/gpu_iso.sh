#!/bin/bash
# isolated stage times: E/W alone (perdir, skip vertical), down sweep alone (sweep, skip E/W)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/iso; mkdir -p $O
timeout -k 10 200 python -u tools/ablate.py --flags 16384,4098,4097,16385 --rounds 3 > $O/c8.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ablate.py --mode sgbm5 --flags 0,4098,1 --rounds 3 > $O/s5.log 2>&1 || exit $?
grep -h flags $O/*.log
