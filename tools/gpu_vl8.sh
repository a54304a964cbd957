#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/vl8; mkdir -p $O
timeout -k 10 200 python -u tools/ablate.py --flags 16384 --rounds 3 > $O/base_c8.log 2>&1 || exit $?
for v in vl8 vl8n5; do
STEREO_MATCH_AMD_LIB=tools/exp/lib$v.so timeout -k 10 200 python -u tools/ablate.py --flags 16384 --rounds 3 > $O/${v}_c8.log 2>&1 || exit $?
STEREO_MATCH_AMD_LIB=tools/exp/lib$v.so timeout -k 10 200 python -u tools/ablate.py --mode sgbm5 --flags 0 --rounds 3 > $O/${v}_s5.log 2>&1 || exit $?
done
grep -h flags $O/*.log
