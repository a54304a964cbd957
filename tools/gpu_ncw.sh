#!/bin/bash
# sweep strip width (own waves per workgroup) and hand-off ablations
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ncw; mkdir -p $O
timeout -k 10 200 python -u tools/ablate.py --flags 16384,16793600,33570816 --rounds 3 > $O/base_c8.log 2>&1 || exit $?
for n in 9 11 13 15; do
  STEREO_MATCH_AMD_LIB=tools/exp/libncw$n.so timeout -k 10 200 python -u tools/ablate.py --flags 16384 --rounds 3 > $O/ncw${n}_c8.log 2>&1 || exit $?
  STEREO_MATCH_AMD_LIB=tools/exp/libncw$n.so timeout -k 10 200 python -u tools/ablate.py --mode sgbm5 --flags 0 --rounds 3 > $O/ncw${n}_s5.log 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/ablate.py --mode sgbm5 --flags 0,16777216,33554432 --rounds 3 > $O/base_s5.log 2>&1 || exit $?
grep -h flags $O/*.log
