#!/bin/bash
# engine choice by launch-group size (sgbm5 / sgbm8 / census8): sweeps vs per-direction at caps 1..4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/gsz; mkdir -p $O
F=0,4096,65536,69632,131072,135168,196608,200704,262144,266240
timeout -k 10 300 python -u tools/ablate.py --mode sgbm5 --flags $F --rounds 3 > $O/s5.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ablate.py --mode sgbm8 --flags $F --rounds 3 > $O/s8.log 2>&1 || exit $?
F=4096,16384,69632,81920,135168,147456,266240,278528
timeout -k 10 300 python -u tools/ablate.py --mode census8 --flags $F --rounds 3 > $O/c8.log 2>&1 || exit $?
grep -h flags $O/*.log
