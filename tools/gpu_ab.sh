#!/bin/bash
# Ablation timing: bash tools/gpu_ab.sh <mode> <flags,...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python tools/ablate.py --mode "$1" --flags "$2" --rounds 3
