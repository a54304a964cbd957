#!/bin/bash
# Build an experimental variant of the engine library with extra sweep-kernel
# defines into tools/exp/lib<tag>.so (timed by tools/gpu_abl_quick.sh).
#   bash tools/build_exp.sh <tag> -DSWEEP_NOPOLL ...
set -eu
cd "$(dirname "$0")/../stereo_match_amd/csrc"
tag=$1; shift
make -j4 sm_api.o > /dev/null
mkdir -p ../../tools/exp
for m in 0 1 2; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC "$@" -DSWEEP_MODE=$m -c -o /tmp/exp_${tag}_$m.o sm_sweep.hip 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o ../../tools/exp/lib$tag.so sm_api.o /tmp/exp_${tag}_0.o /tmp/exp_${tag}_1.o /tmp/exp_${tag}_2.o
echo "built tools/exp/lib$tag.so"
