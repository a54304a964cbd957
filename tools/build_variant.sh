#!/bin/bash
# Build the engine with extra compile definitions into var/lib_<name>.so (in-tree, git-ignored,
# travels to the GPU box); select it at run time with STEREO_MATCH_AMD_LIB.
#   tools/build_variant.sh ncw11 -DSWEEP_NCW=11
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; shift
OBJ=/tmp/smvar_$NAME; mkdir -p "$OBJ" "$ROOT/var"
SRC="$ROOT/stereo_match_amd/csrc"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall $*"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC $F -c -o "$OBJ/api.o" "$SRC/sm_api.hip" &
for m in 0 1 2 3 4; do
  $HIPCC $F -DSWEEP_MODE=$m -c -o "$OBJ/sw$m.o" "$SRC/sm_sweep.hip" &
  $HIPCC $F -DSWEEP_MODE=$m -DSWEEP_WIDE=1 -c -o "$OBJ/sww$m.o" "$SRC/sm_sweep.hip" &
  $HIPCC $F -DSWEEP_MODE=$m -DSWEEP_WIDE=2 -c -o "$OBJ/swl$m.o" "$SRC/sm_sweep.hip" &
done
$HIPCC $F -c -o "$OBJ/ew.o" "$SRC/sm_ew.hip" &
wait
$HIPCC --offload-arch=gfx950 -fPIC -shared -o "$ROOT/var/lib_$NAME.so" "$OBJ"/api.o "$OBJ"/sw[0-4].o "$OBJ"/sww[0-4].o "$OBJ"/swl[0-4].o "$OBJ"/ew.o
echo "built var/lib_$NAME.so"
