#!/bin/bash
# Rebuild only sm_api.hip with extra compile definitions and link it with the main build's
# sweep / E/W objects into var/lib_<name>.so (select with STEREO_MATCH_AMD_LIB).  For
# knobs that live in sm_api.hip and the headers it includes (cost kernels, launch shapes).
#   tools/build_api_variant.sh pf4 -DPREFILTER_ROWS=4
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; shift
SRC="$ROOT/stereo_match_amd/csrc"
make -s -C "$SRC" >/dev/null  # the shared objects must exist
mkdir -p "$ROOT/var"
OBJ=/tmp/smapi_$NAME.o
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall "$@" -c -o "$OBJ" "$SRC/sm_api.hip"
$HIPCC --offload-arch=gfx950 -fPIC -shared -o "$ROOT/var/lib_$NAME.so" "$OBJ" "$SRC"/sm_sweep_[mw][0-2].o "$SRC/sm_ew.o"
echo "built var/lib_$NAME.so"
