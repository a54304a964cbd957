#!/bin/bash
# Scratch (spill) bytes and VGPRs of every fused-sweep instance (all modes, strip widths), from the
# compiler's resource remarks: the host refuses a wide / MODE 3 instance that uses scratch, so a
# spill silently moves a configuration to another engine.
# Usage: bash tools/spills.sh [out.txt]   (one line per kernel: wide mode name vgprs scratch)
SRC="$(cd "$(dirname "$0")/../stereo_match_amd/csrc" && pwd)"
OUT=${1:-/dev/stdout}
T=$(mktemp -d)
for w in 0 1 2; do for m in 0 1 2 3 4; do
  (cd "$SRC" && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -DSWEEP_MODE=$m -DSWEEP_WIDE=$w -c \
     -o $T/o_$w$m.o sm_sweep.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
   sed 's/ *\[-Rpass-analysis=kernel-resource-usage\]//' |
   awk -v w=$w -v m=$m '/Function Name:/ {n=$NF} / VGPRs:/ {v=$NF} /ScratchSize/ {print "wide=" w, "mode=" m, n, "vgpr=" v, "scratch=" $NF}' \
   > $T/r_$w$m.txt) &
done; done; wait
cat $T/r_*.txt | sed 's/_ZN3smk7k_sweepI//;s/EEvNS_9SweepArgsE//' | sort > "$OUT"
rm -rf "$T"
