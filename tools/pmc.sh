#!/bin/bash
# PMC passes (separate rocprofv3 runs, --pmc with kernel-trace only) over tools/ablate.py.
# Usage: bash tools/pmc.sh <tag> <ablate flags> ["pass1 counters" "pass2 counters" ...]
# env: MODE (ablate --mode, default census8), KF (kernel-name regex, default paths|wta|sweep)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; FLAGS=$2; shift 2
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d $OUT/p$i -o run --output-format csv -- python tools/ablate.py --mode ${MODE:-census8} --flags $FLAGS --rounds 1 --pairs 8 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - "$OUT" "${KF:-paths|wta|sweep}" <<'PY'
import csv, glob, re, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if not re.search(sys.argv[2], k): continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
