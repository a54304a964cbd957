"""Summarise tools/valu.sh SQ counters per kernel and bench stage.

VALU issue fraction of a kernel = SQ_INSTS_VALU x ISSUE_CYCLES / (SIMDs x kernel
cycles), with kernel cycles = GRBM_GUI_ACTIVE / XCDs (GRBM_GUI_ACTIVE counts busy
cycles on every XCD) and ISSUE_CYCLES = 4: a SIMD issues at most one wave64 VALU
instruction per ~4 cycles whatever the number of waves (MI355X_MICROARCH.md
constants table 'vector-instruction ISSUE cost' v_add 4; tools/ubench/valu_rate.hip
measures 4.6-5.1 cycles per instruction per SIMD at 2-4 waves per SIMD with 8
independent chains, profiles/r03/valu_rate.log).  SQ_WAVE_CYCLES / SQ_WAIT_ANY /
SQ_ACTIVE_INST_ANY count quad-cycles (MI355X_MICROARCH.md).
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (source_hash: the stamp bench.py checks before using these numbers)

ISSUE_CYCLES = 4
SIMDS = 1024
XCDS = 8

out, config, mode = sys.argv[1], sys.argv[2], sys.argv[3]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {"config": config, "mode": mode, "kernels": {}, "issue_cycles_per_instr": ISSUE_CYCLES, "simds": SIMDS,
           "source": "rocprofv3 --pmc SQ_INSTS_VALU ... GRBM_GUI_ACTIVE over bench.py (tools/valu.sh); "
                     "frac = SQ_INSTS_VALU * 4 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8 XCDs)"}
sweep = any("k_sweep" in n for n in vals)
for k, d in vals.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / XCDS
    e = {c.lower(): v for c, v in m.items()}
    e["kernel_cycles"] = cyc
    e["valu_issue_frac"] = m["SQ_INSTS_VALU"] * ISSUE_CYCLES / (SIMDS * cyc) if cyc else None
    if m.get("SQ_WAVE_CYCLES"):
        e["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"]
        e["active_frac"] = m.get("SQ_ACTIVE_INST_ANY", 0) / m["SQ_WAVE_CYCLES"]
    summary["kernels"][k] = e
    stage = bench.kernel_stage(k, vals)
    if stage:  # a stage's kernels summed (instructions and the cycles of its launches)
        st = summary.setdefault("stages", {}).get(stage)
        if st is None:
            summary["stages"][stage] = dict(e, kernel=k)
        else:
            st["kernel"] += " + " + k
            for c in ("sq_insts_valu", "sq_waves", "sq_wave_cycles", "sq_wait_any", "sq_active_inst_any", "kernel_cycles"):
                if c in e and c in st:
                    st[c] += e[c]
            st["valu_issue_frac"] = st["sq_insts_valu"] * ISSUE_CYCLES / (SIMDS * st["kernel_cycles"]) \
                if st.get("kernel_cycles") else None
            if st.get("sq_wave_cycles"):
                st["wait_any_frac"] = st.get("sq_wait_any", 0) / st["sq_wave_cycles"]
                st["active_frac"] = st.get("sq_active_inst_any", 0) / st["sq_wave_cycles"]
summary["pairs_per_launch"] = None
for line in open(out + "/pmc.log"):
    if line.startswith("{"):
        try:
            summary["pairs_per_launch"] = json.loads(line)["roofline"]["pairs_per_launch"]
        except (ValueError, KeyError):
            pass
summary["engine"] = "sweep" if sweep else "perdir"
summary["src_sha16"] = bench.source_hash()
json.dump(summary, open(out + "/summary.json", "w"), indent=1)
print(json.dumps({k: v for k, v in summary.items() if k != "kernels"}, indent=1))
