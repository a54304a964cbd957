"""Recompute the per-stage sums of a tools/traffic.sh or tools/valu.sh summary JSON from its
per-kernel entries with bench.kernel_stage (after a change of the stage mapping; the counters
themselves are untouched).  python tools/restage.py profiles/r05/sgbm5_traffic.json ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ISSUE_CYCLES, SIMDS = 4, 1024

for path in sys.argv[1:]:
    s = json.load(open(path))
    names = list(s["kernels"])
    stages = {}
    for k, e in s["kernels"].items():
        stage = bench.kernel_stage(k, names)
        if not stage:
            continue
        if "hbm_bytes" in e:  # traffic summary
            st = stages.setdefault(stage, {"kernel": "", "hbm_bytes_per_launch": 0.0, "read_bytes": 0.0,
                                           "write_bytes": 0.0})
            st["kernel"] = (st["kernel"] + " + " if st["kernel"] else "") + k
            st["hbm_bytes_per_launch"] += e.get("hbm_bytes") or 0
            st["read_bytes"] += e.get("read_bytes_corrected") or 0
            st["write_bytes"] += e.get("write_bytes") or 0
        else:  # SQ counter summary
            st = stages.get(stage)
            if st is None:
                stages[stage] = dict(e, kernel=k)
                continue
            st["kernel"] += " + " + k
            for c in ("sq_insts_valu", "sq_waves", "sq_wave_cycles", "sq_wait_any", "sq_active_inst_any", "kernel_cycles"):
                if c in e and c in st:
                    st[c] += e[c]
            st["valu_issue_frac"] = st["sq_insts_valu"] * ISSUE_CYCLES / (SIMDS * st["kernel_cycles"]) \
                if st.get("kernel_cycles") else None
            if st.get("sq_wave_cycles"):
                st["wait_any_frac"] = st.get("sq_wait_any", 0) / st["sq_wave_cycles"]
                st["active_frac"] = st.get("sq_active_inst_any", 0) / st["sq_wave_cycles"]
    s["stages"] = stages
    json.dump(s, open(path, "w"), indent=1)
    print(path, {k: v["kernel"][:60] for k, v in stages.items()})
