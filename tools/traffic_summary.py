"""Summarise tools/traffic.sh counter CSVs: mean HBM bytes per dispatch per kernel.

FETCH_SIZE / WRITE_SIZE are kilobytes; gfx950 FETCH_SIZE reads half the bytes
of a wide coalesced stream (MI355X_MICROARCH.md §HBM), so reads = 2*FETCH_SIZE.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (source_hash: the stamp bench.py checks before using these numbers)

out, config, mode = sys.argv[1], sys.argv[2], sys.argv[3]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {"config": config, "mode": mode, "kernels": {},
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; "
                     "reads = 2*FETCH_SIZE on gfx950 (MI355X_MICROARCH.md)"}
for k, d in vals.items():
    fs = sum(d["FETCH_SIZE"]) / max(len(d["FETCH_SIZE"]), 1) if "FETCH_SIZE" in d else None
    ws = sum(d["WRITE_SIZE"]) / max(len(d["WRITE_SIZE"]), 1) if "WRITE_SIZE" in d else None
    rd = 2 * fs * 1024 if fs is not None else None
    wr = ws * 1024 if ws is not None else None
    summary["kernels"][k] = {"fetch_size_kb": fs, "write_size_kb": ws, "read_bytes_corrected": rd,
                             "write_bytes": wr, "hbm_bytes": (rd or 0) + (wr or 0)}
    sweep = any("k_sweep" in n for n in vals)  # fused-sweep engine
    targs = [t.strip() for t in k.split("<", 1)[1].split(">")[0].split(",")] if "<" in k else []
    fallback = bool(targs) and targs[-1] == "true" and ("k_sgm_paths" in k or "k_wta" in k)  # guarded instances
    if "k_sweep2<" in k or "k_sweep<" in k:  # sweep mode: 0 = down partial, 1/2 = with WTA
        stage = "sweep" if targs[4 if "k_sweep2<" in k else 3] == "0" else "sweep_wta"
    elif fallback:
        stage = None
    else:
        stage = ("horizontal" if "k_ew<" in k or (sweep and "k_sgm_paths" in k) else "paths" if "k_sgm_paths" in k
                 else "wta" if ("k_wta" in k or "k_row_wta" in k)
                 else "cost" if any(c in k for c in ("k_census9x7", "k_sgbm_cost(", "k_cost_volume_f32")) else None)
    if stage:
        summary.setdefault("stages", {})[stage] = {"kernel": k, "hbm_bytes_per_launch": (rd or 0) + (wr or 0),
                                                   "read_bytes": rd, "write_bytes": wr}
# pairs per launch of the profiled run, from the bench line it printed (launch groups can
# be smaller than --pairs-per-gpu: sm_api.hip group_size)
summary["pairs_per_launch"] = None
for log in glob.glob(out + "/*.log"):
    for line in open(log):
        if line.startswith("{"):
            try:
                summary["pairs_per_launch"] = json.loads(line)["roofline"]["pairs_per_launch"]
            except (ValueError, KeyError):
                pass
summary["engine"] = "sweep" if any("k_sweep" in n for n in vals) else "perdir"
summary["src_sha16"] = bench.source_hash()
json.dump(summary, open(out + "/summary.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
