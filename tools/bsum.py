"""One-line summaries of bench.py JSON lines: python tools/bsum.py gpurun_out/x/*.log"""
import json
import sys

for f in sys.argv[1:]:
    try:
        lines = [x for x in open(f) if x.startswith("{")]
    except OSError as e:
        print(f, e)
        continue
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])
    st = {k: round(v, 1) for k, v in d.get("stage_us_per_pair", {}).items() if v}
    print(f, round(d["value"], 1), "pipe", round(d["pipeline_roofline"]["frac"] or 0, 3), st,
          {k: d[k] for k in ("counters",) if k in d})
