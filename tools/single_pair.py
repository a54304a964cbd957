"""Single-pair latency of the reference surface (one pair per call, as
stereo_vision.py:178-182 runs it): stage breakdown of sm_compute_disparity at
settings.ini values (D=160) for each engine flag set.
    python tools/single_pair.py [--flags 0,4096] [--calls 20] [--runs "0/ew=16;16384/ncw=5"]
A run is debug flags, then /knob=value items (ew: SM_TUNE_EW_LANES, ncw: SM_TUNE_SWEEP_NCW,
bands: SM_TUNE_BANDS, bw: SM_TUNE_BAND_WARMUP, eww: SM_TUNE_EW_WARMUP, cw: SM_TUNE_COST_WGS);
--runs replaces --flags."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="0,4096")
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--D", type=int, default=160)
    ap.add_argument("--runs", default="")
    ap.add_argument("--stages", default="", help="comma list: time only these stages (e.g. call); default all")
    args = ap.parse_args()
    import stereo_match_amd as sm
    from stereo_match_amd import _lib, synthetic, wls
    from stereo_match_amd.stereo_vision import matcher_from_settings

    s = dict(sm.DEFAULT_SETTINGS, window_size=5, num_disparities=args.D)
    H, W = synthetic.CONFIGS["kitti"][:2]
    gl, gr, _ = synthetic.random_dot_pair(H, W, args.D, seed=77)
    lm = matcher_from_settings(s)
    prm = lm.params()
    wf = wls.createDisparityWLSFilter(lm)
    wf.setLambda(s["lmbda"])
    wf.setSigmaColor(s["sigma"])
    wp = wf.params(H, W)
    e = _lib.Engine(0)
    ref = None
    knobs = {"ew": e.TUNE_EW_LANES, "ncw": e.TUNE_SWEEP_NCW, "bands": e.TUNE_BANDS, "bw": e.TUNE_BAND_WARMUP,
             "eww": e.TUNE_EW_WARMUP, "cw": e.TUNE_COST_WGS, "stag": e.TUNE_LR_STAGGER}
    runs = args.runs.split(";") if args.runs else args.flags.split(",")
    for run in runs:
        parts = run.split("/")
        f = int(parts[0])
        tune = {k: int(v) for k, v in (p.split("=") for p in parts[1:])}
        e.set_debug_flags(f)
        for k in knobs:
            e.set_tuning(knobs[k], tune.get(k, 0))
        d, fl = e.compute_disparity(gl, gr, prm, wp)
        if ref is None:
            ref = (d, fl)
        same = bool(np.array_equal(d, ref[0]) and np.array_equal(fl, ref[1]))
        e.set_timing(True, stages=args.stages.split(",") if args.stages else None)
        e.reset_timing()
        c0 = e.counters()
        ts = []
        for _ in range(args.calls):
            t0 = time.perf_counter()
            e.compute_disparity(gl, gr, prm, wp)
            ts.append(time.perf_counter() - t0)
        st = e.timing()
        e.set_timing(False)
        c1 = e.counters()
        print(json.dumps({"run": run, "same_as_first": same, "ms_per_call": round(float(np.median(ts)) * 1e3, 3),
                          "counters_per_call": {k: (c1[k] - c0[k]) / args.calls for k in c1 if c1[k] != c0[k]},
                          "stage_us_per_call": {k: round(v[0] * 1e3 / args.calls, 1) for k, v in st.items() if v[0] > 0}}))


if __name__ == "__main__":
    main()
