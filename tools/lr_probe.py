"""Latency of small launch groups at settings.ini values (KITTI, D=160, MODE_SGBM):
device time per sm_compute_batch_device call for 1 and 2 pairs under each engine
flag, stage by stage.  The one-pair-per-call surface (stereo_vision.py:178-182)
runs two matchers of this shape per call.
    python tools/lr_probe.py [--runs "0;16384;16384/ew=16"] [--pairs 1,2] [--calls 30]
A run is debug flags, then /knob=value items (ew: SM_TUNE_EW_LANES, ncw: SM_TUNE_SWEEP_NCW)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", default="0;16384")
    ap.add_argument("--pairs", default="1,2")
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--D", type=int, default=160)
    args = ap.parse_args()
    import torch

    import stereo_match_amd as sm
    from stereo_match_amd import _lib, synthetic
    from stereo_match_amd.stereo_vision import matcher_from_settings

    s = dict(sm.DEFAULT_SETTINGS, window_size=5, num_disparities=args.D)
    H, W = synthetic.CONFIGS["kitti"][:2]
    prm = matcher_from_settings(s).params()
    e = _lib.Engine(0)
    npmax = max(int(x) for x in args.pairs.split(","))
    ls, rs = [], []
    for i in range(npmax):
        gl, gr, _ = synthetic.random_dot_pair(H, W, args.D, seed=100 + i)
        ls.append(gl)
        rs.append(gr)
    dl = torch.from_numpy(np.stack(ls)).cuda()
    dr = torch.from_numpy(np.stack(rs)).cuda()
    out = torch.empty((npmax, H, W), dtype=torch.int16, device="cuda")
    knobs = {"ew": e.TUNE_EW_LANES, "ncw": e.TUNE_SWEEP_NCW}
    first = {}  # npairs -> the first run's maps (every run must reproduce them)
    for run in args.runs.split(";"):
        parts = run.split("/")
        f = int(parts[0])
        tune = {k: int(v) for k, v in (p.split("=") for p in parts[1:])}
        for npairs in [int(x) for x in args.pairs.split(",")]:
            e.set_debug_flags(f)
            for k, v in tune.items():
                e.set_tuning(knobs[k], v)
            e.compute_batch_device(dl.data_ptr(), dr.data_ptr(), npairs, H * W, H, W, W, prm, out.data_ptr())
            e.synchronize()
            ref = first.setdefault(npairs, out[:npairs].cpu().clone())
            e.set_timing(True)
            e.reset_timing()
            for _ in range(args.calls):
                e.compute_batch_device(dl.data_ptr(), dr.data_ptr(), npairs, H * W, H, W, W, prm, out.data_ptr())
            e.synchronize()
            st = e.timing()
            e.set_timing(False)
            e.set_debug_flags(0)
            for k in tune:
                e.set_tuning(knobs[k], 0)
            print(json.dumps({"run": run, "npairs": npairs, "D": args.D,
                              "us_per_call": {k: round(v[0] * 1e3 / args.calls, 1) for k, v in st.items() if v[0] > 0},
                              "same": bool(torch.equal(ref, out[:npairs].cpu()))}), flush=True)


if __name__ == "__main__":
    main()
