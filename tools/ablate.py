"""Timing ablations of the path kernel (results are wrong under flags != 0).

    python tools/ablate.py [--config kitti] [--pairs 8] [--rounds 5]
Prints per-stage device time per pair for each flag set, interleaved rounds
in one process (CDNA guide §5.4 rule 24)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="kitti")
    ap.add_argument("--mode", default="census8")
    ap.add_argument("--pairs", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--flags", default="0,1,2,4,5,6")
    args = ap.parse_args()
    import torch

    from stereo_match_amd import _lib, synthetic
    H, W, D = synthetic.CONFIGS[args.config]
    p = synthetic.headline_params(D) if args.mode == "census8" else synthetic.parity_params(D)
    if args.mode == "sgbm8":  # OpenCV BT cost, 8 paths (MODE_HH)
        p = dict(p, mode=8)
    prm = synthetic.to_sm_params(p)
    P = args.pairs
    ls, rs = zip(*[synthetic.random_dot_pair(H, W, D, seed=i)[:2] for i in range(P)])
    dL = torch.tensor(np.stack(ls), device="cuda")
    dR = torch.tensor(np.stack(rs), device="cuda")
    out = torch.empty((P, H, W), dtype=torch.int16, device="cuda")
    eng = _lib.Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    flags = [int(f) for f in args.flags.split(",")]
    res = {f: [] for f in flags}
    for _ in range(2):
        eng.compute_batch_device(dL.data_ptr(), dR.data_ptr(), P, H * W, H, W, W, prm, out.data_ptr())
    torch.cuda.synchronize()
    ref = out.clone()
    same = {f: True for f in flags}
    for r in range(args.rounds):
        for f in flags:
            eng.set_debug_flags(f)
            eng.set_timing(True)
            eng.reset_timing()
            for _ in range(3):
                eng.compute_batch_device(dL.data_ptr(), dR.data_ptr(), P, H * W, H, W, W, prm, out.data_ptr())
            t = eng.timing()
            eng.set_timing(False)
            torch.cuda.synchronize()
            same[f] = same[f] and bool(torch.equal(out, ref))
            res[f].append({k: v[0] * 1e3 / max(v[2], 1) for k, v in t.items()})
    eng.set_debug_flags(0)
    import hashlib
    # digest of the default engine's maps: equal across builds = the same results
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "mode": args.mode,
                      "out_sha16": hashlib.sha256(ref.cpu().numpy().tobytes()).hexdigest()[:16]}))
    for f in flags:
        med = {k: float(np.median([x[k] for x in res[f]])) for k in res[f][0]}
        print(json.dumps({"flags": f, "same_as_0": same[f],
                          "us_per_pair": {k: round(v, 1) for k, v in med.items()}}))


if __name__ == "__main__":
    main()
