"""Sweep-engine E/W volumes: packed k_ew vs the per-direction row lines, per D and cost type
(debug_fetch(1) = slots E, W of the last pair).  python tools/ew_check.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from stereo_match_amd import _lib, synthetic
    e = _lib.Engine(0)
    H, W = 40, 420
    for D in (16, 32, 48, 64, 80, 96, 112, 128, 144, 160, 176, 192, 208, 224, 240, 256):
        left, right, _ = synthetic.random_dot_pair(H, W, D, seed=D)
        for cost in (0, 1):
            p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=8 if cost else 5)
            prm = synthetic.to_sm_params(p)
            res = []
            for f in (16384, 16384 | 256):
                e.set_debug_flags(f)
                out = e.compute(left, right, prm)
                vol = np.frombuffer(e.debug_fetch(1), np.uint8 if cost else np.uint16)
                res.append((out, vol))
            e.set_debug_flags(0)
            (o0, v0), (o1, v1) = res
            nv = int((v0 != v1).sum())
            first = int(np.flatnonzero(v0 != v1)[0]) if nv else -1
            print(f"D={D:3d} cost={'census' if cost else 'sgbm  '} out_same={np.array_equal(o0, o1)} "
                  f"vol_diff={nv} first={first} of {v0.size}", flush=True)
    e.close()


if __name__ == "__main__":
    main()
