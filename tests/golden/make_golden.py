"""Generate the committed golden fixtures from the CPU restatement.

    python tests/golden/make_golden.py

Each ``<name>.npz`` holds: ``left``, ``right`` (uint8 [H,W]), ``params``
(JSON text of the oracle params dict), ``expected`` (int16 [H,W], after the
3x3 median) and ``raw`` (int16 [H,W], before the median).  Expected values
come from oracle/sgm_np.py and are cross-checked against oracle/sgm_ref.c
before being written (the two are independent restatements; parity with
OpenCV itself is unpinned — see oracle/sgm_np.py).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import ref_c, sgm_np  # noqa: E402
from stereo_match_amd import synthetic  # noqa: E402


def cases():
    H, W = 48, 96
    l16, r16, _ = synthetic.random_dot_pair(H, W, 16, seed=1)
    l32, r32, _ = synthetic.random_dot_pair(H, W, 32, seed=2)
    k1l, k1r = synthetic.shifted_pair(32, 80, 5, seed=3)
    const = np.full((24, 64), 63, np.uint8)
    yield "census8_d16", l16, r16, synthetic.headline_params(16)
    yield "census8_d32", l32, r32, synthetic.headline_params(32)
    yield "census5_d16", l16, r16, dict(synthetic.headline_params(16), mode=5)
    yield "sgbm5_d16_settings", l16, r16, synthetic.parity_params(16)
    yield "sgbm5_d32_settings", l32, r32, synthetic.parity_params(32)
    yield "sgbm8_hh_d16", l16, r16, dict(synthetic.parity_params(16), mode=8)
    # the params compute_disparity's left matcher really runs with
    # (createDisparityWLSFilter sets uniquenessRatio 0, disp12MaxDiff 1e6)
    yield "sgbm5_d32_wlsleft", l32, r32, dict(synthetic.parity_params(32), uniquenessRatio=0,
                                              disp12MaxDiff=1000000)
    # createRightMatcher: minD = -(0+16)+1, uniq 0, disp12 1e6, on swapped images
    yield "sgbm5_d16_right", r16, l16, sgm_np.right_matcher_params(synthetic.parity_params(16))
    yield "sgbm5_d16_minD_neg5", l16, r16, dict(synthetic.parity_params(16), minDisparity=-5, blockSize=3)
    yield "sgbm5_d16_window3", l16, r16, synthetic.parity_params(16, window_size=3)
    yield "sgbm5_k1_shift5", k1l, k1r, synthetic.parity_params(16)
    yield "census8_const63", const, const, synthetic.headline_params(16)
    yield "sgbm5_const63", const, const, synthetic.parity_params(16)
    # width barely larger than D: few valid columns
    yield "census8_narrow", l16[:, :20].copy(), r16[:, :20].copy(), synthetic.headline_params(16)
    # one row image
    yield "sgbm5_one_row", l32[:1].copy(), r32[:1].copy(), synthetic.parity_params(16)


def main():
    for name, left, right, p in cases():
        out, st = sgm_np.compute(left, right, p, return_stages=True)
        raw = st.get("raw", out)
        c = ref_c.compute(left, right, p)
        if not np.array_equal(out, c):
            raise SystemExit(f"{name}: numpy and C restatements disagree")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), left=left, right=right,
                            params=np.array(json.dumps(p)), expected=out, raw=raw)
        print(f"{name}: {left.shape} valid={np.mean(out > (p.get('minDisparity', 0) - 1) * 16):.3f}")


if __name__ == "__main__":
    main()
