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

from oracle import ref_c, sgm_np, wls_np  # noqa: E402
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


def volume_cases():
    """External f32 cost volumes (mc-cnn mode): vol_<name>.npz
    holds ``vol`` float32 [D,H,W], ``params``, ``offset``, ``scale``,
    ``expected`` and ``raw``."""
    l16, r16, _ = synthetic.random_dot_pair(40, 90, 16, seed=11)
    l32, r32, _ = synthetic.random_dot_pair(36, 100, 32, seed=12)
    v16 = synthetic.absdiff_volume(l16, r16, 16)[0]
    v32 = synthetic.absdiff_volume(l32, r32, 32)[0]
    rng = np.random.default_rng(13)
    vr = (rng.standard_normal((16, 30, 70)) * 0.5).astype(np.float32)
    vr[rng.random(vr.shape) < 0.02] = np.nan
    vr[0, 0, :4] = [np.inf, -np.inf, 0.5, 1.5]  # clamp, clamp, half-even ties
    yield "vol_absdiff_d16_p8", v16, dict(synthetic.cost_volume_params(16)), 0.0, synthetic.VOLUME_SCALE
    yield "vol_absdiff_d32_p5", v32, dict(synthetic.cost_volume_params(32), mode=5), 0.0, synthetic.VOLUME_SCALE
    yield "vol_signed_nan_d16", vr, dict(synthetic.cost_volume_params(16), P1=3, P2=40), 1.0, 1.0
    yield "vol_minD_neg3_d16", v16, dict(synthetic.cost_volume_params(16), minDisparity=-3), 0.0, 1000.0
    # plane counts that are not a multiple of 16 (the reference's own mc-cnn volume has 228,
    # mapTo3D_mc_cnn.py:71): an external volume keeps the planes it was made with
    l20, r20, _ = synthetic.random_dot_pair(32, 84, 20, seed=14)
    l37, r37, _ = synthetic.random_dot_pair(30, 96, 37, seed=15)
    yield "vol_absdiff_d20_p8", synthetic.absdiff_volume(l20, r20, 20)[0], dict(synthetic.cost_volume_params(20)), \
        0.0, synthetic.VOLUME_SCALE
    yield "vol_absdiff_d37_p5_minD2", synthetic.absdiff_volume(l37, r37, 37, minD=2)[0], \
        dict(synthetic.cost_volume_params(37), mode=5, minDisparity=2), 0.0, synthetic.VOLUME_SCALE


def wls_cases():
    """WLS post-filter: wls_<name>.npz holds ``displ``, ``dispr``
    (int16, from the SGBM oracle as compute_disparity runs them), ``guide``
    (uint8), ``params`` (JSON of the wls_np params) and ``expected``."""
    for name, (H, W, D, seed, ws) in dict(d16=(40, 96, 16, 21, 5), d32_ws3=(48, 120, 32, 22, 3)).items():
        left, right, _ = synthetic.random_dot_pair(H, W, D, seed=seed)
        settings = synthetic.parity_params(D, window_size=ws)
        lp = dict(settings, uniquenessRatio=0, disp12MaxDiff=1000000)  # createDisparityWLSFilter mutation
        displ = ref_c.compute(left, right, lp)
        dispr = ref_c.compute(right, left, sgm_np.right_matcher_params(settings))
        wp = dict(lmbda=80000.0, sigma=1.2, radius=(5 + 1) // 2, min_disp=0, left_offset=D, right_offset=0)
        yield "wls_" + name, displ, dispr, left, wp
    left, right, _ = synthetic.random_dot_pair(30, 70, 16, seed=23)
    d = ref_c.compute(left, right, synthetic.parity_params(16))
    yield "wls_generic_noconf", d, None, left, dict(lmbda=8000.0, sigma=1.5, use_confidence=False)


def main():
    for name, displ, dispr, guide, wp in wls_cases():
        out = wls_np.wls_filter(displ, guide, dispr, wp)
        arrs = dict(displ=displ, guide=guide, params=np.array(json.dumps(wp)), expected=out)
        if dispr is not None:
            arrs["dispr"] = dispr
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
        print(f"{name}: {displ.shape} filled={np.mean(out >= 0):.3f}")
    for name, vol, p, off, sc in volume_cases():
        out, st = sgm_np.compute_volume(vol, p, off, sc, return_stages=True)
        c = ref_c.compute_volume(vol, p, off, sc)
        if not np.array_equal(out, c):
            raise SystemExit(f"{name}: numpy and C restatements disagree")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), vol=vol, params=np.array(json.dumps(p)),
                            offset=np.float32(off), scale=np.float32(sc), expected=out, raw=st["raw"])
        print(f"{name}: {vol.shape} valid={np.mean(out > (p.get('minDisparity', 0) - 1) * 16):.3f}")
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
