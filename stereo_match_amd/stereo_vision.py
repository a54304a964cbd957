"""Drop-in for the reference hot path ``compute_disparity``.

Reference: ``stereo_vision/stereo_vision.py:132-184``::

    compute_disparity(gray_l, gray_r, disparity_settings, method="SGBM")
        -> (displ int16[H,W] x16, filtered_img int16[H,W] x16)

Same argument meaning, same P1/P2 derivation (``:148-149``), same
``RuntimeError('Method not supported')`` (``:167-168``).  The left and
right SGBM matches and the WLS post-filter (``:172-175,182``,
:mod:`stereo_match_amd.wls`) all run on the MI355X through the C-ABI, in
the reference's call order (so ``createDisparityWLSFilter``'s mutation of
the left matcher applies to ``displ`` exactly as in the reference).
``sm_compute_disparity`` in the C-ABI is the same flow in one call; for
the usual inputs (two same-shape 2-D uint8 numpy images, ``method="SGBM"``)
this function runs through it (one host round trip, the matchers and the
WLS filter overlapped on the device: DESIGN.md §4.5), with the matchers'
parameters captured before ``createDisparityWLSFilter`` mutates the left one,
exactly as the three calls below see them; other inputs take the three calls.
"""
from __future__ import annotations

import numpy as np

from . import matcher as _m
from ._lib import SM_E_UNSUPPORTED, SmError


def matcher_from_settings(disparity_settings, method="SGBM", device=0):
    """The left matcher ``compute_disparity`` builds (reference :148-168)."""
    p1 = 8 * 3 * disparity_settings['window_size'] ** 2
    p2 = 32 * 3 * disparity_settings['window_size'] ** 2
    if method == "SGBM":
        paths = int(disparity_settings.get('paths', 5))
        return _m.StereoSGBM_create(minDisparity=disparity_settings['min_disparity'],
                                    numDisparities=disparity_settings['num_disparities'],
                                    blockSize=disparity_settings['block_size'],
                                    P1=p1,
                                    P2=p2,
                                    disp12MaxDiff=disparity_settings['disp12_max_diff'],
                                    uniquenessRatio=disparity_settings['uniqueness_ratio'],
                                    speckleWindowSize=disparity_settings['speckle_window_size'],
                                    speckleRange=disparity_settings['speckle_range'],
                                    preFilterCap=disparity_settings['pre_filter_cap'],
                                    mode=_m.STEREO_SGBM_MODE_HH if paths == 8 else _m.STEREO_SGBM_MODE_SGBM,
                                    cost=disparity_settings.get('cost', 'sgbm'),
                                    device=device)
    elif method == "BM":
        return _m.StereoBM_create(numDisparities=disparity_settings['num_disparities'],
                                  blockSize=disparity_settings['block_size'], device=device)
    else:
        raise RuntimeError('Method not supported')


def compute_disparity(gray_l, gray_r, disparity_settings, method="SGBM", device=0):
    """Computes disparity between two rectified grayscale images.

    Returns ``(displ, filtered_img)``, both int16 disparity × 16.
    """
    from . import wls

    left_matcher = matcher_from_settings(disparity_settings, method, device)
    one_call = method == "SGBM" and _one_call_inputs(gray_l, gray_r)
    prm = left_matcher.params() if one_call else None  # before the WLS filter's mutation (:172)
    right_matcher = _m.createRightMatcher(left_matcher)
    wls_filter = wls.createDisparityWLSFilter(left_matcher)
    wls_filter.setLambda(disparity_settings['lmbda'])
    wls_filter.setSigmaColor(disparity_settings['sigma'])

    if one_call:  # sm_compute_disparity: the same three steps in one call
        from . import _lib
        H, W = gray_l.shape
        return _lib.engine(device).compute_disparity(gray_l, gray_r, prm, wls_filter.params(H, W))
    displ = left_matcher.compute(gray_l, gray_r)
    dispr = right_matcher.compute(gray_r, gray_l)
    filtered_img = wls_filter.filter(displ, gray_l, None, dispr)
    return displ, filtered_img


def _one_call_inputs(gray_l, gray_r) -> bool:
    """Two host images the one-call ABI takes as they are: same-shape 2-D uint8 numpy arrays."""
    return (isinstance(gray_l, np.ndarray) and isinstance(gray_r, np.ndarray) and gray_l.ndim == 2
            and gray_l.shape == gray_r.shape and gray_l.dtype == np.uint8 and gray_r.dtype == np.uint8
            and gray_l.size > 0)
