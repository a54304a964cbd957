"""CPU oracle (numpy) for cv::reprojectImageTo3D — TEST INFRASTRUCTURE ONLY
(same import rule as oracle/sgm_np.py).

PARITY STATUS: *parity unpinned* (OpenCV ``calib3d`` is not in the image; the
reference holds no fixtures).  Restated from upstream
``cv::reprojectImageTo3D`` (float64 arithmetic, FLT_EPSILON test against the
map minimum, bigZ = 10000 for handleMissingValues).  One deliberate
difference in form: upstream accumulates ``qx += Q(0,0)`` along the row,
this restatement (and the HIP kernel) evaluates ``Q01·y + Q03 + Q00·x``
directly — the two differ by float64 rounding only, far below the float32
output's resolution.  Reference call sites: disparity_calculation.py:302,
mapTo3D_mc_cnn.py:124, stereo_vision/stereo_vision.py:203-209.
"""
from __future__ import annotations

import numpy as np


def reproject_image_to_3d(disparity: np.ndarray, Q: np.ndarray, handle_missing: bool = False) -> np.ndarray:
    d = np.asarray(disparity)
    if d.dtype not in (np.int16, np.float32):
        raise ValueError("disparity must be int16 or float32")
    Q = np.asarray(Q, np.float64).reshape(4, 4)
    H, W = d.shape
    dd = d.astype(np.float32).astype(np.float64)
    y = np.arange(H, dtype=np.float64)[:, None]
    x = np.arange(W, dtype=np.float64)[None, :]
    q = [Q[r, 1] * y + Q[r, 3] + Q[r, 0] * x for r in range(4)]
    with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
        iW = 1.0 / (q[3] + Q[3, 2] * dd)
        X = (q[0] + Q[0, 2] * dd) * iW
        Y = (q[1] + Q[1, 2] * dd) * iW
        Z = (q[2] + Q[2, 2] * dd) * iW
        if handle_missing:
            md = float(dd.min())
            Z = np.where(np.abs(dd - md) <= np.finfo(np.float32).eps, 10000.0, Z)
        return np.stack([X, Y, Z], -1).astype(np.float32)
