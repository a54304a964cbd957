"""Synthetic rectified stereo pairs — inputs for tests and bench.

There is no dataset in the image (no network), so every measured
configuration uses random-dot pairs of the named configuration's shape:
left = uniform u8 noise smoothed by a 3×3 box; right = left forward-warped
by a known integer disparity field (slanted ground plane 0 → 0.7·D over the
rows plus three fronto-parallel rectangles at D/4, D/2, 3D/4); right pixels
that nothing maps to (occlusions) are refilled with fresh noise.
"""
from __future__ import annotations

import numpy as np

CONFIGS = {
    # name: (H, W, D)
    "tsukuba": (288, 384, 16),
    "kitti": (375, 1242, 128),
    "middlebury": (1988, 2880, 256),
    "mccnn": (375, 1242, 192),
}


def _smooth3(a: np.ndarray) -> np.ndarray:
    p = np.pad(a, 1, mode="edge")
    H, W = a.shape
    return sum(p[i:i + H, j:j + W] for i in range(3) for j in range(3)) / 9.0


def disparity_field(H: int, W: int, D: int) -> np.ndarray:
    """Integer ground-truth disparity (left view)."""
    ys = np.arange(H)[:, None]
    d = np.broadcast_to((0.7 * (D - 1) * ys / max(H - 1, 1)).astype(np.int64), (H, W)).copy()
    for k, frac in enumerate((0.25, 0.5, 0.75)):
        y0, y1 = int(H * (0.15 + 0.25 * k)), int(H * (0.35 + 0.25 * k))
        x0, x1 = int(W * (0.2 + 0.25 * k)), int(W * (0.35 + 0.25 * k))
        d[y0:y1, x0:x1] = int(frac * D)
    return np.minimum(d, D - 1)


def random_dot_pair(H: int, W: int, D: int, seed: int = 2024):
    """Returns (left u8[H,W], right u8[H,W], gt disparity int64[H,W])."""
    rng = np.random.default_rng(seed)
    left = np.clip(_smooth3(rng.integers(0, 256, (H, W)).astype(np.float64)), 0, 255).astype(np.uint8)
    gt = disparity_field(H, W, D)
    fresh = np.clip(_smooth3(rng.integers(0, 256, (H, W)).astype(np.float64)), 0, 255).astype(np.uint8)
    right = fresh.copy()
    xs = np.arange(W)
    for y in range(H):
        order = np.argsort(gt[y], kind="stable")  # larger disparity (closer) written last, wins
        xr = xs[order] - gt[y, order]
        ok = xr >= 0
        right[y, xr[ok]] = left[y, xs[order][ok]]
    return left, right, gt


def shifted_pair(H: int, W: int, shift: int, seed: int = 0):
    """Constant-disparity pair (KAT K1): right[x] = left[x + shift]."""
    rng = np.random.default_rng(seed)
    base = np.clip(_smooth3(rng.integers(0, 256, (H, W + shift)).astype(np.float64)), 0, 255).astype(np.uint8)
    return np.ascontiguousarray(base[:, :W]), np.ascontiguousarray(base[:, shift:shift + W])


def headline_params(D: int = 128) -> dict:
    """North-star mode: census 9x7 + 8 paths (P1/P2 as libSGM's census defaults;
    no reference value exists), uniqueness 15, disp12MaxDiff 1."""
    return dict(minDisparity=0, numDisparities=D, blockSize=5, P1=10, P2=120, disp12MaxDiff=1,
                uniquenessRatio=15, preFilterCap=63, speckleWindowSize=0, speckleRange=2,
                mode=8, cost=1)


def parity_params(D: int = 128, window_size: int = 5) -> dict:
    """OpenCV-parity mode with settings.ini values (P1 = 8*3*ws^2, P2 = 32*3*ws^2)."""
    return dict(minDisparity=0, numDisparities=D, blockSize=5, P1=8 * 3 * window_size ** 2,
                P2=32 * 3 * window_size ** 2, disp12MaxDiff=1, uniquenessRatio=15, preFilterCap=63,
                speckleWindowSize=0, speckleRange=2, mode=5, cost=0)


def cost_volume_params(D: int = 192) -> dict:
    """mc-cnn volume mode (config C): 8 paths; P1/P2 in quantised cost units
    (costs scaled by VOLUME_SCALE, so P1 ~ 0.05 and P2 ~ 0.5 of the [0,1] cost
    range), uniqueness 15, disp12MaxDiff 1."""
    return dict(minDisparity=0, numDisparities=D, blockSize=5, P1=200, P2=2000, disp12MaxDiff=1,
                uniquenessRatio=15, preFilterCap=63, speckleWindowSize=0, speckleRange=2, mode=8, cost=2)


VOLUME_SCALE = 4000.0  # [0,1] costs -> [0, 4000] of the 12-bit quantised range


def absdiff_volume(left: np.ndarray, right: np.ndarray, D: int, minD: int = 0) -> np.ndarray:
    """Config C stand-in for an mc-cnn output: float32 (1, D, H, W),
    d-major, plane d = |L(x) − R(x − minD − d)| / 255 averaged over a 3×3
    window; NaN where x − minD − d falls outside the right image (mc-cnn leaves
    those undefined too)."""
    L = _smooth3(left.astype(np.float64)).astype(np.float32)
    R = _smooth3(right.astype(np.float64)).astype(np.float32)
    H, W = left.shape
    vol = np.full((1, D, H, W), np.nan, np.float32)
    for d in range(D):
        s = minD + d
        lo, hi = max(s, 0), min(W, W + s)
        if lo < hi:
            vol[0, d, :, lo:hi] = np.abs(L[:, lo:hi] - R[:, lo - s:hi - s]) / np.float32(255.0)
    return vol


def to_sm_params(p: dict):
    """Oracle-style dict -> C-ABI SmParams (mode 5/8, cost 0/1)."""
    from ._lib import SmParams

    return SmParams(int(p.get("minDisparity", 0)), int(p.get("numDisparities", 16)), int(p.get("blockSize", 3)),
                    int(p.get("P1", 0)), int(p.get("P2", 0)), int(p.get("disp12MaxDiff", 0)),
                    int(p.get("uniquenessRatio", 0)), int(p.get("preFilterCap", 0)),
                    int(p.get("speckleWindowSize", 0)), int(p.get("speckleRange", 0)), int(p.get("cost", 0)),
                    int(p.get("mode", 5)))
