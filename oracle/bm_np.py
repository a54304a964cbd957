"""CPU oracle (numpy) for cv::StereoBM — TEST INFRASTRUCTURE ONLY (same import
rule as oracle/sgm_np.py).

PARITY STATUS: *parity unpinned* (OpenCV is not in the image and the reference
holds no fixtures).  The reference reaches StereoBM through
``cv2.StereoBM_create(numDisparities, blockSize)`` for ``method="BM"``
(``stereo_vision/stereo_vision.py:164-166``), then ``createRightMatcher`` /
``createDisparityWLSFilter`` (:171-172), which for BM set textureThreshold 0,
uniquenessRatio 0, disp12MaxDiff 1e6 (and speckleWindowSize 0).  Restated
from upstream ``modules/calib3d/src/stereobm.cpp`` (OpenCV 3.3-3.4 era):

* ``prefilterXSobel`` (the default PREFILTER_XSOBEL): per row pair, Sobel-x
  with a [1 2 1] vertical kernel (rows reflected at the top / bottom),
  ``clip(d, -cap, cap) + cap``; columns 0 and W-1, and the last row of an odd
  height, are ``cap``.
* ``findStereoCorrespondenceBM``: with ``lofs = max(ndisp-1+minD, 0)``,
  ``rofs = -min(ndisp-1+minD, 0)``, ``width1 = W - rofs - ndisp + 1``, output
  column ``X = x + lofs`` (x in [0, width1)) and disparity index d in
  [0, ndisp) (disparity ``ndisp-1+minD-d``):
  ``SAD[y,x,d] = sum_{|dy|,|dx| <= SW2} |Lp[y+dy, clamp(x1+lofs, 0, W-1)] -
  Rp[y+dy, clamp(x1+rofs, 0, W-ndisp) + d]|`` with ``x1 = x+dx``;
  texture ``= sum |Lp - cap|`` over the same window (left clamp);
  WTA = first minimum over d ascending (largest disparity wins ties);
  ``tsum < textureThreshold`` -> FILTERED; uniqueness (if > 0):
  ``thresh = minsad + minsad*u/100``, any ``|d-mind| > 1`` with
  ``sad <= thresh`` -> FILTERED; sub-pixel with the end mirror
  ``sad[-1] = sad[1]``, ``sad[ndisp] = sad[ndisp-2]``:
  ``den = p + n - 2 sad[mind] + |p - n|`` (p = sad[mind+1], n = sad[mind-1]),
  ``disp = ((ndisp-mind-1+minD)*256 + (den ? (p-n)*256/den : 0) + 15) >> 4``
  (C-truncating division).
* Only pixels inside ``getValidDisparityROI`` (x in [maxD+SW2, W-SW2),
  y in [SW2, H-SW2), maxD = minD+ndisp-1) and inside [lofs, lofs+width1) are
  computed; every other pixel is ``FILTERED = (minD-1)*16``.  Inside that
  region the windows never need the row clamp, so the result does not depend
  on OpenCV's row striping.
* ``validateDisparity`` when disp12MaxDiff >= 0, then ``filterSpeckles(disp,
  FILTERED, speckleWindowSize, speckleRange)`` (speckleRange NOT scaled by 16
  for BM).
"""
from __future__ import annotations

import numpy as np

from .sgm_np import filter_speckles

PREFILTER_NORMALIZED_RESPONSE = 0
PREFILTER_XSOBEL = 1


def normalize_bm(p: dict) -> dict:
    q = dict(preFilterType=PREFILTER_XSOBEL, preFilterSize=9, preFilterCap=31, blockSize=21, minDisparity=0,
             numDisparities=64, textureThreshold=10, uniquenessRatio=15, speckleWindowSize=0, speckleRange=0,
             disp12MaxDiff=-1)
    q.update(p)
    return {k: int(v) for k, v in q.items()}


def check_bm(H, W, q):
    if q["preFilterType"] not in (PREFILTER_NORMALIZED_RESPONSE, PREFILTER_XSOBEL):
        raise ValueError("preFilterType must be NORMALIZED_RESPONSE or XSOBEL")
    if q["preFilterSize"] < 5 or q["preFilterSize"] > 255 or q["preFilterSize"] % 2 == 0:
        raise ValueError("preFilterSize must be odd and in [5, 255]")
    if q["preFilterCap"] < 1 or q["preFilterCap"] > 63:
        raise ValueError("preFilterCap must be in [1, 63]")
    bs = q["blockSize"]
    if bs < 5 or bs > 255 or bs % 2 == 0 or bs >= min(H, W):
        raise ValueError("blockSize must be odd, in [5, 255] and smaller than the image")
    if q["numDisparities"] <= 0 or q["numDisparities"] % 16 != 0:
        raise ValueError("numDisparities must be a positive multiple of 16")
    if q["textureThreshold"] < 0 or q["uniquenessRatio"] < 0:
        raise ValueError("textureThreshold / uniquenessRatio must be >= 0")


def prefilter_xsobel(img: np.ndarray, cap: int) -> np.ndarray:
    src = np.asarray(img, np.int64)
    H, W = src.shape
    out = np.full((H, W), cap, np.int64)
    if W < 3:
        return out.astype(np.uint8)
    yy = np.arange(H)
    up = np.where(yy > 0, yy - 1, min(1, H - 1))       # row y-1, reflected at the top
    dn = np.where(yy < H - 1, yy + 1, max(H - 2, 0))   # row y+1, reflected at the bottom
    dx = src[:, 2:] - src[:, :-2]
    v = dx[up] + 2 * dx + dx[dn]
    out[:, 1:-1] = np.clip(v, -cap, cap) + cap
    if H % 2 == 1:
        out[H - 1] = cap
    return out.astype(np.uint8)


def valid_roi(H, W, q):
    SW2 = q["blockSize"] // 2
    maxD = q["minDisparity"] + q["numDisparities"] - 1
    xmin = max(0, maxD) + SW2
    xmax = W - SW2
    ymin, ymax = SW2, H - SW2
    if xmax - xmin <= 0 or ymax - ymin <= 0:
        return 0, 0, 0, 0
    return xmin, ymin, xmax - xmin, ymax - ymin


def _box(a: np.ndarray, r: int):
    """Sums over (2r+1)^2 windows fully inside a (valid-mode)."""
    c = np.cumsum(np.cumsum(np.pad(a, ((1, 0), (1, 0))), 0), 1)
    k = 2 * r + 1
    return c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]


def stereo_bm(left: np.ndarray, right: np.ndarray, params: dict, return_cost=False):
    """StereoBM(...).compute(left, right) restated: int16 disparity x16."""
    q = normalize_bm(params)
    L = np.asarray(left, np.uint8)
    R = np.asarray(right, np.uint8)
    if L.shape != R.shape or L.ndim != 2:
        raise ValueError("left/right must be same-size single-channel uint8")
    H, W = L.shape
    check_bm(H, W, q)
    if q["preFilterType"] != PREFILTER_XSOBEL:
        raise NotImplementedError("PREFILTER_NORMALIZED_RESPONSE is not restated")
    ndisp, mind0, cap = q["numDisparities"], q["minDisparity"], q["preFilterCap"]
    SW2 = q["blockSize"] // 2
    FILTERED = (mind0 - 1) * 16
    out = np.full((H, W), FILTERED, np.int64)
    cost = np.zeros((H, W), np.int64)
    lofs = max(ndisp - 1 + mind0, 0)
    rofs = -min(ndisp - 1 + mind0, 0)
    width1 = W - rofs - ndisp + 1
    vx, vy, vw, vh = valid_roi(H, W, q)
    xs, xe = max(0, vx - lofs), min(width1, vx + vw - lofs)
    if not (lofs >= W or rofs >= W or width1 < 1 or vw == 0 or xe <= xs):
        Lp = prefilter_xsobel(L, cap).astype(np.int64)
        Rp = prefilter_xsobel(R, cap).astype(np.int64)
        y0, y1 = vy, vy + vh
        rows = np.arange(y0 - SW2, y1 + SW2)
        x1 = np.arange(xs - SW2, xe + SW2)
        lcol = np.clip(x1 + lofs, 0, W - 1)
        rcol = np.clip(x1 + rofs, 0, W - ndisp)
        Lw = Lp[rows][:, lcol]
        h, w = y1 - y0, xe - xs
        sad = np.empty((ndisp, h, w), np.int64)
        for d in range(ndisp):
            sad[d] = _box(np.abs(Lw - Rp[rows][:, rcol + d]), SW2)
        tex = _box(np.abs(Lw - cap), SW2)
        mind = np.argmin(sad, axis=0)  # first minimum over ascending index
        minsad = np.take_along_axis(sad, mind[None], 0)[0]
        res = np.full((h, w), FILTERED, np.int64)
        ok = tex >= q["textureThreshold"]
        u = q["uniquenessRatio"]
        if u > 0:
            thresh = minsad + (minsad * u // 100)
            dd = np.arange(ndisp)[:, None, None]
            far = (dd < mind[None] - 1) | (dd > mind[None] + 1)
            ok &= ~np.any(far & (sad <= thresh[None]), axis=0)
        ext = np.concatenate([sad[1:2], sad, sad[ndisp - 2:ndisp - 1]], 0)  # sad[-1] = sad[1], sad[ndisp] = sad[ndisp-2]
        p = np.take_along_axis(ext, (mind + 2)[None], 0)[0]
        n = np.take_along_axis(ext, mind[None], 0)[0]
        den = p + n - 2 * minsad + np.abs(p - n)
        num = (p - n) * 256
        sub = np.where(den != 0, np.where(num >= 0, num // np.where(den != 0, den, 1),
                                          -((-num) // np.where(den != 0, den, 1))), 0)
        val = ((ndisp - mind - 1 + mind0) * 256 + sub + 15) >> 4
        res = np.where(ok, val, FILTERED)
        out[y0:y1, xs + lofs:xe + lofs] = res
        cost[y0:y1, xs + lofs:xe + lofs] = np.where(ok, minsad, 0)
    if q["disp12MaxDiff"] >= 0:
        out = validate_disparity(out, cost, mind0, ndisp, q["disp12MaxDiff"])
    out = out.astype(np.int16)
    if q["speckleWindowSize"] > 0 and q["speckleRange"] >= 0:
        out = filter_speckles(out, FILTERED, q["speckleWindowSize"], q["speckleRange"])
    return (out, cost) if return_cost else out


def validate_disparity(disp, cost, minD, ndisp, disp12MaxDiff):
    """cv::validateDisparity (32S cost), in place on a copy."""
    disp = np.array(disp, np.int64)
    H, W = disp.shape
    maxD = minD + ndisp
    minX1, maxX1 = max(maxD, 0), W + min(minD, 0)
    INV = (minD - 1) * 16
    md = disp12MaxDiff * 16
    for y in range(H):
        d2 = np.full(W, INV, np.int64)
        c2 = np.full(W, np.iinfo(np.int32).max, np.int64)
        row, crow = disp[y], cost[y]
        for x in range(minX1, maxX1):
            d = row[x]
            if d == INV:
                continue
            x2 = x - ((d + 8) >> 4)
            if c2[x2] > crow[x]:
                c2[x2] = crow[x]
                d2[x2] = d
        for x in range(minX1, maxX1):
            d = row[x]
            if d == INV:
                continue
            xa, xb = x - (d >> 4), x - ((d + 15) >> 4)
            if (0 <= xa < W and d2[xa] > INV and abs(d2[xa] - d) > md) and \
               (0 <= xb < W and d2[xb] > INV and abs(d2[xb] - d) > md):
                row[x] = INV
    return disp


def right_matcher_params(params: dict) -> dict:
    """ximgproc::createRightMatcher(StereoBM)."""
    q = normalize_bm(params)
    return dict(numDisparities=q["numDisparities"], blockSize=q["blockSize"],
                minDisparity=-(q["minDisparity"] + q["numDisparities"]) + 1, textureThreshold=0,
                uniquenessRatio=0, disp12MaxDiff=1000000, speckleWindowSize=0)
