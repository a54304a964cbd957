"""CPU oracle (numpy) for the WLS disparity post-filter — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.

PARITY STATUS: *parity unpinned*.  The reference reaches this arithmetic
through ``cv2.ximgproc.createDisparityWLSFilter(left_matcher)`` +
``wls_filter.filter(displ, gray_l, None, dispr)``
(``stereo_vision/stereo_vision.py:171-182``, settings ``lmbda``/``sigma`` at
``:174-175``), i.e. opencv_contrib ``modules/ximgproc/src/disparity_filters.cpp``
(``DisparityWLSFilterImpl``) and ``fgs_filter.cpp``
(``FastGlobalSmootherFilterImpl``).  Neither is in this image, and the
reference holds no fixtures for it, so this is a restatement of upstream's
published algorithm (version unpinned, OpenCV 3.3–3.4 era per SURVEY.md §8c):

1. Depth-discontinuity maps (``computeDepthDiscontinuityMaps``): on the
   left ROI of ``displ`` and the mirrored ROI of ``dispr``, the
   (2r+1)² ``boxFilter`` mean and ``sqrBoxFilter`` mean of the int16
   disparities (BORDER_REFLECT_101 at the image edge; pixels outside the ROI
   but inside the image are read, as OpenCV filters on a non-isolated ROI
   do), ``conf = max(1 − roll_off·(E[d²] − E[d]²), 0)``.
2. Left-right consistency (``ComputeDiscontinuityAwareLRC_ParBody``): for
   left ROI column j, ``ri = j − (dl >> 4)``; if ``ri`` is inside the right
   ROI, ``conf = min(conf_l[j], conf_r[ri])`` when ``|dl + dr[ri]| <
   LRC_thresh`` else 0; confidence ×255.
3. Fast global smoother (Min et al. 2014, ``fgs_filter.cpp``) over the ROI,
   guided by the left gray view: edge weights ``−exp(−|Δg|/σ)``, per
   iteration one horizontal and one vertical tridiagonal (Thomas) solve of
   ``(I + λ·L_w) u = f`` (one reciprocal of the pivot per element, as
   upstream's SIMD-friendly form), ``λ *= 0.25`` per iteration, 3 iterations
   — run on ``conf·disp`` and on ``conf``.
4. ``filtered = round_half_even(FGS(conf·disp) / FGS(conf))`` (0 where the
   denominator is 0, OpenCV 3.x ``divide``), saturated to int16, written
   into a map pre-filled with ``16·(minDisparity − 1)``.

All arithmetic is float32 in a fixed operation order (no FMA), so the HIP
kernels reproduce it bit for bit; the weight table is built in float64
(``exp``/``sqrt``) and rounded to float32 once — the HIP library builds the
same table on the host.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def weight_table(sigma: float) -> np.ndarray:
    """w[k] = float32(−exp(−sqrt(k²)/σ)) for |Δg| = k ∈ [0, 255] (gray guide)."""
    k = np.arange(256, dtype=np.float64)
    return (-np.exp(-np.sqrt(k * k) / float(np.float32(sigma)))).astype(np.float32)


def _reflect101(i, n):
    """cv::borderInterpolate(BORDER_REFLECT_101): reflect until inside (windows
    wider than the image reflect more than once)."""
    if n == 1:
        return np.zeros_like(i)
    i = np.asarray(i).copy()
    while True:
        bad = (i < 0) | (i >= n)
        if not bad.any():
            return i
        i = np.where(i < 0, -i, np.where(i >= n, 2 * n - 2 - i, i))


def _box_means(disp: np.ndarray, r: int, y0, y1, x0, x1):
    """(mean, mean of squares) float32 over [y0,y1)×[x0,x1), window (2r+1)²,
    reading the whole image with reflect-101 at its edges."""
    H, W = disp.shape
    ys = _reflect101(np.arange(y0 - r, y1 + r), H)
    xs = _reflect101(np.arange(x0 - r, x1 + r), W)
    d = disp.astype(np.int64)[ys][:, xs]
    n = (2 * r + 1) ** 2
    h, w = y1 - y0, x1 - x0
    s = np.zeros((h, w), np.int64)
    s2 = np.zeros((h, w), np.int64)
    for dy in range(2 * r + 1):
        for dx in range(2 * r + 1):
            blk = d[dy:dy + h, dx:dx + w]
            s += blk
            s2 += blk * blk
    scale = 1.0 / n  # double, as OpenCV's ColumnSum
    return (s * scale).astype(np.float32), (s2 * scale).astype(np.float32)


def depth_discontinuity(disp, r, roll_off, roi):
    """Full-size float32 map, ROI filled (zeros elsewhere)."""
    x0, y0, w, h = roi
    out = np.zeros(disp.shape, np.float32)
    if w <= 0 or h <= 0:
        return out
    m, m2 = _box_means(disp, r, y0, y0 + h, x0, x0 + w)
    var = m2 - m * m
    out[y0:y0 + h, x0:x0 + w] = np.maximum(f32(1.0) - f32(roll_off) * var, f32(0.0))
    return out


def confidence_map(displ, dispr, p):
    """computeConfidenceMap: float32 [H, W] (×255)."""
    H, W = displ.shape
    roi = p["roi"]
    x0, y0, w, h = roi
    rroi = (W - (x0 + w), y0, w, h)
    conf_l = depth_discontinuity(displ, p["radius"], p["roll_off"], roi)
    conf_r = depth_discontinuity(dispr, p["radius"], p["roll_off"], rroi)
    conf = conf_l.copy()
    if w > 0:
        dl = displ.astype(np.int64)[:, x0:x0 + w]
        j = np.arange(x0, x0 + w)[None, :]
        ri = j - (dl >> 4)
        inside = (ri >= rroi[0]) & (ri < rroi[0] + rroi[2])
        ric = np.clip(ri, 0, W - 1)
        rows = np.arange(H)[:, None]
        dr = dispr.astype(np.int64)[rows, ric]
        ok = np.abs(dl + dr) < p["lrc_thresh"]
        val = np.where(ok, np.minimum(conf_l[:, x0:x0 + w], conf_r[rows, ric]), f32(0.0))
        conf[:, x0:x0 + w] = np.where(inside, val, conf_l[:, x0:x0 + w])
    return conf * f32(255.0)


def _solve_rows(u_list, C, lam):
    """Thomas solve along axis 1 for every row; C[:, j] couples j and j+1
    (C[:, -1] == 0).  Fixed float32 op order, one reciprocal per element:
    r = 1/(1 − λ(C[j−1]+C[j]) − λC[j−1]·c'[j−1]); c'[j] = λC[j]·r;
    d'[j] = (f[j] − λC[j−1]·d'[j−1])·r; x[j] = d'[j] − c'[j]·x[j+1]."""
    lam = f32(lam)
    h, w = C.shape
    inter = np.empty((h, w), np.float32)
    ip = np.zeros(h, np.float32)
    cp = np.zeros(h, np.float32)
    prev = [np.zeros(h, np.float32) for _ in u_list]
    for j in range(w):
        cj = C[:, j]
        t = f32(1.0) - lam * (cp + cj)
        lcp = lam * cp
        r = f32(1.0) / (t - lcp * ip)
        ip = (lam * cj) * r
        inter[:, j] = ip
        for k, u in enumerate(u_list):
            prev[k] = (u[:, j] - lcp * prev[k]) * r
            u[:, j] = prev[k]
        cp = cj
    for j in range(w - 2, -1, -1):
        for u in u_list:
            u[:, j] = u[:, j] - inter[:, j] * u[:, j + 1]


def fgs(u_list, guide, lam, sigma, num_iter=3, attenuation=0.25):
    """FastGlobalSmootherFilter on float32 arrays (in place), gray guide."""
    g = guide.astype(np.int64)
    tab = weight_table(sigma)
    h, w = g.shape
    Ch = np.zeros((h, w), np.float32)
    Cv = np.zeros((h, w), np.float32)
    if w > 1:
        Ch[:, :-1] = tab[np.abs(g[:, 1:] - g[:, :-1])]
    if h > 1:
        Cv[:-1, :] = tab[np.abs(g[1:, :] - g[:-1, :])]
    lam = f32(lam)
    for _ in range(num_iter):
        _solve_rows(u_list, Ch, lam)
        ut = [np.ascontiguousarray(u.T) for u in u_list]
        _solve_rows(ut, np.ascontiguousarray(Cv.T), lam)
        for u, t in zip(u_list, ut):
            u[...] = t.T
        lam = lam * f32(attenuation)
    return u_list


def normalize_wls(p: dict, H: int, W: int) -> dict:
    q = dict(lmbda=8000.0, sigma=1.0, lrc_thresh=24, radius=5, roll_off=0.001, num_iter=3,
             attenuation=0.25, use_confidence=True, min_disp=0, left_offset=0, right_offset=0,
             top_offset=0, bottom_offset=0)
    q.update(p)
    q["roi"] = (q["left_offset"], q["top_offset"], W - q["left_offset"] - q["right_offset"],
                H - q["top_offset"] - q["bottom_offset"])
    return q


def wls_filter(displ: np.ndarray, guide: np.ndarray, dispr, params: dict, return_stages=False):
    """DisparityWLSFilter::filter(displ, guide, None, dispr) restated."""
    displ = np.asarray(displ, np.int16)
    guide = np.asarray(guide, np.uint8)
    H, W = displ.shape
    if guide.shape != (H, W):
        raise ValueError("guide must be a gray image of the disparity map's size")
    p = normalize_wls(params, H, W)
    x0, y0, w, h = p["roi"]
    out = np.full((H, W), 16 * (p["min_disp"] - 1), np.int16)
    if w <= 0 or h <= 0:
        return (out, {}) if return_stages else out
    src = guide[y0:y0 + h, x0:x0 + w]
    d = displ[y0:y0 + h, x0:x0 + w].astype(np.float32)
    stages = {}
    if p["use_confidence"]:
        dispr = np.asarray(dispr, np.int16)
        if dispr.shape != (H, W):
            raise ValueError("right disparity map must match the left one")
        conf = confidence_map(displ, dispr, p)
        cc = conf[y0:y0 + h, x0:x0 + w].copy()
        num = cc * d
        den = cc.copy()
        fgs([num, den], src, p["lmbda"], p["sigma"], p["num_iter"], p["attenuation"])
        with np.errstate(divide="ignore", invalid="ignore"):
            q = np.where(den != 0, num / np.where(den != 0, den, f32(1.0)), f32(0.0)).astype(np.float32)
        stages = dict(conf=conf, num=num, den=den)
    else:
        q = d.copy()
        fgs([q], src, p["lmbda"], p["sigma"], p["num_iter"], p["attenuation"])
    r = np.clip(np.rint(q), -32768, 32767)
    out[y0:y0 + h, x0:x0 + w] = np.where(np.isnan(r), 0, r).astype(np.int16)
    return (out, stages) if return_stages else out
