"""CPU oracle (numpy) for the stereo_match hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product path
(``stereo_match_amd``) never imports it and fails loudly without its HIP
library.

PARITY STATUS: *parity unpinned*.  The reference path
(``stereo_vision/stereo_vision.py:132-184`` → ``cv2.StereoSGBM_create`` /
``left_matcher.compute``) keeps all of its arithmetic inside third-party
OpenCV (``opencv-contrib-python``, version unpinned by the reference — no
requirements file; era 3.3–3.4 per SURVEY.md §8c).  OpenCV is not installed in
this image and the reference ships no golden vectors or tests,
so this restatement is pinned only by hand-derived known-answer tests
(``tests/test_oracle_kats.py``) and by bit-exact agreement with an
independently structured C restatement (``oracle/sgm_ref.c``) that follows
OpenCV's own row-streaming loop structure.

What is restated (upstream OpenCV ``modules/calib3d/src/stereosgbm.cpp``):

* ``calcPixelCostBT``: Sobel-x prefilter clipped to ``preFilterCap`` plus the
  raw-intensity channel (``>>2``), Birchfield–Tomasi sampling-insensitive cost.
* ``computeDisparitySGBM``: ``blockSize²`` box sum with clamped borders and
  the frozen bottom rows of the incremental vertical sum; ``Cbuf`` seeded with
  ``P2`` (so every path value ``L`` equals the textbook Hirschmüller value);
  MODE_SGBM (5 paths: →, ↘, ↓, ↙, ←) or MODE_HH (8 paths); ``S`` saturated to
  int16; WTA with uniqueness, integer (C-truncating) sub-pixel parabola,
  right-view ``disp2`` and the ``disp12MaxDiff`` check.
* ``StereoSGBMImpl::compute``: ``medianBlur(disp, 3)`` (replicate border).
* ``ximgproc::createRightMatcher`` parameters for the right view.

Plus the north-star Census mode (no reference counterpart, own definition,
see DESIGN.md §2): 9×7 census with clamped borders, Hamming cost, the same
recurrence / WTA / LR / median.

The reference call sites this follows: parameter plumbing
``stereo_vision/stereo_vision.py:148-163`` (P1 = 8·3·ws², P2 = 32·3·ws²) and
defaults ``disparity_calculation.py:87-92`` / ``settings.ini:1-23``.
"""
from __future__ import annotations

import numpy as np

DISP_SHIFT = 4
DISP_SCALE = 1 << DISP_SHIFT
MAX_COST = 32767  # SHRT_MAX, OpenCV's CostType ceiling

# Direction = (dx, dy): current cell = predecessor + (dx, dy).
DIR_E, DIR_SE, DIR_S, DIR_SW, DIR_W, DIR_N, DIR_NW, DIR_NE = (
    (1, 0), (1, 1), (0, 1), (-1, 1), (-1, 0), (0, -1), (-1, -1), (1, -1))
# MODE_SGBM: r0=(-1,0) r1=(-1,-1) r2=(0,-1) r3=(1,-1) predecessors in the
# top-down pass plus the backward horizontal pass fused with WTA.
DIRS_5 = (DIR_E, DIR_SE, DIR_S, DIR_SW, DIR_W)
DIRS_8 = (DIR_E, DIR_SE, DIR_S, DIR_SW, DIR_W, DIR_N, DIR_NW, DIR_NE)

COST_SGBM = 0
COST_CENSUS = 1
COST_VOLUME = 2  # external f32 cost volume (mc-cnn)
VOLUME_CMAX = 4095  # quantised external costs live in [0, 4095]


# --------------------------------------------------------------------------
# Parameters
# --------------------------------------------------------------------------
def normalize_params(p: dict) -> dict:
    """StereoSGBM parameter normalisation.

    Keys follow cv2.StereoSGBM_create's kwargs (``minDisparity``,
    ``numDisparities``, ``blockSize``, ``P1``, ``P2``, ``disp12MaxDiff``,
    ``uniquenessRatio``, ``speckleWindowSize``, ``speckleRange``,
    ``preFilterCap``, ``mode``) plus ``cost`` (COST_SGBM / COST_CENSUS).
    ``mode`` is 5 (MODE_SGBM) or 8 (MODE_HH / 8-path).
    """
    q = dict(p)
    q.setdefault("minDisparity", 0)
    q.setdefault("numDisparities", 16)
    q.setdefault("blockSize", 3)
    q.setdefault("P1", 0)
    q.setdefault("P2", 0)
    q.setdefault("disp12MaxDiff", 0)
    q.setdefault("uniquenessRatio", 0)
    q.setdefault("speckleWindowSize", 0)
    q.setdefault("speckleRange", 0)
    q.setdefault("preFilterCap", 0)
    q.setdefault("mode", 5)
    q.setdefault("cost", COST_SGBM)
    bs = q["blockSize"] if q["blockSize"] > 0 else 5
    P1 = q["P1"] if q["P1"] > 0 else 2
    P2 = max(q["P2"] if q["P2"] > 0 else 5, P1 + 1)
    return dict(
        minD=int(q["minDisparity"]), D=int(q["numDisparities"]), bs=int(bs),
        P1=int(P1), P2=int(P2),
        ftzero=(max(int(q["preFilterCap"]), 15) | 1),
        uniq=int(q["uniquenessRatio"]) if q["uniquenessRatio"] >= 0 else 10,
        disp12=int(q["disp12MaxDiff"]) if q["disp12MaxDiff"] > 0 else 1,
        speckle_ws=int(q["speckleWindowSize"]), speckle_range=int(q["speckleRange"]),
        mode=int(q["mode"]), cost=int(q["cost"]))


def geometry(W: int, minD: int, D: int):
    maxD = minD + D
    minX1 = max(maxD, 0)
    maxX1 = W + min(minD, 0)
    return minX1, maxX1


# --------------------------------------------------------------------------
# Pixel costs
# --------------------------------------------------------------------------
def prefilter(img: np.ndarray, ftzero: int):
    """calcPixelCostBT's two channels: clipped Sobel-x and raw intensity.

    Columns 0 and W-1 of BOTH channels are forced to clipTab[0] == ftzero.
    """
    I = img.astype(np.int64)
    H, W = I.shape
    g = np.full((H, W), ftzero, np.int64)
    raw = I.copy()
    raw[:, 0] = ftzero
    raw[:, W - 1] = ftzero
    if W >= 3:
        dx = I[:, 2:] - I[:, :-2]                      # I[x+1]-I[x-1], x=1..W-2
        yn = np.maximum(np.arange(H) - 1, 0)
        ys = np.minimum(np.arange(H) + 1, H - 1)
        val = 2 * dx + dx[yn] + dx[ys]
        g[:, 1:W - 1] = np.clip(val, -ftzero, ftzero) + ftzero
    return g, raw


def _bt_minmax(v: np.ndarray):
    """(v0, v1) = min/max(v, (v+v[x-1])/2, (v+v[x+1])/2), edges use v."""
    vl = v.copy()
    vr = v.copy()
    vl[:, 1:] = (v[:, 1:] + v[:, :-1]) // 2
    vr[:, :-1] = (v[:, :-1] + v[:, 1:]) // 2
    return np.minimum(np.minimum(vl, vr), v), np.maximum(np.maximum(vl, vr), v)


def pixel_cost_bt(left, right, minD, D, ftzero):
    """Per-pixel BT cost pix[y, x1, d], x = x1 + minX1, right column x-minD-d."""
    H, W = left.shape
    minX1, maxX1 = geometry(W, minD, D)
    width1 = maxX1 - minX1
    pix = np.zeros((H, max(width1, 0), D), np.int64)
    if width1 <= 0:
        return pix
    xs = np.arange(minX1, maxX1)
    xr = xs[:, None] - (minD + np.arange(D))[None, :]  # [width1, D]
    for ch, shift in zip(zip(prefilter(left, ftzero), prefilter(right, ftzero)), (0, 2)):
        u_img, v_img = ch
        u0, u1 = _bt_minmax(u_img)
        v0, v1 = _bt_minmax(v_img)
        u = u_img[:, xs][:, :, None]
        uu0 = u0[:, xs][:, :, None]
        uu1 = u1[:, xs][:, :, None]
        v = v_img[:, xr]
        vv0 = v0[:, xr]
        vv1 = v1[:, xr]
        c0 = np.maximum(np.maximum(0, u - vv1), vv0 - u)
        c1 = np.maximum(np.maximum(0, v - uu1), uu0 - v)
        pix += np.minimum(c0, c1) >> shift
    return pix


def wrap16(a):
    return ((np.asarray(a, np.int64) + 32768) & 0xFFFF) - 32768


def box_cost_sgbm(pix: np.ndarray, bs: int, mode: int):
    """Box-summed cost WITHOUT the +P2 seed (C_true), int16-wrapped.

    hsum: clamped horizontal window over the width1 domain.  Vertical: rows
    y <= H-1-SH2 are the clamped window sum; later rows (y >= 1) are never
    updated by OpenCV's incremental loop — MODE_SGBM reuses one C row, so
    they stay frozen at C[H-1-SH2]; MODE_HH keeps one C row per y, so they
    keep the seed alone (C_true = 0).
    """
    H, width1, D = pix.shape
    SW2 = SH2 = bs // 2
    if width1 == 0:
        return pix.copy()
    idx = np.clip(np.arange(width1)[:, None] + np.arange(-SW2, SW2 + 1)[None, :], 0, width1 - 1)
    hsum = pix[:, idx, :].sum(axis=2)  # [H, width1, D]
    C = np.empty_like(hsum)
    last = H - 1 - SH2
    for y in range(H):
        frozen = y >= 1 and y > last
        if frozen and mode == 8:
            C[y] = 0
            continue
        yc = max(0, min(y, last))
        rows = np.clip(np.arange(yc - SH2, yc + SH2 + 1), 0, H - 1)
        C[y] = hsum[rows].sum(axis=0)
    return wrap16(C)


def census9x7(img: np.ndarray) -> np.ndarray:
    """Census 9x7 (own definition): 62 bits, row-major window
    order (dy=-3..3, dx=-4..4) skipping the centre, bit k set iff
    I[neighbour] < I[centre]; neighbour coordinates clamped to the image."""
    I = img.astype(np.int64)
    H, W = I.shape
    out = np.zeros((H, W), np.uint64)
    ys = np.arange(H)
    xs = np.arange(W)
    k = 0
    for dy in range(-3, 4):
        for dx in range(-4, 5):
            if dy == 0 and dx == 0:
                continue
            n = I[np.clip(ys + dy, 0, H - 1)][:, np.clip(xs + dx, 0, W - 1)]
            out |= (n < I).astype(np.uint64) << np.uint64(k)
            k += 1
    return out


_POP8 = np.array([bin(i).count("1") for i in range(256)], np.int64)


def popcount64(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, np.uint64)
    return _POP8[a.view(np.uint8).reshape(a.shape + (8,))].sum(-1)


def census_cost(left, right, minD, D):
    H, W = left.shape
    minX1, maxX1 = geometry(W, minD, D)
    width1 = maxX1 - minX1
    if width1 <= 0:
        return np.zeros((H, 0, D), np.int64)
    cl = census9x7(left)
    cr = census9x7(right)
    xs = np.arange(minX1, maxX1)
    xr = xs[:, None] - (minD + np.arange(D))[None, :]
    return popcount64(cl[:, xs][:, :, None] ^ cr[:, xr])


def cost_volume(left, right, prm) -> np.ndarray:
    """C_true[y, x1, d] (int64 values of the int16 cost)."""
    if prm["cost"] == COST_CENSUS:
        return census_cost(left, right, prm["minD"], prm["D"])
    pix = pixel_cost_bt(left, right, prm["minD"], prm["D"], prm["ftzero"])
    return box_cost_sgbm(pix, prm["bs"], prm["mode"])


def quantize_volume(vol: np.ndarray, prm, offset: float, scale: float) -> np.ndarray:
    """External matching cost (mc-cnn ``(1, D, H, W)`` / ``(D, H, W)`` float32,
    d-major — the layout ``mapTo3D_mc_cnn.py:71`` memmaps) → C[y, x1, d].

    Own definition (no reference arithmetic exists: the reference only loads
    the volume): ``q = rint((c + offset) * scale)`` in float32 (two IEEE
    roundings, round-half-even), clamped to [0, VOLUME_CMAX]; NaN → CMAX.
    Volume plane d holds the cost of left pixel x against right pixel
    x − (minD + d); columns follow the matcher geometry [minX1, maxX1)."""
    v = np.asarray(vol, np.float32)
    if v.ndim == 4:
        v = v[0]
    D = prm["D"]
    if v.shape[0] != D:
        raise ValueError("volume has %d planes, numDisparities is %d" % (v.shape[0], D))
    H, W = v.shape[1:]
    minX1, maxX1 = geometry(W, prm["minD"], D)
    sub = v[:, :, minX1:maxX1]
    with np.errstate(invalid="ignore", over="ignore"):
        t = (sub + np.float32(offset)) * np.float32(scale)
        q = np.rint(t)
        q = np.where(np.isnan(q), np.float32(VOLUME_CMAX), q)
        q = np.clip(q, 0, VOLUME_CMAX)
    return q.astype(np.int64).transpose(1, 2, 0)


def volume_window(vol: np.ndarray, prm):
    """The automatic quantisation window (sm_aggregate_cost_f32* with scale 0; own
    definition, parity unpinned: the reference only memmaps the volume,
    ``mapTo3D_mc_cnn.py:71``): over the finite costs of the cells that get quantised
    (every plane, every row, columns [minX1, maxX1)), offset = -min and
    scale = 4095 / (max - min) in float32 (one IEEE subtraction, one IEEE division);
    (0, 1) without finite costs or with max == min."""
    v = np.asarray(vol, np.float32)
    if v.ndim == 4:
        v = v[0]
    W = v.shape[2]
    minX1, maxX1 = geometry(W, prm["minD"], v.shape[0])
    sub = v[:, :, minX1:maxX1]
    fin = sub[np.isfinite(sub)]
    if fin.size == 0:
        return 0.0, 1.0
    mn, mx = np.float32(fin.min()), np.float32(fin.max())
    d = np.float32(mx - mn)
    sc = np.float32(VOLUME_CMAX) / d if d > 0 and np.isfinite(d) else np.float32(1.0)
    return float(np.float32(-mn)), float(sc)


def quantize_counts(vol: np.ndarray, prm, offset: float, scale: float):
    """(clamped, nan) cell counts of quantize_volume: finite-or-infinite costs whose
    rint((c + offset) * scale) fell outside [0, 4095] (or was NaN), and NaN costs."""
    v = np.asarray(vol, np.float32)
    if v.ndim == 4:
        v = v[0]
    W = v.shape[2]
    minX1, maxX1 = geometry(W, prm["minD"], v.shape[0])
    sub = v[:, :, minX1:maxX1]
    nan = np.isnan(sub)
    with np.errstate(invalid="ignore", over="ignore"):
        q = np.rint((sub + np.float32(offset)) * np.float32(scale))
        bad = (q < 0) | (q > VOLUME_CMAX) | np.isnan(q)
    return int(np.sum(bad & ~nan)), int(np.sum(nan))


# --------------------------------------------------------------------------
# Path aggregation
# --------------------------------------------------------------------------
def _step(Cs, Lp, minLp, P1, P2):
    """One recurrence step, vectorised over lines.  Cs, Lp: [..., D]."""
    D = Cs.shape[-1]
    big = np.full(Lp.shape[:-1] + (1,), MAX_COST, np.int64)
    Lm = np.concatenate([big, Lp[..., :D - 1]], -1)   # Lp[d-1]
    Lq = np.concatenate([Lp[..., 1:], big], -1)       # Lp[d+1]
    delta = (minLp + P2)[..., None]
    # OpenCV: L = (C_true + P2) + min(Lp, Lp±1 + P1, delta) - delta
    L = (Cs + P2) + np.minimum(np.minimum(Lp, np.minimum(Lm, Lq) + P1), delta) - delta
    return L, L.min(-1)


def aggregate_path(C: np.ndarray, d: tuple, P1: int, P2: int) -> np.ndarray:
    """L_r over the whole [H, width1, D] domain for direction d=(dx, dy).

    Paths start at the first in-domain cell with Lp ≡ 0, minLp = 0, so the
    first L is C_true (OpenCV clears the Lr/minLr borders to 0).
    """
    H, width1, D = C.shape
    dx, dy = d
    L = np.zeros_like(C)
    if width1 == 0 or H == 0:
        return L
    if dy == 0:
        Lp = np.zeros((H, D), np.int64)
        mp = np.zeros(H, np.int64)
        xr = range(width1) if dx > 0 else range(width1 - 1, -1, -1)
        for x in xr:
            Lp, mp = _step(C[:, x], Lp, mp, P1, P2)
            L[:, x] = Lp
        return L
    Lp = np.zeros((width1, D), np.int64)
    mp = np.zeros(width1, np.int64)
    yr = range(H) if dy > 0 else range(H - 1, -1, -1)
    for y in yr:
        # predecessor of (x, y) is (x - dx, y - dy): shift previous row by dx
        if dx == 0:
            Lq, mq = Lp, mp
        else:
            Lq = np.zeros_like(Lp)
            mq = np.zeros_like(mp)
            if dx > 0:
                Lq[1:], mq[1:] = Lp[:-1], mp[:-1]
            else:
                Lq[:-1], mq[:-1] = Lp[1:], mp[1:]
        Lp, mp = _step(C[y], Lq, mq, P1, P2)
        L[y] = Lp
    return L


def aggregate(C, prm, dirs=None):
    if dirs is None:
        dirs = DIRS_5 if prm["mode"] == 5 else DIRS_8
    S = np.zeros_like(C)
    for d in dirs:
        S += aggregate_path(C, d, prm["P1"], prm["P2"])
    # all L >= 0, so sequential saturating adds == one final saturation
    return np.minimum(S, MAX_COST)


# --------------------------------------------------------------------------
# WTA / uniqueness / sub-pixel / disp2 / LR check
# --------------------------------------------------------------------------
def _cdiv(n, m):
    """C integer division (truncation toward zero), m > 0."""
    return np.where(n >= 0, n // m, -((-n) // m))


SIMD_LANES = 8  # CV_SIMD128 int16 lanes (OpenCV 3.x x86 builds: SSE2)


def wta_best(S: np.ndarray, mode: int) -> np.ndarray:
    """bestDisp among the minima of S over d (App. A.6).

    MODE_HH (8 paths) takes the first minimum (scalar loop).  MODE_SGBM
    (5 paths) fuses its WTA into the SIMD loop of the backward pass
    (``if( useSIMD )`` branch of computeDisparitySGBM, always taken on x86):
    lane i of an 8 x int16 register keeps the first minimum among
    d = i, i+8, i+16, ... (strict ``_minS > L0``), and the winner is the
    lowest lane holding the overall minimum (``LSBTab`` of the equality
    mask).  So ties break by (d mod 8) first, then by d.
    """
    if mode != 5:
        return S.argmin(-1)
    D = S.shape[-1]
    d = np.arange(D)
    rank = (d % SIMD_LANES) * D + d
    at_min = S == S.min(-1, keepdims=True)
    return d[np.where(at_min, rank, np.iinfo(np.int64).max).argmin(-1)]


def wta(S: np.ndarray, H, W, prm):
    """Returns disp (int16 [H, W], pre-median) following App. A.6."""
    minD, D = prm["minD"], prm["D"]
    minX1, maxX1 = geometry(W, minD, D)
    width1 = maxX1 - minX1
    INVALID = (minD - 1) * DISP_SCALE
    disp = np.full((H, W), INVALID, np.int64)
    if width1 <= 0:
        return disp.astype(np.int16)
    u = prm["uniq"]
    best = wta_best(S, prm["mode"])
    minS = S.min(-1)
    dd = np.arange(D)
    bad = ((S * (100 - u) < (minS * 100)[..., None])
           & (np.abs(best[..., None] - dd) > 1)).any(-1)
    sat = minS >= MAX_COST                               # OpenCV bestDisp == -1
    valid = ~bad & ~sat
    # neighbours clamped into [0, D) (only 0 < best < D-1 uses them; an external volume may
    # have D < 3 planes)
    bi = np.clip(best, 0, D - 1)
    Sm = np.take_along_axis(S, np.clip(bi - 1, 0, D - 1)[..., None], -1)[..., 0]
    S0 = np.take_along_axis(S, bi[..., None], -1)[..., 0]
    Sq = np.take_along_axis(S, np.clip(bi + 1, 0, D - 1)[..., None], -1)[..., 0]
    den = np.maximum(Sm + Sq - 2 * S0, 1)
    sub = best * DISP_SCALE + _cdiv((Sm - Sq) * DISP_SCALE + den, 2 * den)
    inner = (best > 0) & (best < D - 1)
    d16 = np.where(inner, sub, best * DISP_SCALE) + minD * DISP_SCALE
    disp[:, minX1:maxX1] = np.where(valid, d16, INVALID)
    # disp2: right-view argmin; OpenCV walks x descending with strict '>',
    # so among equal minS the largest x wins.
    disp2 = np.full((H, W), INVALID, np.int64)
    for y in range(H):
        cost2 = np.full(W, MAX_COST, np.int64)
        for x in range(width1 - 1, -1, -1):
            if not valid[y, x]:
                continue
            b = int(best[y, x])
            x2 = x + minX1 - b - minD
            if cost2[x2] > minS[y, x]:
                cost2[x2] = minS[y, x]
                disp2[y, x2] = b + minD
    # LR check
    md = prm["disp12"]
    for y in range(H):
        for x in range(minX1, maxX1):
            d1 = int(disp[y, x])
            if d1 == INVALID:
                continue
            _d = d1 >> DISP_SHIFT
            d_ = (d1 + DISP_SCALE - 1) >> DISP_SHIFT
            _x, x_ = x - _d, x - d_
            if (0 <= _x < W and disp2[y, _x] >= minD and abs(disp2[y, _x] - _d) > md and
                    0 <= x_ < W and disp2[y, x_] >= minD and abs(disp2[y, x_] - d_) > md):
                disp[y, x] = INVALID
    return disp.astype(np.int16)


def wta_index(S: np.ndarray, H, W, prm) -> np.ndarray:
    """The integer WTA index (int16 [H, W]): bestDisp in [0, D) where the pixel passes
    the uniqueness test and S is not saturated (App. A.6), -1 elsewhere and outside
    [minX1, maxX1); before the sub-pixel step, the disp12MaxDiff check and the median.
    The quantity BASELINE.json's north_star states its bit-exact bar on."""
    minD, D = prm["minD"], prm["D"]
    minX1, maxX1 = geometry(W, minD, D)
    out = np.full((H, W), -1, np.int64)
    if maxX1 <= minX1:
        return out.astype(np.int16)
    u = prm["uniq"]
    best = wta_best(S, prm["mode"])
    minS = S.min(-1)
    bad = ((S * (100 - u) < (minS * 100)[..., None])
           & (np.abs(best[..., None] - np.arange(D)) > 1)).any(-1)
    out[:, minX1:maxX1] = np.where(~bad & (minS < MAX_COST), best, -1)
    return out.astype(np.int16)


def median3(disp: np.ndarray) -> np.ndarray:
    """cv::medianBlur(ksize=3) on int16 with replicate border."""
    H, W = disp.shape
    p = np.pad(disp.astype(np.int64), 1, mode="edge")
    stack = np.stack([p[i:i + H, j:j + W] for i in range(3) for j in range(3)])
    return np.sort(stack, axis=0)[4].astype(np.int16)


# --------------------------------------------------------------------------
# Full matcher
# --------------------------------------------------------------------------
def check_supported(H, W, prm):
    """Range the GPU kernels reproduce bit-exactly."""
    if prm["D"] <= 0 or prm["D"] % 16 != 0:
        raise ValueError("numDisparities must be a positive multiple of 16")
    if prm["cost"] == COST_SGBM:
        maxpix = 2 * prm["ftzero"] + (255 >> 2)
        if prm["bs"] * prm["bs"] * maxpix + prm["P2"] > 16383:
            raise ValueError("blockSize/preFilterCap/P2 outside the int16-exact range")


def compute(left: np.ndarray, right: np.ndarray, params: dict, *, median=True,
            return_stages=False):
    """StereoSGBM(...).compute(left, right) restated.  Returns int16 [H, W]."""
    prm = normalize_params(params)
    left = np.asarray(left, np.uint8)
    right = np.asarray(right, np.uint8)
    if left.shape != right.shape or left.ndim != 2:
        raise ValueError("left/right must be same-size single-channel uint8")
    H, W = left.shape
    check_supported(H, W, prm)
    minX1, maxX1 = geometry(W, prm["minD"], prm["D"])
    if minX1 >= maxX1:
        out = np.full((H, W), (prm["minD"] - 1) * DISP_SCALE, np.int16)
        return (out, {}) if return_stages else out
    C = cost_volume(left, right, prm)
    S = aggregate(C, prm)
    raw = wta(S, H, W, prm)
    out = median3(raw) if median else raw
    if prm["speckle_ws"] > 0:
        out = filter_speckles(out, (prm["minD"] - 1) * DISP_SCALE, prm["speckle_ws"],
                              DISP_SCALE * prm["speckle_range"])
    if return_stages:
        return out, dict(C=C, S=S, raw=raw, wta=wta_index(S, H, W, prm))
    return out


def compute_volume(vol: np.ndarray, params: dict, offset: float = 0.0, scale: float = 1.0, *,
                   median=True, return_stages=False):
    """SGM over an external f32 cost volume (mc-cnn): the
    quantised cost (``quantize_volume``) feeds the same path recurrence,
    WTA / uniqueness / sub-pixel / LR and 3×3 median as ``compute``."""
    prm = normalize_params(dict(params, cost=COST_VOLUME))
    v = np.asarray(vol, np.float32)
    H, W = v.shape[-2:]
    if prm["P2"] > 16383 - VOLUME_CMAX:
        raise ValueError("volume mode needs P2 <= %d" % (16383 - VOLUME_CMAX))
    minX1, maxX1 = geometry(W, prm["minD"], prm["D"])
    if minX1 >= maxX1:
        out = np.full((H, W), (prm["minD"] - 1) * DISP_SCALE, np.int16)
        return (out, {}) if return_stages else out
    C = quantize_volume(v, prm, offset, scale)
    S = aggregate(C, prm)
    raw = wta(S, H, W, prm)
    out = median3(raw) if median else raw
    if prm["speckle_ws"] > 0:
        out = filter_speckles(out, (prm["minD"] - 1) * DISP_SCALE, prm["speckle_ws"],
                              DISP_SCALE * prm["speckle_range"])
    if return_stages:
        return out, dict(C=C, S=S, raw=raw)
    return out


def right_matcher_params(params: dict) -> dict:
    """ximgproc::createRightMatcher(StereoSGBM)."""
    q = dict(params)
    minD = q.get("minDisparity", 0)
    D = q.get("numDisparities", 16)
    q.update(minDisparity=-(minD + D) + 1, uniquenessRatio=0,
             disp12MaxDiff=1000000, speckleWindowSize=0)
    return q


def filter_speckles(img: np.ndarray, newval: int, max_speckle: int, max_diff: int):
    """cv::filterSpeckles (4-connected regions whose neighbours differ by at
    most max_diff; regions of <= max_speckle pixels are set to newval)."""
    img = img.astype(np.int64).copy()
    H, W = img.shape
    label = np.zeros((H, W), np.int64)
    is_bad = {}
    cur = 0
    for y in range(H):
        for x in range(W):
            if img[y, x] == newval:
                continue
            if label[y, x]:
                if is_bad[label[y, x]]:
                    img[y, x] = newval
                continue
            cur += 1
            label[y, x] = cur
            stack = [(y, x)]
            count = 0
            while stack:
                py, px = stack.pop()
                count += 1
                dp = img[py, px]
                for qy, qx in ((py + 1, px), (py - 1, px), (py, px + 1), (py, px - 1)):
                    if 0 <= qy < H and 0 <= qx < W and not label[qy, qx]:
                        dq = img[qy, qx]
                        if dq != newval and abs(dp - dq) <= max_diff:
                            label[qy, qx] = cur
                            stack.append((qy, qx))
            bad = count <= max_speckle
            is_bad[cur] = bad
            if bad:
                img[y, x] = newval
    return img.astype(np.int16)
