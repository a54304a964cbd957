"""Pins the CPU restatement (oracle/) with hand-derived known answers and
checks the two independent restatements (numpy direction-wise, C following
OpenCV's row-streaming loops) agree bit for bit.  CPU only."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from oracle import ref_c, sgm_np
from stereo_match_amd import synthetic

DS = sgm_np.DISP_SCALE


def test_k1_constant_shift_recovered():
    """K1: right = left shifted by s -> integer WTA index s on the interior."""
    s = 5
    left, right = synthetic.shifted_pair(48, 96, s, seed=11)
    for p in (synthetic.parity_params(16), synthetic.headline_params(16)):
        out = sgm_np.compute(left, right, p)
        inner = out[3:-3, 16 + 3:-3].astype(int)
        assert np.mean((inner + 8) >> 4 == s) > 0.99


@pytest.mark.parametrize("p", [synthetic.parity_params(16), synthetic.headline_params(16),
                               dict(synthetic.parity_params(32), mode=8)])
def test_k2a_constant_images(p):
    """K2a: constant 63 (= ftzero) images -> zero cost everywhere -> S constant
    -> d=0 valid for x >= minX1, INVALID (-16) left of it, median-invariant."""
    img = np.full((20, 70), 63, np.uint8)
    out = sgm_np.compute(img, img, p)
    D = p["numDisparities"]
    assert (out[:, :D] == -16).all()
    assert (out[:, D:] == 0).all()


def _wta_one_pixel(S_row, uniq):
    D = len(S_row)
    S = np.asarray(S_row, np.int64).reshape(1, 1, D)
    prm = sgm_np.normalize_params(dict(numDisparities=D, uniquenessRatio=uniq, disp12MaxDiff=1000000))
    return int(sgm_np.wta(S, 1, D + 1, prm)[0, D])


def test_k2b_uniqueness_ratio():
    """K2b: S=[100,300,110,500..]: 110*85 < 100*100 and |0-2|>1 -> INVALID;
    S[2]=120 passes (120*85 >= 10000) -> d16 = 0.  S carries no offset (Cbuf is
    seeded with P2, so L is the textbook value)."""
    assert _wta_one_pixel([100, 300, 110] + [500] * 13, 15) == -16
    assert _wta_one_pixel([100, 300, 120] + [500] * 13, 15) == 0
    # |best-d| <= 1 never disqualifies
    assert _wta_one_pixel([100, 101] + [500] * 14, 15) == 0


def test_k3_subpixel_c_truncation():
    """K3: S=[10,4,13,...]: den=15, num=(10-13)*16+15=-33, -33/30 = -1 (C), not -2."""
    assert _wta_one_pixel([10, 4, 13] + [900] * 13, 0) == 16 - 1
    # positive numerator: S=[13,4,10]: num=(13-10)*16+15=63, 63/30=2 -> 18
    assert _wta_one_pixel([13, 4, 10] + [900] * 13, 0) == 16 + 2
    # best at the border: no interpolation
    assert _wta_one_pixel([1, 4, 13] + [900] * 13, 0) == 0
    assert _wta_one_pixel([900] * 15 + [3], 0) == 15 * DS


def _wta_mode(S_row, mode):
    D = len(S_row)
    S = np.asarray(S_row, np.int64).reshape(1, 1, D)
    prm = sgm_np.normalize_params(dict(numDisparities=D, uniquenessRatio=0, disp12MaxDiff=1000000, mode=mode))
    return int(sgm_np.wta(S, 1, D + 1, prm)[0, D])


def test_k7_simd_lane_tie_break():
    """K7: MODE_SGBM's WTA runs in OpenCV's CV_SIMD128 loop (x86): with equal
    minima at d=2 and d=9, lane 1 (d=9) beats lane 2 (d=2); MODE_HH's scalar
    loop keeps the first minimum.  d=9 interpolates S[8..10] = 50,20,80:
    den = 90, num = (50-80)*16+90 = -390, -390/180 = -2 (C) -> 9*16-2."""
    S = [90] * 16
    S[2] = S[9] = 20
    S[1], S[3], S[8], S[10] = 40, 60, 50, 80
    assert _wta_mode(S, 5) == 9 * DS - 2
    # 8 paths: first minimum d=2, S[1..3] = 40,20,60: den 60, num (40-60)*16+60 = -260 -> -2
    assert _wta_mode(S, 8) == 2 * DS - 2
    # same lane: the smaller d wins in both modes
    T = [90] * 16
    T[3] = T[11] = 20
    assert _wta_mode(T, 5) == _wta_mode(T, 8) == 3 * DS  # den 140, num 140 -> 140/280 = 0
    # the rule in the vectorised helper: rank by (d mod 8, d)
    rng = np.random.default_rng(3)
    for _ in range(200):
        row = rng.integers(0, 4, 32)
        m = row.min()
        cand = [d for d in range(32) if row[d] == m]
        want = min(cand, key=lambda d: (d % 8, d))
        assert int(sgm_np.wta_best(row[None], 5)[0]) == want
        assert int(sgm_np.wta_best(row[None], 8)[0]) == cand[0]


def test_k3b_all_saturated_is_invalid():
    """OpenCV's bestDisp stays -1 when every S == 32767 -> pixel invalid."""
    assert _wta_one_pixel([32767] * 16, 0) == -16
    assert _wta_one_pixel([32767] * 16, 15) == -16


@pytest.mark.parametrize("minD", [0, 4, -7, -15])
def test_k4_border_columns_invalid(minD):
    """K4: columns outside [max(minD+D,0), W+min(minD,0)) are (minD-1)*16."""
    l, r, _ = synthetic.random_dot_pair(24, 64, 16, seed=5)
    p = dict(synthetic.parity_params(16), minDisparity=minD)
    raw = sgm_np.compute(l, r, p, return_stages=True)[1]["raw"]
    minX1, maxX1 = sgm_np.geometry(64, minD, 16)
    inv = (minD - 1) * DS
    assert (raw[:, :minX1] == inv).all() and (raw[:, maxX1:] == inv).all()
    assert (raw[:, minX1:maxX1] != inv).any()


def test_k5_census_bit_patterns():
    img = np.zeros((9, 11), np.uint8)
    img[4, 5] = 200
    c = sgm_np.census9x7(img)
    assert int(c[4, 5]) == (1 << 62) - 1         # every neighbour darker
    assert int(c[4, 4]) == 0                      # nothing darker than 0
    img2 = np.full((9, 11), 100, np.uint8)
    img2[1, 1] = 0                                # (dy,dx)=(-3,-4) from (4,5): bit 0
    assert int(sgm_np.census9x7(img2)[4, 5]) == 1
    img2[7, 9] = 0                                # (dy,dx)=(+3,+4): last bit 61
    assert int(sgm_np.census9x7(img2)[4, 5]) == 1 | (1 << 61)
    assert np.array_equal(sgm_np.census9x7(img2), ref_c.census(img2))


def test_params_normalisation():
    q = sgm_np.normalize_params(dict(P1=0, P2=0, blockSize=0, preFilterCap=0, uniquenessRatio=-1,
                                     disp12MaxDiff=0, numDisparities=16))
    assert (q["P1"], q["P2"], q["bs"], q["ftzero"], q["uniq"], q["disp12"]) == (2, 5, 5, 15, 10, 1)
    assert sgm_np.normalize_params(dict(P1=600, P2=100))["P2"] == 601
    assert sgm_np.normalize_params(dict(preFilterCap=62))["ftzero"] == 63
    with pytest.raises(ValueError):
        sgm_np.compute(np.zeros((4, 40), np.uint8), np.zeros((4, 40), np.uint8), dict(numDisparities=24))


def test_box_frozen_bottom_rows_differ_between_modes():
    """MODE_SGBM freezes C for y > H-1-SH2; MODE_HH leaves the P2 seed (C=0)."""
    rng = np.random.default_rng(0)
    pix = rng.integers(0, 50, (10, 20, 16))
    c5 = sgm_np.box_cost_sgbm(pix, 5, 5)
    c8 = sgm_np.box_cost_sgbm(pix, 5, 8)
    assert np.array_equal(c5[:8], c8[:8])
    assert np.array_equal(c5[8], c5[7]) and np.array_equal(c5[9], c5[7])
    assert (c8[8:] == 0).all()


def test_all_invalid_when_too_narrow():
    l = np.zeros((5, 16), np.uint8)
    out = sgm_np.compute(l, l, dict(numDisparities=16))
    assert (out == -16).all()
    assert np.array_equal(out, ref_c.compute(l, l, dict(numDisparities=16)))


def test_golden_fixtures_reproduce(golden_cases):
    for name, left, right, p, expected, raw in golden_cases:
        out, stg = sgm_np.compute(left, right, p, return_stages=True)
        assert np.array_equal(out, expected), name
        assert np.array_equal(stg.get("raw", out), raw), name
        assert np.array_equal(ref_c.compute(left, right, p), expected), name


@settings(max_examples=40, deadline=None)
@given(H=st.integers(1, 24), W=st.integers(17, 70), D=st.sampled_from([16, 32]),
       minD=st.integers(-20, 6), bs=st.sampled_from([1, 3, 5, 7]), mode=st.sampled_from([5, 8]),
       cost=st.sampled_from([0, 1]), uniq=st.sampled_from([0, 5, 15]), d12=st.sampled_from([1, 3, 1000000]),
       pfc=st.sampled_from([1, 20, 63]), seed=st.integers(0, 2 ** 31 - 1))
def test_k6_numpy_c_bit_exact(H, W, D, minD, bs, mode, cost, uniq, d12, pfc, seed):
    rng = np.random.default_rng(seed)
    left = rng.integers(0, 256, (H, W)).astype(np.uint8)
    shift = int(rng.integers(0, D))
    right = np.roll(left, -shift, 1)
    right = np.clip(right.astype(int) + rng.integers(-4, 5, right.shape), 0, 255).astype(np.uint8)
    p = dict(minDisparity=minD, numDisparities=D, blockSize=bs, P1=8 * bs * bs, P2=32 * bs * bs,
             disp12MaxDiff=d12, uniquenessRatio=uniq, preFilterCap=pfc, mode=mode, cost=cost)
    if cost == 1:
        p.update(P1=10, P2=120)
    try:
        a, stg = sgm_np.compute(left, right, p, return_stages=True)
    except ValueError:
        return
    c, cw = ref_c.compute_wta(left, right, p)
    assert np.array_equal(a, c)
    if stg:  # the integer WTA index (SURVEY §8b wta_out): both restatements agree
        assert np.array_equal(stg["wta"], cw)
    else:
        assert (cw == -1).all()


def test_wta_index_kat():
    """K10: the integer WTA index on a constant shift is the shift on the interior, -1 on
    the border band x < minX1, and rejected pixels (uniqueness) carry -1 while their
    disparity is INVALID before the LR check."""
    left, right = synthetic.shifted_pair(40, 120, 5, seed=3)
    p = dict(minDisparity=0, numDisparities=16, blockSize=5, P1=600, P2=2400, disp12MaxDiff=1, uniquenessRatio=15,
             preFilterCap=63, mode=5, cost=0)
    raw, wta = ref_c.compute_wta(left, right, p, median=False)
    assert (wta[:, :16] == -1).all()
    inner = wta[4:-4, 20:-4]
    assert (inner == 5).mean() > 0.99
    # -1 exactly where the pre-LR map would be invalid: the LR check only removes more
    assert ((wta == -1) <= (raw == -16)).all()


def test_speckle_filter_matches_c():
    rng = np.random.default_rng(3)
    img = rng.integers(-16, 200, (20, 30)).astype(np.int16)
    img[rng.random(img.shape) < 0.3] = -16
    a = sgm_np.filter_speckles(img, -16, 3, 32)
    lib = ref_c.load()
    b = img.copy()
    lib.sgm_ref_filter_speckles.argtypes = [ref_c.ctypes.c_void_p] + [ref_c.ctypes.c_int] * 5
    lib.sgm_ref_filter_speckles(b.ctypes.data, 20, 30, -16, 3, 32)
    assert np.array_equal(a, b)


# ---------------------------------------------------------------- mc-cnn volume mode
def test_volume_quantisation_kat():
    """q = rint((c + offset) * scale) (float32, half-even), clamp [0, 4095], NaN -> 4095."""
    prm = sgm_np.normalize_params(dict(numDisparities=16, cost=2))
    c = np.array([0.5, 1.5, 2.5, -0.4, -7, 4095.4, 4095.6, 1e9, np.inf, -np.inf, np.nan, 3.0],
                 np.float32)
    W = c.size + 16  # minX1 = 16: the samples sit at x = 16..
    vol = np.zeros((16, 1, W), np.float32)
    vol[0, 0, 16:] = c
    q = sgm_np.quantize_volume(vol, prm, 0.0, 1.0)[0, :, 0]
    assert q.tolist() == [0, 2, 2, 0, 0, 4095, 4095, 4095, 4095, 0, 4095, 3]
    q2 = sgm_np.quantize_volume(vol, prm, 0.5, 2.0)[0, :, 0]  # (c + .5) * 2
    assert q2[:3].tolist() == [2, 4, 6]


def test_volume_constant_shift_recovered():
    """KAT: a volume that is 0 at d = 7 and 1 elsewhere → raw WTA = 7·16 wherever LR holds."""
    H, W, D = 20, 90, 16
    vol = np.ones((D, H, W), np.float32)
    vol[7] = 0
    p = dict(synthetic.cost_volume_params(D))
    out, st = sgm_np.compute_volume(vol, p, 0.0, 1000.0, return_stages=True)
    raw = st["raw"]
    assert np.all(raw[:, D:] == 7 * 16)
    assert np.all(raw[:, :D] == -16)
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, 1000.0))


def test_golden_volume_fixtures_reproduce(golden_volume_cases):
    for name, vol, p, off, sc, expected, raw in golden_volume_cases:
        out, st = sgm_np.compute_volume(vol, p, off, sc, return_stages=True)
        assert np.array_equal(out, expected), name
        assert np.array_equal(st["raw"], raw), name
        assert np.array_equal(ref_c.compute_volume(vol, p, off, sc), expected), name


@settings(max_examples=25, deadline=None)
@given(H=st.integers(1, 24), W=st.integers(17, 80), Dk=st.integers(1, 2), minD=st.integers(-4, 4),
       mode=st.sampled_from([5, 8]), scale=st.sampled_from([1.0, 37.5, 4000.0]),
       nan_frac=st.sampled_from([0.0, 0.05]), seed=st.integers(0, 2**31 - 1))
def test_volume_numpy_c_bit_exact(H, W, Dk, minD, mode, scale, nan_frac, seed):
    D = 16 * Dk
    rng = np.random.default_rng(seed)
    vol = rng.standard_normal((D, H, W)).astype(np.float32)
    vol[rng.random(vol.shape) < nan_frac] = np.nan
    p = dict(synthetic.cost_volume_params(D), minDisparity=minD, mode=mode, P1=int(rng.integers(1, 60)),
             P2=int(rng.integers(60, 600)))
    assert np.array_equal(sgm_np.compute_volume(vol, p, 0.25, scale), ref_c.compute_volume(vol, p, 0.25, scale))


@settings(max_examples=20, deadline=None)
@given(H=st.integers(1, 16), W=st.integers(4, 70), D=st.integers(1, 45), minD=st.integers(-4, 4),
       mode=st.sampled_from([5, 8]), uniq=st.sampled_from([0, 15, 70]), seed=st.integers(0, 2**31 - 1))
def test_volume_any_plane_count_numpy_c_bit_exact(H, W, D, minD, mode, uniq, seed):
    """External volumes with any plane count (mc-cnn's 228, mapTo3D_mc_cnn.py:71): both
    restatements take D as given (OpenCV's %16 assert is StereoSGBM's own-cost rule)."""
    rng = np.random.default_rng(seed)
    vol = rng.random((D, H, W), dtype=np.float32)
    p = dict(synthetic.cost_volume_params(D), minDisparity=minD, mode=mode, uniquenessRatio=uniq)
    assert np.array_equal(sgm_np.compute_volume(vol, p, 0.0, 4000.0), ref_c.compute_volume(vol, p, 0.0, 4000.0))


def test_volume_reference_plane_count_kat():
    """KAT: 228 planes (the reference's mc-cnn volume), 0 at d = 227 (the last plane, where
    no sub-pixel step applies) and 1 elsewhere -> raw WTA 227·16 on the domain."""
    H, W, D = 6, 240, 228
    vol = np.ones((D, H, W), np.float32)
    vol[D - 1] = 0
    p = dict(synthetic.cost_volume_params(D))
    out, st = sgm_np.compute_volume(vol, p, 0.0, 1000.0, return_stages=True)
    assert np.all(st["raw"][:, D:] == (D - 1) * 16)
    assert np.all(st["raw"][:, :D] == -16)
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, 1000.0))


def test_volume_rejects_bad_shapes():
    with pytest.raises(ValueError):
        sgm_np.compute_volume(np.zeros((16, 4, 40), np.float32), dict(numDisparities=32))
    with pytest.raises(ValueError):
        ref_c.compute_volume(np.zeros((16, 4, 40), np.float32), dict(numDisparities=32))
    with pytest.raises(ValueError):  # P2 outside the int16-exact range
        sgm_np.compute_volume(np.zeros((16, 4, 40), np.float32), dict(numDisparities=16, P2=20000))


# ---------------------------------------------------------------- StereoBM
def test_bm_prefilter_xsobel_kat():
    from oracle import bm_np

    img = np.zeros((5, 6), np.uint8)
    img[:, 3:] = 100  # vertical step between x=2 and x=3
    p = bm_np.prefilter_xsobel(img, 31)
    assert np.all(p[:, 0] == 31) and np.all(p[:, -1] == 31)
    assert np.all(p[:4, 2] == 62) and np.all(p[:4, 3] == 62)  # 4*100 clipped to +cap
    assert np.all(p[:4, 1] == 31) and np.all(p[:4, 4] == 31)
    assert np.all(p[4] == 31)  # odd height: last row = cap


def test_bm_constant_shift_recovered():
    from oracle import bm_np

    left, right = synthetic.shifted_pair(60, 200, 7, seed=3)
    out = bm_np.stereo_bm(left, right, dict(numDisparities=32, blockSize=9, uniquenessRatio=0,
                                            textureThreshold=0))
    roi = out[4:-4, 31 + 4:-4]
    assert np.mean(np.abs(roi.astype(int) - 112) <= 2) > 0.97
    assert np.all(out[:4] == -16) and np.all(out[:, :31 + 4] == -16)


def test_bm_validate_and_arguments():
    from oracle import bm_np

    left, right, _ = synthetic.random_dot_pair(40, 120, 32, seed=4)
    a = bm_np.stereo_bm(left, right, dict(numDisparities=32, blockSize=7, disp12MaxDiff=1))
    b = bm_np.stereo_bm(left, right, dict(numDisparities=32, blockSize=7))
    assert np.all((a == b) | (a == -16))
    for bad in (dict(blockSize=4), dict(blockSize=6), dict(numDisparities=24), dict(preFilterCap=64)):
        with pytest.raises(ValueError):
            bm_np.stereo_bm(left, right, dict(dict(numDisparities=32, blockSize=7), **bad))


def test_k8_int16_wrap_and_saturation_of_the_box_sums():
    """K8 (x86 OpenCV arithmetic, oracle/sgm_ref.c header): constant 0 vs
    255 pair, disparity_test.py's blockSize 23 / preFilterCap 1 / P2 887.
    Interior pixel cost = (255 >> 2) = 63 (the clipped derivatives are flat),
    horizontal sum 23 * 63 = 1449.  Row 0 of C is built by the scalar loop
    with int16 casts: 887 + 12 * 1449 + 11 * 1449 wraps to -31322.  Rows >= 1
    use the saturating SIMD update (C - hsumSub) + hsumAdd: -31322 - 1449
    saturates at -32768, + 1449 = -31319, and stays there."""
    p = dict(minDisparity=0, numDisparities=16, blockSize=23, P1=222, P2=887, disp12MaxDiff=20,
             uniquenessRatio=0, preFilterCap=1, mode=5, cost=0)
    l = np.zeros((40, 80), np.uint8)
    r = np.full((40, 80), 255, np.uint8)
    C = ref_c.cost_volume(l, r, p)
    assert (C[0, 12:51] == -31322).all()  # windows clear of the border columns
    assert (C[1:, 12:51] == -31319).all()


def test_k9_colour_replicated_channels():
    """K9: a BGR pair whose three channels equal the gray pair costs three
    times the gray cost per pixel (each channel adds its own derivative and
    raw BT terms), inside the int16-exact range."""
    l, r, _ = synthetic.random_dot_pair(30, 90, 16, seed=4)
    p = dict(synthetic.parity_params(16), blockSize=3, P1=10, P2=96)
    C1 = ref_c.cost_volume(l, r, p).astype(np.int64)
    C3 = ref_c.cost_volume(np.repeat(l[..., None], 3, -1), np.repeat(r[..., None], 3, -1), p).astype(np.int64)
    assert np.array_equal(C3 - 96, 3 * (C1 - 96))
