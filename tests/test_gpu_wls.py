"""GPU parity of the WLS post-filter and of the whole compute_disparity
(left SGBM + right SGBM + WLS) against the CPU restatements.  Bar:
bit-exact int16 (the kernels run the oracle's float32 operation order with
FP contraction off).  Parity with ximgproc itself is unpinned."""
import numpy as np
import pytest

from oracle import ref_c, sgm_np, wls_np
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(0)
    yield e
    e.close()


def wls_params(p: dict, H, W) -> _lib.SmWlsParams:
    q = wls_np.normalize_wls(p, H, W)
    return _lib.SmWlsParams(q["lmbda"], q["sigma"], q["lrc_thresh"], q["radius"], int(q["use_confidence"]),
                            q["min_disp"], q["left_offset"], q["right_offset"], q["top_offset"],
                            q["bottom_offset"], q["num_iter"], q["attenuation"], q["roll_off"])


def test_golden_wls_fixtures(eng, golden_wls_cases):
    for name, displ, dispr, guide, p, expected in golden_wls_cases:
        out = eng.wls_filter(displ, guide, dispr, wls_params(p, *displ.shape))
        assert np.array_equal(out, expected), f"{name}: {np.sum(out != expected)} px differ"


def _pair_maps(H, W, D, seed, ws=5, minD=0):
    left, right, gt = synthetic.random_dot_pair(H, W, D, seed=seed)
    settings = dict(synthetic.parity_params(D, window_size=ws), minDisparity=minD)
    lp = dict(settings, uniquenessRatio=0, disp12MaxDiff=1000000)
    displ = ref_c.compute(left, right, lp)
    dispr = ref_c.compute(right, left, sgm_np.right_matcher_params(settings))
    return left, right, gt, settings, displ, dispr


_rng = np.random.default_rng(77)
_CASES = [dict(H=int(_rng.integers(2, 80)), W=int(_rng.integers(40, 260)), D=16 * int(_rng.integers(1, 3)),
               minD=int(_rng.integers(-4, 4)), r=int(_rng.integers(0, 5)), lam=float(_rng.choice([10.0, 8000.0, 80000.0])),
               sigma=float(_rng.choice([0.7, 1.2, 3.0])), top=int(_rng.integers(0, 3)), seed=int(_rng.integers(0, 1 << 30)))
          for _ in range(10)]


@pytest.mark.parametrize("c", _CASES, ids=lambda c: "H{H}W{W}D{D}m{minD}r{r}".format(**c))
def test_wls_random_vs_oracle(eng, c):
    left, _, _, _, displ, dispr = _pair_maps(c["H"], c["W"], c["D"], c["seed"], minD=c["minD"])
    H, W = displ.shape
    p = dict(lmbda=c["lam"], sigma=c["sigma"], radius=c["r"], min_disp=c["minD"],
             left_offset=max(0, c["minD"] + c["D"]), right_offset=max(0, -c["minD"]),
             top_offset=min(c["top"], H - 1), bottom_offset=0)
    out = eng.wls_filter(displ, left, dispr, wls_params(p, H, W))
    assert np.array_equal(out, wls_np.wls_filter(displ, left, dispr, p))


def test_wls_no_confidence(eng):
    left, _, _, _, displ, _ = _pair_maps(50, 160, 32, 5)
    p = dict(lmbda=8000.0, sigma=1.5, use_confidence=False)
    out = eng.wls_filter(displ, left, None, wls_params(p, *displ.shape))
    assert np.array_equal(out, wls_np.wls_filter(displ, left, None, p))


def test_wls_full_size_kitti(eng):
    H, W, D = synthetic.CONFIGS["kitti"]
    left, _, gt, _, displ, dispr = _pair_maps(H, W, D, 42)
    p = dict(lmbda=80000.0, sigma=1.2, radius=3, left_offset=D)
    out = eng.wls_filter(displ, left, dispr, wls_params(p, H, W))
    exp = wls_np.wls_filter(displ, left, dispr, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"
    roi = out[:, D:]
    assert np.all(roi >= 0)
    assert np.mean(np.abs(((roi.astype(np.int64) + 8) >> 4) - gt[:, D:]) <= 1) > 0.97


def test_compute_disparity_end_to_end():
    """stereo_vision.compute_disparity drop-in: (displ, filtered) vs the
    oracle chain run in the reference's order."""
    import stereo_match_amd as sm

    H, W, D = 96, 300, 64
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=8)
    s = dict(sm.DEFAULT_SETTINGS, window_size=5, num_disparities=D, lmbda=80000, sigma=1.2)
    displ, filt = sm.compute_disparity(left, right, s)
    lp = dict(synthetic.parity_params(D), blockSize=s["block_size"], uniquenessRatio=0, disp12MaxDiff=1000000,
              minDisparity=s["min_disparity"], preFilterCap=s["pre_filter_cap"], speckleRange=s["speckle_range"])
    settings = dict(lp, uniquenessRatio=s["uniqueness_ratio"], disp12MaxDiff=s["disp12_max_diff"])
    exp_l = ref_c.compute(left, right, lp)
    exp_r = ref_c.compute(right, left, sgm_np.right_matcher_params(settings))
    assert np.array_equal(displ, exp_l)
    wp = dict(lmbda=80000.0, sigma=1.2, radius=-(-s["block_size"] // 2), min_disp=s["min_disparity"],
              left_offset=max(0, s["min_disparity"] + D), right_offset=max(0, -s["min_disparity"]))
    assert np.array_equal(filt, wls_np.wls_filter(exp_l, left, exp_r, wp))
    # the one-call C-ABI flow gives the same maps
    eng = _lib.engine(0)
    sp = synthetic.to_sm_params(settings)
    d2, f2 = eng.compute_disparity(left, right, sp, wls_params(dict(wp), H, W))
    assert np.array_equal(d2, displ) and np.array_equal(f2, filt)
    dw = _lib.wls_default_params(sp)
    assert (dw.left_offset, dw.right_offset, dw.depth_discontinuity_radius, dw.min_disp) == (D, 0, 3, 0)


def test_compute_disparity_batch_device_and_torch():
    import torch

    import stereo_match_amd as sm
    from stereo_match_amd import wls

    H, W, D, n = 64, 220, 32, 3
    pairs = [synthetic.random_dot_pair(H, W, D, seed=50 + i)[:2] for i in range(n)]
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    settings = synthetic.parity_params(D)
    sp = synthetic.to_sm_params(settings)
    wp = _lib.wls_default_params(sp)
    wp.lambda_, wp.sigma_color = 80000.0, 1.2
    outs = [torch.empty((n, H, W), dtype=torch.int16, device="cuda") for _ in range(3)]
    eng = _lib.engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.compute_disparity_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, sp, wp,
                                       *(o.data_ptr() for o in outs))
    got = [o.cpu().numpy() for o in outs]
    for i, (a, b) in enumerate(pairs):
        d2, f2 = eng.compute_disparity(a, b, sp, wp)
        assert np.array_equal(got[0][i], d2) and np.array_equal(got[2][i], f2), i
    # torch tensors through the Python filter object
    m = sm.StereoSGBM_create(numDisparities=D, blockSize=5, P1=600, P2=2400, disp12MaxDiff=1, uniquenessRatio=15,
                             preFilterCap=63)
    f = wls.createDisparityWLSFilter(m)
    f.setLambda(80000.0)
    f.setSigmaColor(1.2)
    t = f.filter(outs[0][0], L[0], None, outs[1][0])
    assert np.array_equal(t.cpu().numpy(), got[2][0])


def test_wls_bad_args(eng):
    d = np.zeros((10, 40), np.int16)
    g = np.zeros((10, 40), np.uint8)
    with pytest.raises(ValueError):
        eng.wls_filter(d, g, None, wls_params(dict(), 10, 40))  # confidence needs dispr
    with pytest.raises(ValueError):
        eng.wls_filter(d, g, d, wls_params(dict(left_offset=-1), 10, 40))


@pytest.mark.parametrize("H,W,r", [(2, 20, 6), (3, 24, 64), (1, 40, 5), (5, 2, 9)])
def test_wls_radius_wider_than_map(eng, H, W, r):
    # the confidence window reflects more than once (cv::borderInterpolate REFLECT_101)
    rng = np.random.default_rng(H * 1000 + W + r)
    displ = rng.integers(-16, 40 * 16, (H, W)).astype(np.int16)
    dispr = (-rng.integers(0, 40 * 16, (H, W))).astype(np.int16)
    guide = rng.integers(0, 256, (H, W)).astype(np.uint8)
    p = dict(lmbda=8000.0, sigma=1.5, lrc_thresh=24, radius=r, use_confidence=True, left_offset=0,
             right_offset=0, top_offset=0, bottom_offset=0, num_iter=2, min_disp=0)
    out = eng.wls_filter(displ, guide, dispr, wls_params(p, H, W))
    assert np.array_equal(out, wls_np.wls_filter(displ, guide, dispr, p))


@pytest.mark.parametrize("lam", [0.0, 80000.0, 2.0e6, 1.0e7, 3.0e8])
def test_wls_pivot_reciprocal_both_paths(eng, lam):
    # pivots <= 1 + 2*lambda: below 2^24 the smoother uses rcp + one FMA step (exact there,
    # tools/ubench/rcp_exact.hip), above it IEEE division; both must equal the oracle
    H, W = 30, 160
    rng = np.random.default_rng(int(lam) % 1000 + 7)
    displ = rng.integers(-16, 40 * 16, (H, W)).astype(np.int16)
    dispr = (-rng.integers(0, 40 * 16, (H, W))).astype(np.int16)
    guide = rng.integers(0, 256, (H, W)).astype(np.uint8)
    p = dict(lmbda=lam, sigma=1.2, lrc_thresh=24, radius=3, use_confidence=True, left_offset=20,
             right_offset=0, top_offset=0, bottom_offset=0, num_iter=3, min_disp=0)
    out = eng.wls_filter(displ, guide, dispr, wls_params(p, H, W))
    with np.errstate(all="ignore"):  # lambda 3e8: float32 pivots cancel to 0 (inf/nan) in both
        ref = wls_np.wls_filter(displ, guide, dispr, p)
    assert np.array_equal(out, ref)


from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(H=st.integers(2, 60), W=st.integers(20, 200), lo=st.integers(0, 40), ro=st.integers(0, 10),
       to=st.integers(0, 5), bo=st.integers(0, 5), r=st.integers(0, 6), lam=st.floats(0.0, 1e5),
       sigma=st.floats(0.3, 5.0), lrc=st.integers(0, 64), conf=st.booleans(), it=st.integers(1, 4),
       seed=st.integers(0, 2**31 - 1))
def test_hypothesis_wls_vs_oracle(eng, H, W, lo, ro, to, bo, r, lam, sigma, lrc, conf, it, seed):
    rng = np.random.default_rng(seed)
    displ = rng.integers(-16, 40 * 16, (H, W)).astype(np.int16)
    dispr = (-rng.integers(0, 40 * 16, (H, W))).astype(np.int16)
    guide = rng.integers(0, 256, (H, W)).astype(np.uint8)
    p = dict(lmbda=float(np.float32(lam)), sigma=float(np.float32(sigma)), lrc_thresh=lrc, radius=r,
             use_confidence=conf, left_offset=lo, right_offset=ro, top_offset=to, bottom_offset=bo, num_iter=it,
             min_disp=int(rng.integers(-3, 3)))
    out = eng.wls_filter(displ, guide, dispr if conf else None, wls_params(p, H, W))
    assert np.array_equal(out, wls_np.wls_filter(displ, guide, dispr if conf else None, p))


def test_compute_disparity_repeatable_with_side_stream_prepare():
    """The WLS guide-only work (weights, pivots) runs on its own stream beside the two
    matchers; every call must give the filter-alone result.  This caught a store-data
    hazard (sm_wls.hpp tile_store) that only showed with kernels running side by side."""
    import torch

    import stereo_match_amd as sm
    from stereo_match_amd import wls
    from stereo_match_amd.stereo_vision import matcher_from_settings

    for D in (64, 128):
        s = dict(sm.DEFAULT_SETTINGS, window_size=5, num_disparities=D)
        H, W = 120, 420
        gl, gr, _ = synthetic.random_dot_pair(H, W, D, seed=D + 3)
        lm = matcher_from_settings(s)
        prm = lm.params()
        wf = wls.createDisparityWLSFilter(lm)
        wf.setLambda(s["lmbda"])
        wf.setSigmaColor(s["sigma"])
        wp = wf.params(H, W)
        eng = _lib.Engine(0)
        try:
            L = torch.tensor(gl, device="cuda")
            R = torch.tensor(gr, device="cuda")
            dl = torch.empty((H, W), dtype=torch.int16, device="cuda")
            dr = torch.empty_like(dl)
            fo = torch.empty_like(dl)
            first = None
            for i in range(12):
                eng.compute_disparity_batch_device(L.data_ptr(), R.data_ptr(), 1, H * W, H, W, W, prm, wp,
                                                   dl.data_ptr(), dr.data_ptr(), fo.data_ptr())
                eng.synchronize()
                if first is None:
                    first = (dl.cpu().numpy(), dr.cpu().numpy())
                    alone = eng.wls_filter(first[0], gl, first[1], wp)
                assert np.array_equal(fo.cpu().numpy(), alone), (D, i)
        finally:
            eng.close()


def test_compute_disparity_on_caller_stream():
    """After sm_set_stream the right matcher (twin context, own stream) and the WLS
    guide work (third stream) still fork from and join into the caller's stream:
    the maps written there equal the default-stream call's, read right after a
    synchronize of that stream only (twin ordering after sm_set_stream)."""
    import torch

    H, W, D, n = 80, 260, 32, 2
    pairs = [synthetic.random_dot_pair(H, W, D, seed=70 + i)[:2] for i in range(n)]
    sp = synthetic.to_sm_params(synthetic.parity_params(D))
    wp = _lib.wls_default_params(sp)
    wp.lambda_, wp.sigma_color = 8000.0, 1.5
    eng = _lib.Engine(0)
    try:
        L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
        R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
        outs = []
        for use_stream in (False, True):
            dl, dr, fo = (torch.full((n, H, W), 99, dtype=torch.int16, device="cuda") for _ in range(3))
            s = torch.cuda.Stream()
            torch.cuda.synchronize()  # the inputs and the 99-filled outputs are in place
            if use_stream:
                eng.set_stream(s.cuda_stream)
            try:
                eng.compute_disparity_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, sp, wp,
                                                   dl.data_ptr(), dr.data_ptr(), fo.data_ptr())
                if use_stream:
                    s.synchronize()
                else:
                    eng.synchronize()
                outs.append([t.cpu().numpy() for t in (dl, dr, fo)])
            finally:
                eng.set_stream(None)
        for a, b in zip(*outs):
            assert np.array_equal(a, b)
    finally:
        eng.close()


@pytest.mark.gpu
def test_compute_disparity_batch_device_npairs_guard():
    """npairs < 0 -> SM_E_ARG before any launch is sized from it; npairs == 0 is a no-op
    that leaves the outputs untouched (the WLS preparation used to launch first)."""
    import torch

    H, W, D = 40, 120, 16
    sp = synthetic.to_sm_params(synthetic.parity_params(D))
    wp = _lib.wls_default_params(sp)
    L = torch.zeros((1, H, W), dtype=torch.uint8, device="cuda")
    outs = [torch.full((1, H, W), 7, dtype=torch.int16, device="cuda") for _ in range(3)]
    eng = _lib.engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        with pytest.raises(ValueError):
            eng.compute_disparity_batch_device(L.data_ptr(), L.data_ptr(), -1, H * W, H, W, W, sp, wp,
                                               *(o.data_ptr() for o in outs))
        eng.compute_disparity_batch_device(L.data_ptr(), L.data_ptr(), 0, H * W, H, W, W, sp, wp,
                                           *(o.data_ptr() for o in outs))
        eng.synchronize()
        assert all(bool((o == 7).all()) for o in outs)
    finally:
        eng.set_stream(None)
