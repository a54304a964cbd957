"""GPU parity of StereoBM (method="BM") against oracle/bm_np.py:
bit-exact int16 (integer SAD, texture, uniqueness, sub-pixel, validate,
speckles).  Parity with OpenCV itself is unpinned."""
import numpy as np
import pytest

from oracle import bm_np, wls_np
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(0)
    yield e
    e.close()


def bm_params(p: dict) -> _lib.SmBmParams:
    q = bm_np.normalize_bm(p)
    return _lib.SmBmParams(q["minDisparity"], q["numDisparities"], q["blockSize"], q["preFilterType"],
                           q["preFilterSize"], q["preFilterCap"], q["textureThreshold"], q["uniquenessRatio"],
                           q["speckleWindowSize"], q["speckleRange"], q["disp12MaxDiff"])


_rng = np.random.default_rng(4321)
_CASES = [dict(H=int(_rng.integers(12, 90)), W=int(_rng.integers(70, 300)), D=16 * int(_rng.integers(1, 5)),
               bs=int(_rng.choice([5, 7, 9, 15, 21])), minD=int(_rng.integers(-6, 6)),
               uniq=int(_rng.choice([0, 5, 15])), tex=int(_rng.choice([0, 10, 200])),
               d12=int(_rng.choice([-1, 1, 4])), cap=int(_rng.choice([15, 31, 63])),
               sws=int(_rng.choice([0, 0, 30])), seed=int(_rng.integers(0, 1 << 30))) for _ in range(14)]


@pytest.mark.parametrize("c", _CASES, ids=lambda c: "H{H}W{W}D{D}bs{bs}m{minD}u{uniq}t{tex}v{d12}".format(**c))
def test_bm_random_vs_oracle(eng, c):
    left, right, _ = synthetic.random_dot_pair(c["H"], c["W"], c["D"], seed=c["seed"])
    if c["bs"] >= min(c["H"], c["W"]):
        pytest.skip("window larger than the image")
    p = dict(numDisparities=c["D"], blockSize=c["bs"], minDisparity=c["minD"], uniquenessRatio=c["uniq"],
             textureThreshold=c["tex"], disp12MaxDiff=c["d12"], preFilterCap=c["cap"],
             speckleWindowSize=c["sws"], speckleRange=16)
    out = eng.bm_compute(left, right, bm_params(p))
    exp = bm_np.stereo_bm(left, right, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


@pytest.mark.parametrize("D,bs", [(128, 21), (256, 41), (64, 5)])
def test_bm_full_size_kitti(eng, D, bs):
    H, W, _ = synthetic.CONFIGS["kitti"]
    left, right, gt = synthetic.random_dot_pair(H, W, D, seed=12)
    p = dict(numDisparities=D, blockSize=bs)
    out = eng.bm_compute(left, right, bm_params(p))
    assert np.array_equal(out, bm_np.stereo_bm(left, right, p))
    rp = bm_np.right_matcher_params(p)
    assert np.array_equal(eng.bm_compute(right, left, bm_params(rp)), bm_np.stereo_bm(right, left, rp))


def test_compute_disparity_bm_end_to_end():
    """method="BM": left BM (WLS-mutated), right BM, WLS with BM offsets."""
    import stereo_match_amd as sm

    H, W, D = 100, 320, 64
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=21)
    s = dict(sm.DEFAULT_SETTINGS, num_disparities=D, block_size=15, lmbda=80000, sigma=1.2)
    displ, filt = sm.compute_disparity(left, right, s, method="BM")
    lp = dict(numDisparities=D, blockSize=15, textureThreshold=0, uniquenessRatio=0, disp12MaxDiff=1000000)
    rp = bm_np.right_matcher_params(dict(numDisparities=D, blockSize=15))
    exp_l = bm_np.stereo_bm(left, right, lp)
    exp_r = bm_np.stereo_bm(right, left, rp)
    assert np.array_equal(displ, exp_l)
    wp = dict(lmbda=80000.0, sigma=1.2, radius=5, min_disp=0, left_offset=D + 7, right_offset=7, top_offset=7,
              bottom_offset=7)
    assert np.array_equal(filt, wls_np.wls_filter(exp_l, left, exp_r, wp))


def test_bm_torch_batch_and_errors(eng):
    import torch

    import stereo_match_amd as sm

    H, W, D, n = 60, 200, 32, 3
    pairs = [synthetic.random_dot_pair(H, W, D, seed=70 + i)[:2] for i in range(n)]
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    out = torch.empty((n, H, W), dtype=torch.int16, device="cuda")
    p = dict(numDisparities=D, blockSize=9)
    e = _lib.engine(0)
    e.set_stream(torch.cuda.current_stream().cuda_stream)
    e.bm_compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, bm_params(p), out.data_ptr())
    got = out.cpu().numpy()
    for i, (a, b) in enumerate(pairs):
        assert np.array_equal(got[i], bm_np.stereo_bm(a, b, p)), i
    m = sm.StereoBM_create(numDisparities=D, blockSize=9)
    assert np.array_equal(m.compute(L[0], R[0]).cpu().numpy(), got[0])
    for bad in (dict(blockSize=4), dict(numDisparities=40), dict(preFilterCap=0)):
        with pytest.raises(ValueError):
            eng.bm_compute(pairs[0][0], pairs[0][1], bm_params(dict(p, **bad)))
    with pytest.raises(_lib.SmError):
        eng.bm_compute(pairs[0][0], pairs[0][1], bm_params(dict(p, preFilterType=0)))


from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(H=st.integers(6, 50), W=st.integers(10, 160), Dk=st.integers(1, 4), minD=st.integers(-20, 20),
       bs=st.sampled_from([5, 7, 9, 11, 15, 21]), cap=st.integers(1, 63), tex=st.integers(0, 300),
       uniq=st.integers(0, 40), d12=st.integers(-1, 5), sws=st.sampled_from([0, 0, 10]), srange=st.integers(0, 32),
       seed=st.integers(0, 2**31 - 1))
def test_hypothesis_bm_vs_oracle(eng, H, W, Dk, minD, bs, cap, tex, uniq, d12, sws, srange, seed):
    D = 16 * Dk
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=seed)
    p = dict(numDisparities=D, blockSize=bs, minDisparity=minD, preFilterCap=cap, textureThreshold=tex,
             uniquenessRatio=uniq, disp12MaxDiff=d12, speckleWindowSize=sws, speckleRange=srange)
    if bs >= min(H, W):
        with pytest.raises(ValueError):
            eng.bm_compute(left, right, bm_params(p))
        return
    assert np.array_equal(eng.bm_compute(left, right, bm_params(p)), bm_np.stereo_bm(left, right, p))
