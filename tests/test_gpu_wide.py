"""GPU: OpenCV-SGBM outside the int16-exact range and on BGR input
(sm_wide.hpp) against the C oracle's x86 int16 arithmetic
(oracle/sgm_ref.c header): the reference's direct-matcher configurations
disparity_test.py:165-177 and try_try.py:69-77, the K8 box-sum wrap /
saturation, and random wide configurations."""
import numpy as np
import pytest

from oracle import ref_c
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

# /root/reference/disparity_test.py:165-177
DISPARITY_TEST = dict(minDisparity=0, numDisparities=16, blockSize=23, P1=222, P2=887, disp12MaxDiff=20,
                      uniquenessRatio=0, speckleWindowSize=0, speckleRange=0, preFilterCap=1, mode=5, cost=0)
# /root/reference/try_try.py:66-77 (window_size 3, min_disp 16, num_disp 112 - 16), BGR input (:56-57)
TRY_TRY = dict(minDisparity=16, numDisparities=96, blockSize=16, P1=8 * 3 * 9, P2=32 * 3 * 9, disp12MaxDiff=1,
               uniquenessRatio=10, speckleWindowSize=100, speckleRange=32, preFilterCap=0, mode=5, cost=0)


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(0)
    yield e
    e.close()


def _bgr(gray, seed):
    """A BGR pair built from a gray one: channels differ (shifted / inverted copies)."""
    rng = np.random.default_rng(seed)
    noise = rng.integers(0, 20, gray.shape, dtype=np.uint8)
    return np.ascontiguousarray(np.stack([gray, np.roll(gray, 1, 0) // 2 + noise, 255 - gray], -1))


def _run(eng, left, right, p):
    return eng.compute(left, right, synthetic.to_sm_params(p))


@pytest.mark.parametrize("H,W", [(48, 120), (120, 330), (375, 1242)])
def test_disparity_test_params_gray(eng, H, W):
    left, right, _ = synthetic.random_dot_pair(H, W, 16, seed=H)
    out = _run(eng, left, right, DISPARITY_TEST)
    assert np.array_equal(out, ref_c.compute(left, right, DISPARITY_TEST))
    C = np.frombuffer(eng.debug_fetch(0), np.int16).reshape(ref_c.cost_volume(left, right, DISPARITY_TEST).shape)
    assert np.array_equal(C, ref_c.cost_volume(left, right, DISPARITY_TEST))


def test_k8_box_sum_wrap_and_saturation_on_gpu(eng):
    l = np.zeros((40, 80), np.uint8)
    r = np.full((40, 80), 255, np.uint8)
    out = _run(eng, l, r, DISPARITY_TEST)
    assert np.array_equal(out, ref_c.compute(l, r, DISPARITY_TEST))
    C = np.frombuffer(eng.debug_fetch(0), np.int16).reshape(40, 64, 16)
    assert (C[0, 12:51] == -31322).all() and (C[1:, 12:51] == -31319).all()


@pytest.mark.parametrize("H,W", [(60, 200), (192, 320)])
def test_try_try_params_bgr(eng, H, W):
    gl, gr, _ = synthetic.random_dot_pair(H, W, 96, seed=W)
    left, right = _bgr(gl, 1), _bgr(gr, 1)
    out = _run(eng, left, right, TRY_TRY)
    assert np.array_equal(out, ref_c.compute(left, right, TRY_TRY))
    # the cv2-style shim takes the BGR arrays too
    import stereo_match_amd as sm

    m = sm.StereoSGBM_create(minDisparity=16, numDisparities=96, blockSize=16, P1=216, P2=864, disp12MaxDiff=1,
                             uniquenessRatio=10, speckleWindowSize=100, speckleRange=32)
    assert np.array_equal(m.compute(left, right), out)


_rng = np.random.default_rng(77)
WIDE = []
for _i in range(24):
    D = int(_rng.choice([16, 32, 48, 64, 112]))
    bs = int(_rng.choice([3, 5, 12, 13, 16, 19, 23, 31]))
    WIDE.append(dict(H=int(_rng.integers(bs // 2 + 2, 70)), W=int(_rng.integers(D + bs, D + 220)), D=D, bs=bs,
                     cn=int(_rng.choice([1, 3])), mode=int(_rng.choice([5, 8])),
                     minD=int(_rng.choice([0, 0, 7, -11])), pfc=int(_rng.choice([1, 31, 63, 100])),
                     P1=int(_rng.integers(1, 400)), P2x=int(_rng.choice([2, 4, 40])),
                     uniq=int(_rng.choice([0, 5, 15])), d12=int(_rng.choice([1, 3, 1000000])),
                     seed=int(_rng.integers(0, 1 << 30))))


@pytest.mark.parametrize("c", WIDE, ids=lambda c: "H{H}W{W}D{D}bs{bs}cn{cn}p{mode}".format(**c))
def test_random_wide_configs(eng, c):
    gl, gr, _ = synthetic.random_dot_pair(c["H"], c["W"], c["D"], seed=c["seed"])
    left, right = (gl, gr) if c["cn"] == 1 else (_bgr(gl, c["seed"]), _bgr(gr, c["seed"]))
    p = dict(minDisparity=c["minD"], numDisparities=c["D"], blockSize=c["bs"], P1=c["P1"],
             P2=min(c["P1"] * c["P2x"], 32767), disp12MaxDiff=c["d12"], uniquenessRatio=c["uniq"],
             preFilterCap=c["pfc"], mode=c["mode"], cost=0)
    out = _run(eng, left, right, p)
    exp = ref_c.compute(left, right, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


def test_wide_batch_device_bgr(eng):
    import torch

    H, W, n = 50, 180, 3
    pairs = []
    for s in range(n):
        a, b, _ = synthetic.random_dot_pair(H, W, 32, seed=400 + s)
        pairs.append((_bgr(a, s), _bgr(b, s)))
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    out = torch.empty((n, H, W), dtype=torch.int16, device="cuda")
    p = dict(synthetic.parity_params(32), blockSize=7)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W * 3, H, W, W * 3, synthetic.to_sm_params(p),
                                 out.data_ptr(), channels=3)
        got = out.cpu().numpy()
    finally:
        eng.set_stream(None)
    for i, (a, b) in enumerate(pairs):
        assert np.array_equal(got[i], ref_c.compute(a, b, p)), i


def test_box_sums_past_int16_saturate_like_opencv(eng):
    """blockSize 55, BGR, preFilterCap 126: a 55-wide window of 3-channel BT costs
    (up to 3 * (2*127 + 63) each) passes 32767, where OpenCV's running int16 sums
    saturate (rows entering during the scan) or wrap (the rows of the first C row);
    k_wide_hsum_scan reproduces both (sm_wide.hpp hsum)."""
    rng = np.random.default_rng(5)
    H, W, D = 70, 200, 16
    gl = rng.integers(0, 256, (H, W), dtype=np.uint8)
    gr = (255 - gl).astype(np.uint8)
    left, right = _bgr(gl, 3), _bgr(gr, 4)
    p = dict(minDisparity=0, numDisparities=D, blockSize=55, P1=100, P2=800, disp12MaxDiff=1000000,
             uniquenessRatio=0, preFilterCap=126, mode=5, cost=0)
    out = _run(eng, left, right, p)
    C_ref = ref_c.cost_volume(left, right, p)
    assert (C_ref == 32767).any() and (C_ref < 0).any()  # both the saturation and the wrap happen
    C = np.frombuffer(eng.debug_fetch(0), np.int16).reshape(C_ref.shape)
    assert np.array_equal(C, C_ref), f"{int((C != C_ref).sum())} cost cells differ"
    assert np.array_equal(out, ref_c.compute(left, right, p))
