"""The integer WTA index at the boundary (SURVEY §8b ``wta_out``): OpenCV's
``bestDisp`` per pixel, -1 where the uniqueness test (or saturation) rejects it
and outside [minX1, maxX1), before the sub-pixel step, the disp12MaxDiff check
and the median -- the quantity BASELINE.json's north star states its bit-exact
bar on.  Compared with the C oracle's index (``ref_c.compute_wta``, itself
checked against ``sgm_np.wta_index`` in tests/test_oracle_kats.py) at full KITTI
size, for the headline census 8 paths and the reference's MODE_SGBM, through
every engine (fused sweeps, per-direction, OpenCV int16 arithmetic)."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import ref_c
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

PERDIR = 4096  # sm_api.hip DBG_LEGACY: per-direction engine
SWEEP8 = 16384  # force the fused sweeps


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(0)
    yield e
    e.close()


def _oracle(pairs, p):
    with ThreadPoolExecutor(8) as ex:  # ctypes releases the GIL; one pair per thread
        return list(ex.map(lambda lr: ref_c.compute_wta(lr[0], lr[1], p, median=False), pairs))


@pytest.mark.parametrize("mode", ["census8", "sgbm5"])
def test_wta_index_kitti_batch(eng, mode):
    """8 KITTI pairs in one device batch (the bench's launch group: fused sweeps)."""
    import torch

    H, W, D = synthetic.CONFIGS["kitti"]
    p = synthetic.headline_params(D) if mode == "census8" else synthetic.parity_params(D)
    pairs = [synthetic.random_dot_pair(H, W, D, seed=1000 + i)[:2] for i in range(8)]
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    out = torch.empty((8, H, W), dtype=torch.int16, device="cuda")
    wta = torch.full((8, H, W), 7777, dtype=torch.int16, device="cuda")
    eng.compute_wta_batch_device(L.data_ptr(), R.data_ptr(), 8, H * W, H, W, W, synthetic.to_sm_params(p),
                                 out.data_ptr(), wta.data_ptr())
    eng.synchronize()
    raw_gpu = eng.debug_fetch(2)  # pre-median map of the last pair
    ref = _oracle(pairs, p)
    got = wta.cpu().numpy()
    for i, (raw, w) in enumerate(ref):
        assert np.array_equal(got[i], w), f"pair {i}: {int((got[i] != w).sum())} px differ"
    assert np.array_equal(np.frombuffer(raw_gpu, np.int16).reshape(H, W), ref[-1][0])
    # a real distribution: most pixels pass, some are rejected, the border band is -1
    assert 0.5 < (got >= 0).mean() < 1.0
    assert (got[:, :, :D] == -1).all()


@pytest.mark.parametrize("engine_flags", [PERDIR, SWEEP8], ids=["perdir", "sweeps"])
@pytest.mark.parametrize("mode", ["census8", "sgbm5", "census5", "sgbm8"])
def test_wta_index_host_api_engines(eng, engine_flags, mode):
    """sm_compute's wta_out on one pair, each engine forced."""
    H, W, D = 96, 333, 64
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=55)
    cost, paths = {"census8": (1, 8), "sgbm5": (0, 5), "census5": (1, 5), "sgbm8": (0, 8)}[mode]
    p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=paths)
    eng.set_debug_flags(engine_flags)
    try:
        disp, wta = eng.compute_wta(left, right, synthetic.to_sm_params(p))
    finally:
        eng.set_debug_flags(0)
    rdisp, rwta = ref_c.compute_wta(left, right, p)
    assert np.array_equal(disp, rdisp)
    assert np.array_equal(wta, rwta)


def test_wta_index_opencv_int16_path(eng):
    """blockSize 23 / preFilterCap 1 (disparity_test.py:165-177): the sm_wide.hpp path."""
    H, W, D = 64, 200, 16
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=8)
    p = dict(minDisparity=0, numDisparities=16, blockSize=23, P1=222, P2=887, disp12MaxDiff=20, uniquenessRatio=0,
             preFilterCap=1, speckleWindowSize=0, speckleRange=0)
    disp, wta = eng.compute_wta(left, right, synthetic.to_sm_params(p))
    rdisp, rwta = ref_c.compute_wta(left, right, p)
    assert np.array_equal(disp, rdisp)
    assert np.array_equal(wta, rwta)


def test_wta_index_no_domain(eng):
    """numDisparities >= width: no column in [minX1, maxX1), every index -1."""
    left, right, _ = synthetic.random_dot_pair(20, 40, 16, seed=1)
    p = dict(synthetic.parity_params(48))
    disp, wta = eng.compute_wta(left, right, synthetic.to_sm_params(p))
    assert (wta == -1).all()
    assert (disp == -16).all()


def test_wta_index_row_lds_limit(eng):
    """The WTA row kernels keep a row's keys, sub-pixel values and (with the index output)
    the index in LDS: W * 10 + 16 bytes.  Past 64 KB (W > 6551) the call reports
    SM_E_UNSUPPORTED with a message, instead of failing at launch."""
    H, W, D = 2, 6600, 16
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=4)
    p = synthetic.to_sm_params(synthetic.parity_params(D))
    eng.set_debug_flags(PERDIR)
    try:
        with pytest.raises(_lib.SmError, match="LDS"):
            eng.compute_wta(left, right, p)
        disp = eng.compute(left, right, p)  # without the index: W * 8 + 16 bytes still fit
    finally:
        eng.set_debug_flags(0)
    assert np.array_equal(disp, ref_c.compute(left, right, synthetic.parity_params(D)))


def test_abi_version():
    assert _lib.load().sm_abi_version() == _lib.ABI_VERSION == 3
