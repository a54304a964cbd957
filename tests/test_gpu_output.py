"""GPU parity of the output stage: reprojectImageTo3D vs the
numpy restatement (bit-exact float32, NaN/inf positions identical)."""
import numpy as np
import pytest

from oracle import ref_c, reproject_np
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

Q_REF = np.float32([[1, 0, 0, -640], [0, -1, 0, 360], [0, 0, 0, -1164], [0, 0, 1, 0]])  # disparity_calculation.py:295


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("handle_missing", [False, True])
def test_reproject_int16_filtered_map(handle_missing):
    import stereo_match_amd as sm

    H, W, D = 120, 300, 64
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=2)
    disp = ref_c.compute(left, right, synthetic.parity_params(D))
    got = sm.reprojectImageTo3D(disp, Q_REF, handleMissingValues=handle_missing, ddepth=5)
    assert got.dtype == np.float32 and got.shape == (H, W, 3)
    assert _same(got, reproject_np.reproject_image_to_3d(disp, Q_REF, handle_missing))


def test_reproject_float_and_project_points_3d():
    import stereo_match_amd as sm

    rng = np.random.default_rng(5)
    Q = rng.standard_normal((4, 4))
    d = (rng.random((57, 83)) * 100).astype(np.float32)
    assert _same(sm.reprojectImageTo3D(d, Q), reproject_np.reproject_image_to_3d(d, Q))
    d16 = (rng.integers(-16, 2000, (40, 60))).astype(np.int16)
    exp = reproject_np.reproject_image_to_3d(d16.astype(np.float32) / np.float32(16), Q_REF.astype(np.float32))
    assert _same(sm.project_points_3D(d16, Q_REF), exp)


def test_reproject_torch_batch_device():
    import torch

    H, W = 64, 96
    rng = np.random.default_rng(9)
    maps = rng.integers(-16, 1500, (3, H, W)).astype(np.int16)
    t = torch.tensor(maps, device="cuda")
    out = torch.empty((3, H, W, 3), dtype=torch.float32, device="cuda")
    eng = _lib.engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.reproject_device(t.data_ptr(), 0, 3, H, W, Q_REF, True, out.data_ptr())
    got = out.cpu().numpy()
    for i in range(3):
        assert _same(got[i], reproject_np.reproject_image_to_3d(maps[i], Q_REF, True)), i
