"""Round 4 GPU parity: the latency sweep strips (kLatNcw compute waves, single-set halos),
the E/W line widths of the sweep engine (sm_set_tuning SM_TUNE_EW_LANES) and the tuning
API's argument checks.  Every case is bit-exact against the C oracle (oracle/sgm_ref.c)."""
import numpy as np
import pytest

from oracle import ref_c
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

SWEEP8 = 16384  # sm_api.hip DBG_SWEEP8: the fused sweeps at any pair count
LAT_NCW = 5     # sm_sweep.hpp kLatNcw


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(0)
    yield e
    e.close()


def _params(cost, D, mode, minD=0, bs=5):
    if cost:
        return dict(synthetic.headline_params(D), minDisparity=minD, mode=mode)
    return dict(synthetic.parity_params(D), minDisparity=minD, mode=mode, blockSize=bs, P1=8 * bs * bs,
                P2=32 * bs * bs)


def _run(eng, left, right, p, flags=SWEEP8, **tune):
    eng.set_debug_flags(flags)
    for k, v in tune.items():
        eng.set_tuning(getattr(eng, "TUNE_" + k.upper()), v)
    try:
        return eng.compute(left, right, synthetic.to_sm_params(p))
    finally:
        eng.set_debug_flags(0)
        for k in tune:
            eng.set_tuning(getattr(eng, "TUNE_" + k.upper()), 0)


_rng = np.random.default_rng(404)
LAT_CASES = []
for _ in range(16):
    D = int(_rng.choice([64, 96, 128, 160, 192, 224]))
    H = int(_rng.integers(1, 40))
    W = int(_rng.integers(D + 1, D + 260))
    LAT_CASES.append(dict(H=H, W=W, D=D, minD=int(_rng.choice([0, 0, 4, -7])), cost=int(_rng.integers(0, 2)),
                          mode=int(_rng.choice([5, 8])), seed=int(_rng.integers(0, 1 << 30))))


@pytest.mark.parametrize("c", LAT_CASES, ids=lambda c: "H{H}W{W}D{D}m{minD}c{cost}p{mode}".format(**c))
def test_latency_strips_random_shapes(eng, c):
    """Latency strips (3 own waves, 4-column halos handed off every 4 rows) forced on random
    shapes: ragged strips, one to dozens of strips, both cost types and sweep modes."""
    left, right, _ = synthetic.random_dot_pair(c["H"], c["W"], c["D"], seed=c["seed"])
    p = _params(c["cost"], c["D"], c["mode"], c["minD"])
    out = _run(eng, left, right, p, sweep_ncw=LAT_NCW)
    exp = ref_c.compute(left, right, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


@pytest.mark.parametrize("cost,mode,D", [(0, 5, 160), (1, 8, 128), (0, 8, 128)])
def test_latency_strips_full_kitti(eng, cost, mode, D):
    """Full KITTI frame on the latency strips (settings.ini D = 160 MODE_SGBM; census 8 paths)."""
    H, W, _ = synthetic.CONFIGS["kitti"]
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=D + mode)
    p = _params(cost, D, mode)
    out = _run(eng, left, right, p, sweep_ncw=LAT_NCW)
    exp = ref_c.compute(left, right, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


@pytest.mark.parametrize("lanes", [-1, 8, 16, 32, 64])
@pytest.mark.parametrize("cost,mode,D", [(0, 5, 128), (0, 8, 128), (0, 5, 160), (1, 8, 128), (0, 5, 64), (1, 8, 96)])
def test_ew_lanes_bit_exact(eng, lanes, cost, mode, D):
    """Every E/W line width built for D gives the oracle's maps (row lines -1; packed lines
    of 8, 16, 32 or 64 lanes); unbuilt widths are refused, not silently replaced."""
    left, right, _ = synthetic.random_dot_pair(61, 2 * D + 150, D, seed=lanes * 7 + D)
    p = _params(cost, D, mode)
    built = (lanes in (-1, 8) or (lanes == 16 and D % 32 == 0) or (lanes == 32 and D % 64 == 0)
             or (lanes == 64 and D in (128, 256)))
    if not built:
        with pytest.raises(_lib.SmError):
            _run(eng, left, right, p, ew_lanes=lanes)
        return
    out = _run(eng, left, right, p, ew_lanes=lanes)
    exp = ref_c.compute(left, right, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


def test_sgbm5_batch_default_ew_lanes(eng):
    """A KITTI batch of 4 sgbm5 pairs (sweep engine by default: packed 32-lane E/W lines at
    D = 128) against the oracle pair by pair."""
    import torch

    H, W, D = synthetic.CONFIGS["kitti"]
    ls, rs = [], []
    for i in range(4):
        left, right, _ = synthetic.random_dot_pair(H, W, D, seed=900 + i)
        ls.append(left)
        rs.append(right)
    dl = torch.from_numpy(np.stack(ls)).cuda()
    dr = torch.from_numpy(np.stack(rs)).cuda()
    out = torch.empty((4, H, W), dtype=torch.int16, device="cuda")
    p = synthetic.parity_params(D)
    eng.compute_batch_device(dl.data_ptr(), dr.data_ptr(), 4, H * W, H, W, W, synthetic.to_sm_params(p),
                             out.data_ptr())
    eng.synchronize()
    got = out.cpu().numpy()
    for i in range(4):
        exp = ref_c.compute(ls[i], rs[i], p)
        assert np.array_equal(got[i], exp), f"pair {i}: {np.sum(got[i] != exp)} px differ"


def test_tuning_arguments(eng):
    """Unknown keys and out-of-range values are SM_E_ARG (ValueError); an unbuilt strip width
    fails the call (SM_E_UNSUPPORTED) instead of running another one."""
    with pytest.raises(ValueError):
        eng.set_tuning(99, 0)
    with pytest.raises(ValueError):
        eng.set_tuning(eng.TUNE_EW_LANES, 12)
    with pytest.raises(ValueError):
        eng.set_tuning(eng.TUNE_SWEEP_NCW, -1)
    left, right, _ = synthetic.random_dot_pair(20, 200, 64, seed=3)
    with pytest.raises(_lib.SmError):
        _run(eng, left, right, _params(1, 64, 8), sweep_ncw=3)
