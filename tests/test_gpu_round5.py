"""Round 5 GPU parity: the horizontal paths inside the fused down sweep (MODE 3 line waves,
speculative strip segments) and the patch pass that repairs segments whose guessed start
state was wrong.  Every case is bit-exact against the C oracle
(oracle/sgm_ref.c); the adversarial cases force repairs (a 1-column warmup, textureless
bands, smooth costs, tiny D, one-strip images) and check the repair counter moved."""
import numpy as np
import pytest

from oracle import ref_c
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

SWEEP8 = 16384  # sm_api.hip DBG_SWEEP8: the fused sweeps at any pair count


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


def _check(out, left, right, p):
    exp = ref_c.compute(left, right, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


_rng = np.random.default_rng(505)
CASES = []
for _ in range(30):
    D = int(_rng.choice([16, 32, 48, 64, 96, 128, 160, 192, 256]))
    H = int(_rng.integers(1, 48))
    W = int(_rng.integers(D + 1, D + 320)) if _rng.random() < 0.85 else int(_rng.integers(1, D + 3))
    CASES.append(dict(H=H, W=W, D=D, minD=int(_rng.choice([0, 0, 0, 5, -9, -D + 1])), cost=int(_rng.integers(0, 2)),
                      mode=int(_rng.choice([5, 8])), warm=int(_rng.choice([0, 0, 1, 2, 5])),
                      guess=int(_rng.integers(0, 2)), seed=int(_rng.integers(0, 1 << 30))))


@pytest.mark.parametrize("c", CASES, ids=lambda c: "H{H}W{W}D{D}m{minD}c{cost}p{mode}w{warm}g{guess}".format(**c))
def test_lines_random_shapes(eng, c):
    """The in-sweep lines on random shapes: ragged last strips, single-strip images, both cost
    types and path counts, default and short warmups, zero and wrong start guesses."""
    left, right, _ = synthetic.random_dot_pair(c["H"], c["W"], c["D"], seed=c["seed"])
    p = _params(c["cost"], c["D"], c["mode"], c["minD"])
    out = _run(eng, left, right, p, ew_warmup=c["warm"], ew_guess=c["guess"])
    _check(out, left, right, p)


@pytest.mark.parametrize("cost,mode,D", [(1, 8, 128), (0, 5, 128), (0, 8, 128), (0, 5, 160), (1, 5, 64)])
@pytest.mark.parametrize("warm,guess", [(0, 0), (1, 0), (1, 1)])
def test_lines_full_kitti(eng, cost, mode, D, warm, guess):
    """Full KITTI frames: default warmup, the shortest warmup, and a deliberately wrong start
    state (SM_TUNE_EW_GUESS: every segment that does not meet the truth inside its warmup is
    repaired; with the shortest warmup, so that they are): bit-exact, and the repair counter
    counts the repairs.  (One pair of 5 paths runs on the row bands, whose default u16 warmup
    is long enough for even a wrong guess to meet the truth.)"""
    H, W, _ = synthetic.CONFIGS["kitti"]
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=D + mode + cost)
    p = _params(cost, D, mode)
    c0 = eng.counters()
    out = _run(eng, left, right, p, ew_warmup=warm, ew_guess=guess)
    _check(out, left, right, p)
    c1 = eng.counters()
    assert c1["line_groups"] > c0["line_groups"], "the wide MODE 3 instance ran"
    if guess:
        assert c1["ew_repairs"] > c0["ew_repairs"]


def _bands(H, W, period=40, seed=0):
    """Textureless vertical bands alternating with random texture: states cannot meet inside
    a flat band, so the segments that start there are repaired across it."""
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (H, W)).astype(np.uint8)
    flat = (np.arange(W) // period) % 2 == 0
    img[:, flat] = 90
    return img


ADV = [
    ("const", lambda H, W: (np.full((H, W), 77, np.uint8), np.full((H, W), 77, np.uint8))),
    ("const_lr_differ", lambda H, W: (np.full((H, W), 40, np.uint8), np.full((H, W), 200, np.uint8))),
    ("bands", lambda H, W: (_bands(H, W, 40, 1), np.roll(_bands(H, W, 40, 1), -7, axis=1))),
    ("wide_bands", lambda H, W: (_bands(H, W, 150, 2), np.roll(_bands(H, W, 150, 2), -3, axis=1))),
    ("hgradient", lambda H, W: (np.tile(np.arange(W, dtype=np.int64) % 256, (H, 1)).astype(np.uint8),
                                np.tile((np.arange(W, dtype=np.int64) + 5) % 256, (H, 1)).astype(np.uint8))),
    ("noise_lr_indep", lambda H, W: (np.random.default_rng(3).integers(0, 256, (H, W)).astype(np.uint8),
                                     np.random.default_rng(4).integers(0, 256, (H, W)).astype(np.uint8))),
]


@pytest.mark.parametrize("name,make", ADV, ids=[a[0] for a in ADV])
@pytest.mark.parametrize("cost,mode,D,P1,P2", [(1, 8, 64, 10, 120), (1, 8, 32, 60, 61), (0, 5, 64, 200, 201),
                                               (0, 8, 16, 8, 32), (1, 5, 128, 1, 193)])
@pytest.mark.parametrize("guess", [0, 1])
def test_lines_adversarial(eng, name, make, cost, mode, D, P1, P2, guess):
    """Inputs chosen against the speculation: flat images, flat bands, smooth horizontal
    gradients, uncorrelated noise; P2 = P1 + 1 (the smallest P2 the matcher keeps) and a
    large P2; tiny D; zero and wrong start guesses."""
    H, W = 23, 3 * D + 257
    left, right = make(H, W)
    p = dict(_params(cost, D, mode), P1=P1, P2=P2)
    out = _run(eng, left, right, p, ew_guess=guess)
    _check(out, left, right, p)


@pytest.mark.parametrize("name", ["const", "wide_bands"])
def test_lines_open_strips_carry_the_true_state(eng, name):
    """Flat images and flat bands wider than a strip with a wrong start guess: the repaired
    values of a segment never meet the speculative ones inside its strip (SM_COUNTER_EW_OPEN),
    so the patch pass carries the true state into the next strips (its phase B) — over a full
    KITTI row of strips, both cost types."""
    make = dict(ADV)[name]
    H, W, D = 12, synthetic.CONFIGS["kitti"][1], 128
    left, right = make(H, W)
    for cost, mode in ((1, 8), (0, 5)):
        p = dict(_params(cost, D, mode), P1=10, P2=120)
        c0 = eng.counters()
        out = _run(eng, left, right, p, ew_guess=1)
        _check(out, left, right, p)
        c1 = eng.counters()
        assert c1["ew_open"] > c0["ew_open"], (name, cost, c1)
        assert c1["ew_repairs"] - c0["ew_repairs"] >= c1["ew_open"] - c0["ew_open"]


def test_lines_match_classic_engine_kitti_batch(eng):
    """8 KITTI census pairs through one launch group: the in-sweep lines and the E/W volume
    kernel (SM_TUNE_SWEEP_LINES -1) give identical maps, and every pair equals the oracle."""
    import torch

    H, W, D = synthetic.CONFIGS["kitti"]
    ls, rs = [], []
    for i in range(8):
        left, right, _ = synthetic.random_dot_pair(H, W, D, seed=5000 + i)
        ls.append(left)
        rs.append(right)
    dl = torch.from_numpy(np.stack(ls)).cuda()
    dr = torch.from_numpy(np.stack(rs)).cuda()
    p = synthetic.headline_params(D)
    outs = []
    for lines in (0, -1):
        out = torch.empty((8, H, W), dtype=torch.int16, device="cuda")
        eng.set_tuning(eng.TUNE_SWEEP_LINES, lines)
        try:
            eng.compute_batch_device(dl.data_ptr(), dr.data_ptr(), 8, H * W, H, W, W, synthetic.to_sm_params(p),
                                     out.data_ptr())
            eng.synchronize()
        finally:
            eng.set_tuning(eng.TUNE_SWEEP_LINES, 0)
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    # every pair against the oracle (not only pairs 0 and 5)
    exp = ref_c.compute_many(list(zip(ls, rs)), p)
    for i in range(8):
        assert np.array_equal(outs[0][i], exp[i]), f"pair {i}: {np.sum(outs[0][i] != exp[i])} px differ"


@pytest.mark.parametrize("D,warm", [(192, 0), (192, 2), (64, 0)])
def test_lines_cost_volume(eng, D, warm):
    """mc-cnn style f32 volumes (u16 costs, 8 paths) through the in-sweep lines."""
    H, W = 40, D + 300
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=D + warm)
    vol = synthetic.absdiff_volume(left, right, D)
    p = synthetic.cost_volume_params(D)
    eng.set_debug_flags(SWEEP8)
    eng.set_tuning(eng.TUNE_EW_WARMUP, warm)
    try:
        out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.0, synthetic.VOLUME_SCALE)
    finally:
        eng.set_debug_flags(0)
        eng.set_tuning(eng.TUNE_EW_WARMUP, 0)
    exp = ref_c.compute_volume(vol[0], p, 0.0, synthetic.VOLUME_SCALE)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


def test_lines_tuning_arguments(eng):
    with pytest.raises(ValueError):
        eng.set_tuning(eng.TUNE_EW_WARMUP, -1)
    with pytest.raises(ValueError):
        eng.set_tuning(eng.TUNE_SWEEP_LINES, 2)
    with pytest.raises(ValueError):
        eng.set_tuning(eng.TUNE_EW_GUESS, 2)
    c = eng.counters()
    assert set(c) == {"sweep_fallbacks", "ew_repairs", "volume_clamped", "volume_nan", "line_groups", "ew_open",
                      "band_repairs", "band_open", "band_groups", "line_strips"}


# ------------------------------------------------------------------ mc-cnn quantisation window
def _signed_volume(H, W, D, seed):
    """An mc-cnn-like volume whose range nothing pins: negative costs, costs far above 1,
    NaN where x - d leaves the right image (synthetic.absdiff_volume) and a few inf."""
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=seed)
    v = synthetic.absdiff_volume(left, right, D)[0]
    rng = np.random.default_rng(seed)
    v = (v * np.float32(7.0) - np.float32(2.5)).astype(np.float32)  # roughly [-2.5, 4.5]
    v[:, :, -5:] = np.float32(np.inf)
    v.flat[rng.integers(0, v.size, 50)] = np.float32(-np.inf)
    v[:, 3, D + 3] = np.float32(np.nan)  # inside the matcher's columns (absdiff's NaNs are left of them)
    return v


@pytest.mark.parametrize("D,mode", [(64, 8), (48, 5), (37, 8)])
def test_volume_automatic_window(eng, D, mode):
    """scale None / 0: the device derives offset = -min, scale = 4095 / (max - min) over the
    finite quantised cells; the maps equal the C oracle run with the same window
    (oracle/sgm_np.volume_window), no finite cost is clamped, NaN cells are counted."""
    from oracle import sgm_np

    H, W = 31, D + 170
    vol = _signed_volume(H, W, D, seed=D)
    p = dict(synthetic.cost_volume_params(D), mode=mode)
    prm = sgm_np.normalize_params(dict(p, cost=2))
    off, sc = sgm_np.volume_window(vol, prm)
    assert sc != 1.0 and off > 0  # a real window: the volume has negative costs
    clamped_exp, nan_exp = sgm_np.quantize_counts(vol, prm, off, sc)
    before = eng.counters()
    out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), scale="auto")  # opt-in automatic window
    after = eng.counters()
    exp = ref_c.compute_volume(vol, p, off, sc)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"
    # only the infinities leave the window
    assert after["volume_clamped"] - before["volume_clamped"] == clamped_exp
    assert clamped_exp == int(np.sum(np.isinf(vol[:, :, prm["minD"] + D:])))
    assert after["volume_nan"] - before["volume_nan"] == nan_exp > 0


def test_volume_nan_scale_at_the_c_abi_derives_the_window(eng):
    """a NaN scale at the C-ABI takes the automatic window (as the header says), not
    a NaN quantisation; the Python surface refuses NaN outright."""
    import ctypes

    from oracle import sgm_np

    D, H, W = 32, 23, 160
    vol = _signed_volume(H, W, D, seed=11)
    p = synthetic.cost_volume_params(D)
    prm = sgm_np.normalize_params(dict(p, cost=2))
    off, sc = sgm_np.volume_window(vol, prm)
    v = np.ascontiguousarray(vol, np.float32)
    out = np.empty((H, W), np.int16)
    rc = eng._lib.sm_aggregate_cost_f32(eng.ctx, v.ctypes.data, D, H, W, ctypes.byref(synthetic.to_sm_params(p)),
                                        0.0, float("nan"), out.ctypes.data)
    assert rc == 0
    assert np.array_equal(out, ref_c.compute_volume(vol, p, off, sc))
    with pytest.raises(ValueError):
        eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.0, float("nan"))


def test_volume_default_window_is_explicit(eng):
    """omitting scale keeps the explicit window (offset 0, scale 1), the round-4
    default; the automatic window is opt-in."""
    D, H, W = 32, 21, 150
    vol = (_signed_volume(H, W, D, seed=12) * np.float32(300)).astype(np.float32)
    p = synthetic.cost_volume_params(D)
    out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p))
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, 1.0))


def test_volume_explicit_window_counts_clamped_cells(eng):
    """The documented fixed window (offset 0, scale 4000) on a volume with negative and large
    costs: bit-exact against the oracle with that window, and every clamped cell counted."""
    from oracle import sgm_np

    D, H, W = 32, 27, 200
    vol = _signed_volume(H, W, D, seed=7)
    p = synthetic.cost_volume_params(D)
    prm = sgm_np.normalize_params(dict(p, cost=2))
    clamped_exp, nan_exp = sgm_np.quantize_counts(vol, prm, 0.0, 4000.0)
    assert clamped_exp > 1000  # the fixed window flattens a large part of this volume
    before = eng.counters()
    out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.0, 4000.0)
    after = eng.counters()
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, 4000.0))
    assert after["volume_clamped"] - before["volume_clamped"] == clamped_exp
    assert after["volume_nan"] - before["volume_nan"] == nan_exp


def test_volume_automatic_window_device_batch(eng):
    """Per-pair windows in one device batch (each pair its own range)."""
    import torch

    from oracle import sgm_np

    D, H, W, n = 32, 20, 150, 3
    vols = [(_signed_volume(H, W, D, seed=40 + i) * np.float32(1 + 3 * i)).astype(np.float32) for i in range(n)]
    p = synthetic.cost_volume_params(D)
    prm = sgm_np.normalize_params(dict(p, cost=2))
    V = torch.tensor(np.stack(vols), device="cuda")
    out = torch.empty((n, H, W), dtype=torch.int16, device="cuda")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.aggregate_cost_f32_device(V.data_ptr(), n, D * H * W, D, H, W, synthetic.to_sm_params(p), 0.0, 0.0,
                                      out.data_ptr())
        eng.synchronize()
    finally:
        eng.set_stream(None)
    got = out.cpu().numpy()
    for i in range(n):
        off, sc = sgm_np.volume_window(vols[i], prm)
        assert np.array_equal(got[i], ref_c.compute_volume(vols[i], p, off, sc)), i
