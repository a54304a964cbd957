"""Round 6 GPU parity: row bands of the 5-path lines engine.  At one or two
pairs per launch group the MODE 3 down sweep splits each pair's rows into bands that start
`vwarm` rows above their own rows from the zero state (a speculation); k_band_patch checks
every column's S / SE / SW state entering each band against the band above's end state and
repairs the chains where they differ, carrying unmet chains into the next boundary.  Every case
is bit-exact against the C oracle (oracle/sgm_ref.c); adversarial inputs and a deliberately
wrong entering state (SM_TUNE_BAND_GUESS) force repairs and carries, which the counters show."""
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


def _params(cost, D, mode=5, minD=0, bs=5):
    if cost:
        return dict(synthetic.headline_params(D), minDisparity=minD, mode=mode)
    return dict(synthetic.parity_params(D), minDisparity=minD, mode=mode, blockSize=bs, P1=8 * bs * bs,
                P2=32 * bs * bs)


def _run(eng, left, right, p, flags=0, **tune):
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


_rng = np.random.default_rng(606)
CASES = []
for _ in range(28):
    cost = int(_rng.integers(0, 2))
    D = int(_rng.choice([32, 64, 96, 128, 160, 192] if cost else [32, 96, 128, 160]))
    CASES.append(dict(H=int(_rng.integers(20, 160)), W=int(_rng.integers(D + 40, D + 420)), D=D, cost=cost,
                      minD=int(_rng.choice([0, 0, 3, -7])), bands=int(_rng.choice([2, 3, 5, 8])),
                      vwarm=int(_rng.choice([0, 0, 1, 3, 9])), guess=int(_rng.choice([0, 0, 1])),
                      seed=int(_rng.integers(0, 1 << 30))))


@pytest.mark.parametrize("c", CASES, ids=[f"{c['H']}x{c['W']}_D{c['D']}_c{c['cost']}_b{c['bands']}_w{c['vwarm']}"
                                          f"_g{c['guess']}" for c in CASES])
def test_bands_random_shapes(eng, c):
    """Random shapes, band counts, warmups (1 row included) and wrong entering states, both
    cost types, minDisparity != 0: bit-exact, and the banded instance ran."""
    left, right, _ = synthetic.random_dot_pair(c["H"], c["W"], c["D"], seed=c["seed"])
    p = _params(c["cost"], c["D"], minD=c["minD"])
    c0 = eng.counters()
    out = _run(eng, left, right, p, flags=SWEEP8, bands=c["bands"], band_warmup=c["vwarm"], band_guess=c["guess"])
    _check(out, left, right, p)
    c1 = eng.counters()
    if c["H"] >= c["bands"]:
        assert c1["band_groups"] > c0["band_groups"], "the banded MODE 3 instance ran"
    if c["guess"] and c["H"] >= 2 * c["bands"]:
        assert c1["band_repairs"] > c0["band_repairs"]


@pytest.mark.parametrize("guess", [0, 1])
def test_bands_settings_ini_full_kitti(eng, guess):
    """The reference's own call (settings.ini: D = 160, window 5, one pair): the default engine
    picks row bands at one pair; bit-exact with and without a wrong entering state."""
    H, W, _ = synthetic.CONFIGS["kitti"]
    D = 160
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=1600 + guess)
    p = synthetic.parity_params(D, 5)
    c0 = eng.counters()
    out = _run(eng, left, right, p, band_guess=guess)
    _check(out, left, right, p)
    c1 = eng.counters()
    assert c1["band_groups"] > c0["band_groups"], "one pair of settings.ini runs on the row bands"
    if guess:
        assert c1["band_repairs"] - c0["band_repairs"] > 1000


def _hstripes(H, W, period, seed):
    """Textureless horizontal stripes (rows flat across the whole image) alternating with random
    texture: the vertical paths cannot meet inside a flat stripe taller than a band."""
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (H, W)).astype(np.uint8)
    flat = (np.arange(H) // period) % 2 == 0
    img[flat, :] = 120
    return img


VADV = [
    ("const", lambda H, W: (np.full((H, W), 77, np.uint8), np.full((H, W), 77, np.uint8))),
    ("hstripes", lambda H, W: (_hstripes(H, W, 30, 1), np.roll(_hstripes(H, W, 30, 1), -5, axis=1))),
    ("tall_stripes", lambda H, W: (_hstripes(H, W, 90, 2), np.roll(_hstripes(H, W, 90, 2), -2, axis=1))),
    ("vgradient", lambda H, W: (np.tile((np.arange(H, dtype=np.int64) % 256)[:, None], (1, W)).astype(np.uint8),
                                np.tile(((np.arange(H, dtype=np.int64) + 3) % 256)[:, None], (1, W)).astype(np.uint8))),
    ("noise_lr_indep", lambda H, W: (np.random.default_rng(13).integers(0, 256, (H, W)).astype(np.uint8),
                                     np.random.default_rng(14).integers(0, 256, (H, W)).astype(np.uint8))),
]


@pytest.mark.parametrize("name,make", VADV, ids=[a[0] for a in VADV])
@pytest.mark.parametrize("cost,D,P1,P2", [(1, 64, 10, 120), (1, 128, 1, 193), (0, 160, 600, 2400),
                                          (0, 96, 200, 201)])
@pytest.mark.parametrize("guess", [0, 1])
def test_bands_adversarial(eng, name, make, cost, D, P1, P2, guess):
    """Inputs chosen against the vertical speculation: flat images, flat horizontal stripes
    shorter and taller than a band, a vertical gradient, uncorrelated noise; P2 = P1 + 1 and a
    large P2; zero and wrong entering states; 6 bands of 30 rows."""
    H, W = 180, D + 300
    left, right = make(H, W)
    p = dict(_params(cost, D), P1=P1, P2=P2)
    out = _run(eng, left, right, p, flags=SWEEP8, bands=6, band_guess=guess)
    _check(out, left, right, p)


@pytest.mark.parametrize("cost", [0, 1])
def test_bands_carry_through_tall_flat_stripes(eng, cost):
    """A flat stripe taller than a band, with a wrong entering state: a repaired chain does not
    meet the speculative one inside its band (SM_COUNTER_BAND_OPEN), so its true state is
    carried into the next boundary."""
    H, W, D = 240, 460, 128
    left, right = VADV[2][1](H, W)
    p = _params(cost, D)
    c0 = eng.counters()
    out = _run(eng, left, right, p, flags=SWEEP8, bands=8, band_guess=1)
    _check(out, left, right, p)
    c1 = eng.counters()
    assert c1["band_open"] > c0["band_open"], c1


def test_bands_two_pairs_and_volume(eng):
    """Two pairs per call (4 bands each by default) through the device batch entry, and an
    external f32 cost volume (u16 costs, 5 paths) on the bands."""
    import torch

    H, W, _ = synthetic.CONFIGS["kitti"]
    D = 128
    pairs = [synthetic.random_dot_pair(H, W, D, seed=2600 + i)[:2] for i in range(2)]
    p = _params(0, D)
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    out = torch.empty((2, H, W), dtype=torch.int16, device="cuda")
    c0 = eng.counters()
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.compute_batch_device(L.data_ptr(), R.data_ptr(), 2, H * W, H, W, W, synthetic.to_sm_params(p),
                                 out.data_ptr())
        eng.synchronize()
    finally:
        eng.set_stream(None)
    got = out.cpu().numpy()
    exp = ref_c.compute_many(pairs, p)
    for i in range(2):
        assert np.array_equal(got[i], exp[i]), i
    assert eng.counters()["band_groups"] > c0["band_groups"]
    # f32 volume, 5 paths, 6 bands
    Hv, Wv, Dv = 150, 400, 96
    l, r, _ = synthetic.random_dot_pair(Hv, Wv, Dv, seed=2700)
    vol = synthetic.absdiff_volume(l, r, Dv)[0]
    pv = dict(synthetic.cost_volume_params(Dv), mode=5)
    eng.set_debug_flags(SWEEP8)
    eng.set_tuning(eng.TUNE_BANDS, 6)
    try:
        o = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(pv), 0.0, synthetic.VOLUME_SCALE)
    finally:
        eng.set_debug_flags(0)
        eng.set_tuning(eng.TUNE_BANDS, 0)
    assert np.array_equal(o, ref_c.compute_volume(vol, pv, 0.0, synthetic.VOLUME_SCALE))


def test_bands_off_matches_bands_on_full_kitti_census(eng):
    """Census 5 paths, one full KITTI pair: bands off (SM_TUNE_BANDS 1, the per-direction
    engine) and the automatic bands give the oracle's map."""
    H, W, D = synthetic.CONFIGS["kitti"]
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=2800)
    p = _params(1, D)
    a = _run(eng, left, right, p, bands=1)
    b = _run(eng, left, right, p)
    exp = ref_c.compute(left, right, p)
    assert np.array_equal(a, exp) and np.array_equal(b, exp)


def test_band_tuning_arguments(eng):
    for key, bad in ((eng.TUNE_BANDS, -1), (eng.TUNE_BAND_WARMUP, -1), (eng.TUNE_BAND_GUESS, 2),
                     (eng.TUNE_COST_WGS, -1), (eng.TUNE_LR_STAGGER, 2)):
        with pytest.raises(ValueError):
            eng.set_tuning(key, bad)


@pytest.mark.parametrize("stagger", [0, -1])
def test_compute_disparity_stagger_matches_serial(stagger):
    """sm_compute_disparity with the left matcher staggered behind the right one's sweep (the
    default) and strictly after it: the same maps, equal to the C oracle's left matcher + the
    numpy WLS restatement (settings.ini, one KITTI pair, D = 160)."""
    from oracle import sgm_np, wls_np
    from stereo_match_amd import settings, wls
    from stereo_match_amd.stereo_vision import matcher_from_settings

    s = dict(settings.DEFAULT_SETTINGS, window_size=5)
    H, W, _ = synthetic.CONFIGS["kitti"]
    D = s["num_disparities"]
    gl, gr, _ = synthetic.random_dot_pair(H, W, D, seed=66)
    lm = matcher_from_settings(s)
    prm = lm.params()
    wf = wls.createDisparityWLSFilter(lm)
    wf.setLambda(s["lmbda"])
    wf.setSigmaColor(s["sigma"])
    wp = wf.params(H, W)
    e = _lib.Engine(0)
    try:
        e.set_tuning(e.TUNE_LR_STAGGER, stagger)
        d, f = e.compute_disparity(gl, gr, prm, wp)
        d2, f2 = e.compute_disparity(gl, gr, prm, wp)  # buffers reused
    finally:
        e.close()
    assert np.array_equal(d, d2) and np.array_equal(f, f2)
    hp = synthetic.parity_params(D, 5)
    lp = dict(hp, uniquenessRatio=0, disp12MaxDiff=1000000)
    dl = ref_c.compute(gl, gr, lp)
    assert np.array_equal(d, dl)
    dr = ref_c.compute(gr, gl, sgm_np.right_matcher_params(hp))
    wpar = dict(lmbda=80000.0, sigma=1.2, radius=(hp["blockSize"] + 1) // 2, min_disp=0, left_offset=D, right_offset=0)
    assert np.array_equal(f, wls_np.wls_filter(dl, gl, dr, wpar))


def test_compute_disparity_one_call_equals_three_calls():
    """The Python compute_disparity (one-call ABI for 2-D uint8 numpy pairs) against the
    reference's three calls made separately through the matcher / WLS objects: identical maps."""
    import stereo_match_amd as sm
    from stereo_match_amd import settings, wls
    from stereo_match_amd.stereo_vision import matcher_from_settings

    s = dict(settings.DEFAULT_SETTINGS, window_size=5)
    H, W = 200, 640
    gl, gr, _ = synthetic.random_dot_pair(H, W, s["num_disparities"], seed=67)
    d1, f1 = sm.compute_disparity(gl, gr, s)
    lm = matcher_from_settings(s)
    rmatch = sm.createRightMatcher(lm)
    wf = wls.createDisparityWLSFilter(lm)
    wf.setLambda(s["lmbda"])
    wf.setSigmaColor(s["sigma"])
    d2 = lm.compute(gl, gr)
    dr = rmatch.compute(gr, gl)
    f2 = wf.filter(d2, gl, None, dr)
    assert np.array_equal(d1, d2) and np.array_equal(f1, f2)


@pytest.mark.parametrize("cost,mode,n", [(1, 8, 8), (0, 5, 7), (1, 5, 3)])
def test_sweep_xcd_placement(eng, cost, mode, n):
    """The XCD-aware strip placement (SM_TUNE_SWEEP_XCD 1: a 1-D grid whose workgroups on one XCD
    hold adjacent strips, padding workgroups exiting at once): every pair equals the oracle."""
    import torch

    H, W, _ = synthetic.CONFIGS["kitti"]
    D = 128
    pairs = [synthetic.random_dot_pair(H, W, D, seed=3100 + 7 * cost + i)[:2] for i in range(n)]
    p = dict(_params(cost, D), mode=mode)
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    out = torch.empty((n, H, W), dtype=torch.int16, device="cuda")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.set_tuning(eng.TUNE_SWEEP_XCD, 1)
    eng.set_debug_flags(SWEEP8)
    try:
        eng.compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, synthetic.to_sm_params(p),
                                 out.data_ptr())
        eng.synchronize()
    finally:
        eng.set_tuning(eng.TUNE_SWEEP_XCD, 0)
        eng.set_debug_flags(0)
        eng.set_stream(None)
    got = out.cpu().numpy()
    exp = ref_c.compute_many(pairs, p)
    for i in range(n):
        assert np.array_equal(got[i], exp[i]), (i, int(np.sum(got[i] != exp[i])))


def test_line_strips_counter(eng):
    """SM_COUNTER_LINE_STRIPS: a KITTI census8 call on the lines engine adds its strips x pairs
    (the bench's boundary-state bytes use it), and nothing for a per-direction call."""
    H, W, _ = synthetic.CONFIGS["kitti"]
    left, right, _ = synthetic.random_dot_pair(H, W, 128, seed=3401)
    p = synthetic.headline_params(128)
    c0 = eng.counters()
    _run(eng, left, right, p, flags=SWEEP8)
    c1 = eng.counters()
    assert c1["line_groups"] == c0["line_groups"] + 1
    strips = c1["line_strips"] - c0["line_strips"]
    # strips of a 1114-column domain: at most 36 columns wide (the wide instance), at least 8
    assert 31 <= strips <= 140, strips
    _run(eng, left, right, p, flags=4096)  # per-direction engine
    assert eng.counters()["line_strips"] == c1["line_strips"]
