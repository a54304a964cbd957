"""GPU parity: the HIP path (through the C-ABI) against the CPU restatement.

Bar: bit-exact int16 output (integer WTA index AND the integer sub-pixel
value — OpenCV's sub-pixel step is integer arithmetic, so the north-star's
1e-4 float tolerance is met with zero error).  Parity with OpenCV itself is
unpinned (see oracle/sgm_np.py).
"""
import numpy as np
import pytest

from oracle import ref_c, sgm_np
from conftest import skip_unless_ablation
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(0)
    yield e
    e.close()


def run(eng, left, right, p):
    return eng.compute(left, right, synthetic.to_sm_params(p))


def test_golden_fixtures(eng, golden_cases):
    for name, left, right, p, expected, raw in golden_cases:
        out = run(eng, left, right, p)
        assert np.array_equal(out, expected), f"{name}: {np.sum(out != expected)} px differ"
        got_raw = np.frombuffer(eng.debug_fetch(2), np.int16).reshape(left.shape)
        assert np.array_equal(got_raw, raw), name


@pytest.mark.parametrize("cost", [0, 1])
def test_cost_volume_matches_oracle(eng, cost):
    left, right, _ = synthetic.random_dot_pair(40, 120, 32, seed=7)
    p = synthetic.headline_params(32) if cost else synthetic.parity_params(32)
    run(eng, left, right, p)
    C = sgm_np.cost_volume(left, right, sgm_np.normalize_params(p))
    dt = np.uint8 if cost else np.uint16
    got = np.frombuffer(eng.debug_fetch(0), dt).reshape(C.shape)
    assert np.array_equal(got.astype(np.int64), C)


def test_census_images_match_oracle(eng):
    left, right, _ = synthetic.random_dot_pair(37, 131, 32, seed=17)
    run(eng, left, right, synthetic.headline_params(32))
    got = np.frombuffer(eng.debug_fetch(3), np.uint64).reshape(2, 37, 131)
    assert np.array_equal(got[0], sgm_np.census9x7(left))
    assert np.array_equal(got[1], sgm_np.census9x7(right))


@pytest.mark.parametrize("cost,mode,D,flags", [(1, 8, 32, 0), (0, 5, 32, 0), (0, 8, 32, 0), (1, 8, 64, 0),
                                                (0, 5, 64, 0), (1, 5, 128, 0), (1, 8, 64, 48), (0, 5, 128, 48),
                                                (1, 8, 128, 1024), (1, 8, 128, 2048), (1, 8, 48, 1024)])
def test_path_volumes_match_oracle(eng, cost, mode, D, flags):
    skip_unless_ablation(flags)
    left, right, _ = synthetic.random_dot_pair(33, 101 + D, D, seed=8)
    p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=mode)
    # flags 48 = fused row kernel (32) + keep its W volume (16), which it normally never writes;
    # 4096 = per-direction engine (the fused sweeps never materialise the per-direction volumes)
    eng.set_debug_flags(flags | 4096)
    try:
        run(eng, left, right, p)
    finally:
        eng.set_debug_flags(0)
    prm = sgm_np.normalize_params(p)
    C = sgm_np.cost_volume(left, right, prm)
    dt = np.uint8 if cost else np.uint16
    vols = np.frombuffer(eng.debug_fetch(1), dt).reshape((mode,) + C.shape)
    # engine direction order: E, W, SE, S, SW, NE, N, NW
    order = [(1, 0), (-1, 0), (1, 1), (0, 1), (-1, 1), (1, -1), (0, -1), (-1, -1)][:mode]
    for k, d in enumerate(order):
        L = sgm_np.aggregate_path(C, d, prm["P1"], prm["P2"])
        assert np.array_equal(vols[k].astype(np.int64), L), f"direction {d}"


CASES = []
_rng = np.random.default_rng(1234)
for _i in range(36):
    D = int(_rng.choice([16, 32, 48, 64, 96, 128, 160, 256]))
    H = int(_rng.integers(1, 50))
    W = int(_rng.integers(D + 1, D + 200)) if _rng.random() < 0.8 else int(_rng.integers(1, D + 3))
    CASES.append(dict(H=H, W=W, D=D, minD=int(_rng.choice([0, 0, 0, 5, -9, -D + 1])),
                      cost=int(_rng.integers(0, 2)), mode=int(_rng.choice([5, 8])),
                      bs=int(_rng.choice([1, 3, 5, 7])), uniq=int(_rng.choice([0, 10, 15])),
                      d12=int(_rng.choice([1, 2, 1000000])), seed=int(_rng.integers(0, 1 << 30))))


@pytest.mark.parametrize("flags", [0, 4096, 16384, 16384 | (1 << 19), 16384 | (1 << 21), 32768],
                         ids=["default", "perdir", "sweep8", "sweep8narrow", "sweep8wide", "hybrid"])
@pytest.mark.parametrize("c", CASES, ids=lambda c: "H{H}W{W}D{D}m{minD}c{cost}p{mode}".format(**c))
def test_random_shapes_vs_c_oracle(eng, c, flags):
    """Default engines (one pair per call: per-direction), the per-direction
    engine (4096), the fused sweeps forced for every configuration (16384; by
    default they need >= 3 pairs per launch group; one pair picks narrow strips
    where the strip-width model prefers them), on narrow strips everywhere
    (1 << 19) and on wide strips wherever built (1 << 21), and the hybrid engine
    (32768, 5 and 8 paths; ablation build)."""
    skip_unless_ablation(flags)
    eng.set_debug_flags(flags)
    try:
        _random_case(eng, c)
    finally:
        eng.set_debug_flags(0)


def _random_case(eng, c):
    left, right, _ = synthetic.random_dot_pair(c["H"], c["W"], c["D"], seed=c["seed"])
    if c["cost"]:
        p = dict(synthetic.headline_params(c["D"]), minDisparity=c["minD"], mode=c["mode"],
                 uniquenessRatio=c["uniq"], disp12MaxDiff=c["d12"])
    else:
        bs = c["bs"]
        p = dict(synthetic.parity_params(c["D"]), minDisparity=c["minD"], mode=c["mode"], blockSize=bs,
                 P1=8 * bs * bs, P2=32 * bs * bs, uniquenessRatio=c["uniq"], disp12MaxDiff=c["d12"])
    expected = ref_c.compute(left, right, p)
    out = run(eng, left, right, p)
    assert np.array_equal(out, expected), f"{np.sum(out != expected)} px differ"


@pytest.mark.parametrize("mode", [8, 5])
@pytest.mark.parametrize("H,W,minD", [(37, 257, 0), (52, 300, 0), (29, 334, -7), (64, 700, 3), (9, 1200, 0)])
def test_d256_wide_strips_32_lane_lines(eng, H, W, minD, mode):
    """Census D = 256 on the wide sweep instance (32-lane lines across two DPP rows, 16-wave
    workgroups of 2-column waves; flags 16384 | 1 << 21): ragged strips, one to several
    dozen strips, both sweep modes of the census cost (8 paths: modes 0 + 2; 5: mode 1)."""
    left, right, _ = synthetic.random_dot_pair(H, W, 256, seed=H * 1000 + W)
    p = dict(synthetic.headline_params(256), minDisparity=minD, mode=mode)
    eng.set_debug_flags(16384 | (1 << 21))
    try:
        out = run(eng, left, right, p)
    finally:
        eng.set_debug_flags(0)
    exp = ref_c.compute(left, right, p)
    assert np.array_equal(out, exp), f"{np.sum(out != exp)} px differ"


@pytest.mark.parametrize("bs,D,minD", [(9, 16, 0), (11, 48, -5), (9, 144, 3), (11, 80, 0), (1, 256, 0), (3, 160, -20)])
def test_sgbm_cost_block_sizes(eng, bs, D, minD):
    """The streaming SGBM cost kernel at every blockSize radius and odd /
    small column-group counts (D = 144, 160: 3 column groups per workgroup)."""
    left, right, _ = synthetic.random_dot_pair(45, 330, D, seed=bs * 1000 + D)
    p = dict(synthetic.parity_params(D), minDisparity=minD, blockSize=bs, P1=8 * bs * bs, P2=32 * bs * bs)
    if bs >= 9:
        p["preFilterCap"] = 15  # int16-exact domain: bs^2 * (2 * cap + 63) + P2 <= 16383
    for mode in (5, 8):
        q = dict(p, mode=mode)
        assert np.array_equal(run(eng, left, right, q), ref_c.compute(left, right, q)), (bs, D, minD, mode)


@pytest.mark.parametrize("name,cost,mode,flags", [("kitti", 1, 8, 0), ("kitti", 0, 5, 0), ("kitti", 0, 8, 0),
                                                  ("kitti", 1, 5, 0), ("mccnn", 1, 8, 0), ("kitti", 1, 8, 32),
                                                  ("kitti", 1, 8, 1024), ("kitti", 1, 8, 512),
                                                  ("kitti", 1, 8, 16384), ("kitti", 0, 8, 16384),
                                                  ("kitti", 0, 5, 4096), ("mccnn", 1, 8, 16384),
                                                  ("kitti", 1, 8, 32768), ("kitti", 0, 8, 32768),
                                                  ("mccnn", 1, 8, 32768), ("kitti", 0, 5, 32768),
                                                  ("kitti", 0, 5, 1 << 22), ("kitti", 0, 8, 4096),
                                                  ("kitti", 0, 5, 16384), ("kitti", 1, 5, 16384),
                                                  # sweep-engine E/W kernel swapped (256), k_sweep2 (128, 1 << 27)
                                                  ("kitti", 1, 8, 16384 | 256), ("kitti", 0, 5, 256),
                                                  ("kitti", 1, 8, 16384 | 128), ("kitti", 1, 8, 16384 | (1 << 27)),
                                                  ("kitti", 1, 5, 128),
                                                  # narrow (1 << 19) and wide (1 << 21) sweep strips
                                                  ("kitti", 1, 8, 16384 | (1 << 19)), ("kitti", 0, 5, 16384 | (1 << 19)),
                                                  ("kitti", 1, 8, 16384 | (1 << 21)), ("kitti", 0, 5, 16384 | (1 << 21)),
                                                  ("kitti", 0, 8, 16384 | (1 << 21)), ("mccnn", 1, 8, 16384 | (1 << 21))])
def test_full_size_bit_exact(eng, name, cost, mode, flags):
    skip_unless_ablation(flags)
    H, W, D = synthetic.CONFIGS[name]
    left, right, gt = synthetic.random_dot_pair(H, W, D, seed=42)
    p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=mode)
    eng.set_debug_flags(flags)
    try:
        out = run(eng, left, right, p)
    finally:
        eng.set_debug_flags(0)
    expected = ref_c.compute(left, right, p)
    assert np.array_equal(out, expected), f"{np.sum(out != expected)} px differ"
    valid = out >= 0
    assert valid.mean() > 0.8
    assert np.mean(np.abs(((out.astype(np.int64) + 8) >> 4) - gt)[valid] <= 1) > 0.98


@pytest.mark.slow
def test_middlebury_full_size(eng):
    H, W, D = synthetic.CONFIGS["middlebury"]
    left, right, gt = synthetic.random_dot_pair(H, W, D, seed=9)
    p = synthetic.headline_params(D)
    out = run(eng, left, right, p)
    again = run(eng, left, right, p)
    assert np.array_equal(out, again)  # deterministic
    valid = out >= 0
    assert valid.mean() > 0.8
    assert np.mean(np.abs(((out.astype(np.int64) + 8) >> 4) - gt)[valid] <= 1) > 0.98
    # bit-exact on a full-width band (rows cut so the C oracle stays quick;
    # a band is a valid image of its own)
    band = slice(700, 900)
    lb, rb = np.ascontiguousarray(left[band]), np.ascontiguousarray(right[band])
    assert np.array_equal(run(eng, lb, rb, p), ref_c.compute(lb, rb, p))


def test_batch_device_matches_single(eng):
    import torch

    H, W, D = 60, 200, 64
    pairs = [synthetic.random_dot_pair(H, W, D, seed=s)[:2] for s in range(3)]
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    out = torch.empty((3, H, W), dtype=torch.int16, device="cuda")
    p = synthetic.headline_params(D)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.compute_batch_device(L.data_ptr(), R.data_ptr(), 3, H * W, H, W, W, synthetic.to_sm_params(p),
                             out.data_ptr())
    got = out.cpu().numpy()  # ordered after the engine's work: same stream
    eng.set_stream(None)
    for i, (a, b) in enumerate(pairs):
        assert np.array_equal(got[i], ref_c.compute(a, b, p))
    # SGBM mode batch too (cost volume per pair inside one launch group)
    q = synthetic.parity_params(D)
    eng.compute_batch_device(L.data_ptr(), R.data_ptr(), 3, H * W, H, W, W, synthetic.to_sm_params(q),
                             out.data_ptr())
    eng.synchronize()
    got = out.cpu().numpy()
    for i, (a, b) in enumerate(pairs):
        assert np.array_equal(got[i], ref_c.compute(a, b, q))


@pytest.mark.parametrize("flags", [0, 32, 64, 96, 4096, 8192, 16384, 16384 | 8192, 32768, 32768 | 64])
def test_batch_pipeline_groups(eng, flags):
    """Batches through the normal pipeline (fused sweeps), the fused row kernel
    (32), the two-stream overlap (64: 7 pairs -> launch groups of 4 + 3 on
    alternating buffer sets, WTA of group g on the second stream beside paths
    of group g+1), the per-direction engine (4096), one pair per sweep
    launch (8192) and the hybrid 8-path engine (32768); then a call with a different geometry reuses (and regrows)
    the sets."""
    import torch

    skip_unless_ablation(flags)
    eng.set_debug_flags(flags)
    try:
        for (H, W, D, n) in [(70, 260, 64, 7), (90, 330, 128, 5)]:
            pairs = [synthetic.random_dot_pair(H, W, D, seed=100 + s)[:2] for s in range(n)]
            L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
            R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
            out = torch.full((n, H, W), 12345, dtype=torch.int16, device="cuda")
            for p in (synthetic.headline_params(D), synthetic.parity_params(D)):
                eng.set_stream(torch.cuda.current_stream().cuda_stream)
                eng.compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W,
                                         synthetic.to_sm_params(p), out.data_ptr())
                got = out.cpu().numpy()  # same stream: ordered after both internal streams
                eng.synchronize()  # raises if a sweep strip hand-off timed out
                eng.set_stream(None)
                for i, (a, b) in enumerate(pairs):
                    assert np.array_equal(got[i], ref_c.compute(a, b, p)), (H, W, D, i, p.get("cost"))
    finally:
        eng.set_debug_flags(0)


def test_torch_tensor_interface():
    import torch

    import stereo_match_amd as sm

    left, right, _ = synthetic.random_dot_pair(50, 150, 32, seed=3)
    m = sm.StereoSGBM_create(numDisparities=32, blockSize=5, P1=600, P2=2400, disp12MaxDiff=1,
                             uniquenessRatio=15, preFilterCap=63)
    a = m.compute(left, right)
    t = m.compute(torch.tensor(left, device="cuda"), torch.tensor(right, device="cuda"))
    assert t.dtype == torch.int16 and t.is_cuda
    assert np.array_equal(t.cpu().numpy(), a)
    assert np.array_equal(a, ref_c.compute(left, right, synthetic.parity_params(32)))


def test_compute_disparity_left_matcher_semantics():
    """compute_disparity's displ: createDisparityWLSFilter (called before
    compute, stereo_vision.py:172 vs :178) sets uniqueness 0 / disp12 1e6."""
    import stereo_match_amd as sm
    from stereo_match_amd import wls

    s = dict(sm.DEFAULT_SETTINGS, window_size=5, num_disparities=32)
    left, right, _ = synthetic.random_dot_pair(48, 160, 32, seed=4)
    lm = sm.matcher_from_settings(s)
    rm = sm.createRightMatcher(lm)
    wls.createDisparityWLSFilter(lm)
    displ = lm.compute(left, right)
    dispr = rm.compute(right, left)
    p = dict(synthetic.parity_params(32), uniquenessRatio=0, disp12MaxDiff=1000000)
    assert np.array_equal(displ, ref_c.compute(left, right, p))
    assert np.array_equal(dispr, ref_c.compute(right, left, sgm_np.right_matcher_params(
        synthetic.parity_params(32))))


def test_unsupported_and_bad_args_raise(eng):
    l = np.zeros((10, 40), np.uint8)
    with pytest.raises(ValueError):
        run(eng, l, l, dict(synthetic.parity_params(16), numDisparities=24))
    with pytest.raises(_lib.SmError):  # beyond the built window (blockSize <= 55)
        run(eng, l, l, dict(synthetic.parity_params(16), blockSize=57))
    with pytest.raises(_lib.SmError):  # preFilterCap > 126: OpenCV's u8 clip table itself wraps
        run(eng, l, l, dict(synthetic.parity_params(16), preFilterCap=200))


def test_timing_counters(eng):
    left, right, _ = synthetic.random_dot_pair(40, 200, 64, seed=5)
    eng.set_timing(True)
    eng.reset_timing()
    for _ in range(3):
        run(eng, left, right, synthetic.headline_params(64))
    t = eng.timing()
    eng.set_timing(False)
    assert t["paths"][1] == 3 and t["total"][1] == 3
    assert 0 < t["paths"][0] <= t["total"][0]
    # sweep engine (5 paths; forced: one pair per call runs per-direction by default):
    # E/W kernel and the WTA sweep are timed on their own too
    eng.set_timing(True)
    eng.reset_timing()
    eng.set_debug_flags(16384)
    try:
        for _ in range(2):
            run(eng, left, right, synthetic.parity_params(64))
    finally:
        eng.set_debug_flags(0)
    t = eng.timing()
    eng.set_timing(False)
    assert t["paths"][1] == 2 and t["horizontal"][1] == 2 and t["sweep_wta"][1] == 2 and t["wta"][1] == 2
    # only the named stages record events (SM_TIMING_ONLY: what bench.py's timed region uses)
    eng.set_timing(True, stages=["sweep_wta"])
    eng.reset_timing()
    eng.set_debug_flags(16384)
    try:
        out = run(eng, left, right, synthetic.parity_params(64))
    finally:
        eng.set_debug_flags(0)
    t = eng.timing()
    eng.set_timing(False)
    assert t["sweep_wta"][1] == 1 and t["sweep_wta"][0] > 0
    assert all(v[1] == 0 for k, v in t.items() if k != "sweep_wta")
    assert np.array_equal(out, ref_c.compute(left, right, synthetic.parity_params(64)))


# ---------------------------------------------------------------- mc-cnn cost volume
def test_golden_volume_fixtures(eng, golden_volume_cases):
    for name, vol, p, off, sc, expected, raw in golden_volume_cases:
        out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), off, sc)
        assert np.array_equal(out, expected), f"{name}: {np.sum(out != expected)} px differ"
        got_raw = np.frombuffer(eng.debug_fetch(2), np.int16).reshape(expected.shape)
        assert np.array_equal(got_raw, raw), name


def test_volume_quantised_cost_matches_oracle(eng):
    rng = np.random.default_rng(21)
    vol = rng.standard_normal((48, 23, 130)).astype(np.float32)
    vol[rng.random(vol.shape) < 0.03] = np.nan
    p = dict(synthetic.cost_volume_params(48), minDisparity=2)
    eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.1, 900.0)
    prm = sgm_np.normalize_params(dict(p, cost=2))
    C = sgm_np.quantize_volume(vol, prm, 0.1, 900.0)
    got = np.frombuffer(eng.debug_fetch(0), np.uint16).reshape(C.shape)
    assert np.array_equal(got, C)


_VCASES = [dict(H=int(_rng.integers(1, 70)), W=int(_rng.integers(20, 300)), D=16 * int(_rng.integers(1, 9)),
                minD=int(_rng.integers(-8, 8)), mode=int(_rng.choice([5, 8])), seed=int(_rng.integers(0, 1 << 30)))
           for _ in range(12)]


@pytest.mark.parametrize("c", _VCASES, ids=lambda c: "H{H}W{W}D{D}m{minD}p{mode}".format(**c))
def test_volume_random_shapes_vs_c_oracle(eng, c):
    rng = np.random.default_rng(c["seed"])
    vol = rng.random((c["D"], c["H"], c["W"]), dtype=np.float32)
    p = dict(synthetic.cost_volume_params(c["D"]), minDisparity=c["minD"], mode=c["mode"])
    out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.0, synthetic.VOLUME_SCALE)
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, synthetic.VOLUME_SCALE))


@pytest.mark.parametrize("mode,flags", [(8, 0), (5, 0), (8, 4096)])
def test_volume_full_size_mccnn(eng, mode, flags):
    """Config C: (1, 192, 375, 1242) float32 |L-R| volume of the KITTI-size pair
    (default engine = fused sweeps; 4096 = per-direction engine)."""
    H, W, D = synthetic.CONFIGS["mccnn"]
    left, right, gt = synthetic.random_dot_pair(H, W, D, seed=7)
    vol = synthetic.absdiff_volume(left, right, D)
    p = dict(synthetic.cost_volume_params(D), mode=mode)
    eng.set_debug_flags(flags)
    try:
        out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.0, synthetic.VOLUME_SCALE)
    finally:
        eng.set_debug_flags(0)
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, synthetic.VOLUME_SCALE))
    valid = out >= 0
    assert valid.mean() > 0.7
    assert np.mean(np.abs(((out.astype(np.int64) + 8) >> 4) - gt)[valid] <= 1) > 0.97


_DVCASES = [dict(H=int(_rng.integers(1, 60)), W=int(_rng.integers(8, 260)), D=int(d),
                 minD=int(_rng.integers(-6, 6)), mode=int(_rng.choice([5, 8])), seed=int(_rng.integers(0, 1 << 30)))
            for d in (1, 2, 3, 5, 17, 20, 37, 100, 127, 150, 228, 255)]


@pytest.mark.parametrize("flags", [0, 4096, 16384])
@pytest.mark.parametrize("c", _DVCASES, ids=lambda c: "H{H}W{W}D{D}m{minD}p{mode}".format(**c))
def test_volume_any_plane_count_vs_c_oracle(eng, c, flags):
    """An external volume keeps the planes it was made with (mc-cnn: 228,
    mapTo3D_mc_cnn.py:71): D not a multiple of 16 runs on padded kernels whose
    pad planes never win (sm_cost.hpp vol_pad_cost), on every engine (flags: 0
    default, 4096 per-direction, 16384 fused sweeps)."""
    rng = np.random.default_rng(c["seed"])
    vol = rng.random((c["D"], c["H"], c["W"]), dtype=np.float32)
    vol[rng.random(vol.shape) < 0.02] = np.nan
    p = dict(synthetic.cost_volume_params(c["D"]), minDisparity=c["minD"], mode=c["mode"])
    eng.set_debug_flags(flags)
    try:
        out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.0, synthetic.VOLUME_SCALE)
    finally:
        eng.set_debug_flags(0)
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, synthetic.VOLUME_SCALE))


@pytest.mark.parametrize("uniq", [0, 15, 60, 99])
def test_volume_d3_uniqueness_no_far_planes(eng, uniq):
    """D <= 3: no disparity is 'far' from the winner, so the uniqueness test can never reject;
    the pad planes must not act as far entries either (any uniquenessRatio)."""
    rng = np.random.default_rng(uniq)
    vol = rng.random((3, 20, 50), dtype=np.float32)
    p = dict(synthetic.cost_volume_params(3), uniquenessRatio=uniq, mode=8)
    out = eng.aggregate_cost_f32(vol, synthetic.to_sm_params(p), 0.0, synthetic.VOLUME_SCALE)
    assert np.array_equal(out, ref_c.compute_volume(vol, p, 0.0, synthetic.VOLUME_SCALE))


def test_volume_reference_mccnn_memmap_as_documented(tmp_path):
    """The reference's own mc-cnn volume shape, (1, 228, 1280, 720) float32 memmapped at
    mapTo3D_mc_cnn.py:71 (made with -disp_max 228, mc_cnn/script.py:9-10), through the
    call INTEGRATION.md §2 shows, bit-exact against the C oracle (synthetic content: the
    reference ships no volume)."""
    import stereo_match_amd as sma

    D, H, W = 228, 1280, 720
    left, right, gt = synthetic.random_dot_pair(H, W, D, seed=228)
    path = tmp_path / "left.bin"
    mm = np.memmap(path, dtype=np.float32, mode="w+", shape=(1, D, H, W))
    mm[:] = synthetic.absdiff_volume(left, right, D)
    mm.flush()
    del mm
    # INTEGRATION.md §2, as written
    vm = sma.StereoSGBM_create(numDisparities=228, P1=200, P2=2000, disp12MaxDiff=1, uniquenessRatio=15,
                               mode=sma.STEREO_SGBM_MODE_HH)
    disp = vm.computeFromCost(np.memmap(path, np.float32, mode="r", shape=(1, 228, 1280, 720)),
                              offset=0.0, scale=4000.0)
    vol = np.memmap(path, np.float32, mode="r", shape=(1, D, H, W))[0]
    p = dict(synthetic.cost_volume_params(D), P1=200, P2=2000, mode=8)
    assert np.array_equal(disp, ref_c.compute_volume(np.asarray(vol), p, 0.0, 4000.0))
    valid = disp >= 0
    assert valid.mean() > 0.6
    assert np.mean(np.abs(((disp.astype(np.int64) + 8) >> 4) - gt)[valid] <= 1) > 0.95


def test_volume_torch_batch_and_matcher():
    import torch

    import stereo_match_amd as sm

    H, W, D, n = 50, 180, 32, 3
    vols = []
    for s in range(n):
        l, r, _ = synthetic.random_dot_pair(H, W, D, seed=30 + s)
        vols.append(synthetic.absdiff_volume(l, r, D)[0])
    p = synthetic.cost_volume_params(D)
    m = sm.StereoSGBM_create(numDisparities=D, P1=p["P1"], P2=p["P2"], disp12MaxDiff=1, uniquenessRatio=15,
                             mode=sm.STEREO_SGBM_MODE_HH)
    a = m.computeFromCost(vols[0][None], 0.0, synthetic.VOLUME_SCALE)
    assert np.array_equal(a, ref_c.compute_volume(vols[0], p, 0.0, synthetic.VOLUME_SCALE))
    t = m.computeFromCost(torch.tensor(vols[0], device="cuda"), 0.0, synthetic.VOLUME_SCALE)
    assert np.array_equal(t.cpu().numpy(), a)
    V = torch.tensor(np.stack(vols), device="cuda")
    out = torch.empty((n, H, W), dtype=torch.int16, device="cuda")
    eng = _lib.engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.aggregate_cost_f32_device(V.data_ptr(), n, D * H * W, D, H, W, synthetic.to_sm_params(p), 0.0,
                                  synthetic.VOLUME_SCALE, out.data_ptr())
    got = out.cpu().numpy()
    for i in range(n):
        assert np.array_equal(got[i], ref_c.compute_volume(vols[i], p, 0.0, synthetic.VOLUME_SCALE)), i


def test_volume_bad_args(eng):
    vol = np.zeros((16, 8, 40), np.float32)
    with pytest.raises(ValueError):  # planes != numDisparities
        eng.aggregate_cost_f32(vol, synthetic.to_sm_params(synthetic.cost_volume_params(32)))
    with pytest.raises(_lib.SmError):  # P2 beyond the exact range
        eng.aggregate_cost_f32(vol, synthetic.to_sm_params(dict(synthetic.cost_volume_params(16), P2=13000)))


# ---------------------------------------------------------------- speckle filter
_SCASES = [dict(H=int(_rng.integers(8, 90)), W=int(_rng.integers(60, 260)), D=16 * int(_rng.integers(1, 4)),
                ws=int(_rng.choice([4, 20, 60, 200])), rng=int(_rng.choice([1, 2, 4])), cost=int(_rng.integers(0, 2)),
                seed=int(_rng.integers(0, 1 << 30))) for _ in range(10)]


@pytest.mark.parametrize("c", _SCASES, ids=lambda c: "H{H}W{W}D{D}ws{ws}r{rng}c{cost}".format(**c))
def test_speckle_filter_in_matcher_vs_c_oracle(eng, c):
    left, right, _ = synthetic.random_dot_pair(c["H"], c["W"], c["D"], seed=c["seed"])
    base = synthetic.headline_params(c["D"]) if c["cost"] else synthetic.parity_params(c["D"])
    p = dict(base, speckleWindowSize=c["ws"], speckleRange=c["rng"])
    out = run(eng, left, right, p)
    assert np.array_equal(out, ref_c.compute(left, right, p))


def test_speckle_filter_standalone_and_full_size(eng):
    import stereo_match_amd as sm

    rng = np.random.default_rng(3)
    # blocky map with many small and a few large regions, plus invalid pixels
    img = (rng.integers(0, 6, (40, 50)) * 40).astype(np.int16)
    img = np.kron(img, np.ones((3, 2), np.int16))[:100, :90]
    img[rng.random(img.shape) < 0.1] = -16
    for ws, md in [(1, 0), (6, 0), (30, 16), (500, 40)]:
        exp = sgm_np.filter_speckles(img, -16, ws, md)
        assert np.array_equal(eng.filter_speckles(img, -16, ws, md), exp), (ws, md)
    a = img.copy()
    sm.filterSpeckles(a, -16, 30, 16)
    assert np.array_equal(a, sgm_np.filter_speckles(img, -16, 30, 16))
    H, W, D = synthetic.CONFIGS["kitti"]
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=11)
    p = dict(synthetic.headline_params(D), speckleWindowSize=100, speckleRange=2)
    assert np.array_equal(run(eng, left, right, p), ref_c.compute(left, right, p))
    # the union-find is lock-free across all XCDs: repeat to catch racy links
    base = ref_c.compute(left, right, synthetic.headline_params(D))
    exp = sgm_np.filter_speckles(base, -16, 100, 32)
    for _ in range(5):
        assert np.array_equal(eng.filter_speckles(base, -16, 100, 32), exp)


def test_single_process_multi_context_batch():
    """sm_compute_batch: host pairs sharded over several contexts (here two
    contexts on the one GPU of the box, each on its own host thread)."""
    engines = [_lib.Engine(0), _lib.Engine(0)]
    try:
        H, W, D = 48, 170, 32
        pairs = [synthetic.random_dot_pair(H, W, D, seed=90 + i)[:2] for i in range(5)]
        p = synthetic.headline_params(D)
        out = _lib.compute_batch(engines, [a for a, _ in pairs], [b for _, b in pairs], synthetic.to_sm_params(p))
        for i, (a, b) in enumerate(pairs):
            assert np.array_equal(out[i], ref_c.compute(a, b, p)), i
        with pytest.raises(ValueError):
            _lib.compute_batch(engines, [pairs[0][0]], [pairs[0][1]],
                               synthetic.to_sm_params(dict(p, numDisparities=24)))
    finally:
        for e in engines:
            e.close()


# ---------------------------------------------------------------- property-based sweep over the whole parameter space
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(H=st.integers(1, 48), W=st.integers(8, 200), Dk=st.integers(1, 6), minD=st.integers(-20, 20),
       cost=st.sampled_from([0, 1]), mode=st.sampled_from([5, 8]), bs=st.sampled_from([1, 3, 5, 7, 9, 11]),
       P1=st.integers(0, 40), P2x=st.integers(0, 8), uniq=st.integers(-1, 30), d12=st.integers(-1, 6),
       pfc=st.integers(0, 63), sws=st.sampled_from([0, 0, 0, 5, 40]), srange=st.integers(0, 4),
       seed=st.integers(0, 2**31 - 1))
def test_hypothesis_matcher_vs_c_oracle(eng, H, W, Dk, minD, cost, mode, bs, P1, P2x, uniq, d12, pfc, sws, srange,
                                        seed):
    D = 16 * Dk
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=seed)
    P2 = P1 * P2x  # 0 lets the normaliser pick max(5, P1+1)
    if cost == 1:
        P1, P2 = min(P1, 40), min(P2, 193)
    p = dict(minDisparity=minD, numDisparities=D, blockSize=bs, P1=P1, P2=P2, disp12MaxDiff=d12,
             uniquenessRatio=uniq, preFilterCap=pfc, speckleWindowSize=sws, speckleRange=srange, mode=mode,
             cost=cost)
    # outside the int16-exact range the wide path (sm_wide.hpp) reproduces OpenCV's
    # x86 saturating arithmetic, which the C oracle restates
    out = run(eng, left, right, p)
    assert np.array_equal(out, ref_c.compute(left, right, p))


@pytest.mark.parametrize("cost,mode", [(1, 8), (0, 5), (0, 8)])
def test_sweep_strip_widths_agree_on_a_kitti_batch(eng, cost, mode):
    """8 KITTI pairs per call (the bench's launch group): the default sweeps (each
    pass picks narrow or wide strips by its model), narrow (1 << 19) and wide
    (1 << 21) strips forced, and the per-direction engine (4096) return the same
    maps, and every pair of every engine equals the C oracle."""
    import torch

    H, W, D = synthetic.CONFIGS["kitti"]
    n = 8
    pairs = [synthetic.random_dot_pair(H, W, D, seed=300 + s)[:2] for s in range(n)]
    p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=mode)
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    outs = {}
    for flags in (0, 1 << 19, 1 << 21, 4096):
        out = torch.full((n, H, W), 12345, dtype=torch.int16, device="cuda")
        eng.set_debug_flags(flags)
        try:
            eng.set_stream(torch.cuda.current_stream().cuda_stream)
            eng.compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, synthetic.to_sm_params(p),
                                     out.data_ptr())
            outs[flags] = out.cpu().numpy()
            eng.synchronize()
        finally:
            eng.set_stream(None)
            eng.set_debug_flags(0)
    exp = ref_c.compute_many(pairs, p)  # every pair against the oracle
    for flags, o in outs.items():
        for i in range(n):
            assert np.array_equal(o[i], exp[i]), (flags, i, int(np.sum(o[i] != exp[i])))
