"""GPU tests added in round 2: the fused sweeps' guarded fallback and CU-mask
sizing, BASELINE config 1 (Tsukuba) and the Middlebury full frame against the C
oracle, the reference surface ``compute_disparity`` at settings.ini values on
a full KITTI frame, and the RCCL gather of int16 maps on one GPU."""
import os
import socket

import numpy as np
import pytest

from oracle import ref_c, sgm_np, wls_np
from conftest import ABLATION_FLAGS, ablation_build
from stereo_match_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

FORCE_FALLBACK = 1 << 23  # sm_api.hip DBG_FORCE_FALLBACK
SWEEP8 = 16384            # force the fused sweeps (any group size, census 8 paths too)
PERDIR = 4096


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(0)
    yield e
    e.close()


def _run(eng, left, right, p, flags=0):
    eng.set_debug_flags(flags)
    try:
        return eng.compute(left, right, synthetic.to_sm_params(p))
    finally:
        eng.set_debug_flags(0)


@pytest.mark.parametrize("cost,mode,extra", [(1, 8, SWEEP8), (0, 5, SWEEP8), (0, 8, SWEEP8), (1, 5, SWEEP8)],
                         ids=["census8", "sgbm5", "sgbm8", "census5"])
def test_forced_sweep_fallback_is_exact(eng, cost, mode, extra):
    """Every sweep group flagged as given-up: the guarded per-direction launches
    recompute it on the device, the call succeeds and the maps are exact."""
    H, W, D = 80, 300, 64
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=21)
    p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=mode)
    before = eng.counters()["sweep_fallbacks"]
    out = _run(eng, left, right, p, extra | FORCE_FALLBACK)
    assert np.array_equal(out, ref_c.compute(left, right, p))
    assert eng.counters()["sweep_fallbacks"] == before + 1
    # unflagged: the guarded launches do nothing
    out = _run(eng, left, right, p, extra)
    assert np.array_equal(out, ref_c.compute(left, right, p))
    assert eng.counters()["sweep_fallbacks"] == before + 1


def test_forced_fallback_batch_device(eng):
    import torch

    H, W, D, n = 70, 260, 64, 5
    pairs = [synthetic.random_dot_pair(H, W, D, seed=300 + s)[:2] for s in range(n)]
    L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
    R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
    out = torch.full((n, H, W), 777, dtype=torch.int16, device="cuda")
    p = synthetic.parity_params(D)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.set_debug_flags(FORCE_FALLBACK | SWEEP8 | (2 << 16))  # groups of 2 pairs: 3 groups, all recomputed
    before = eng.counters()["sweep_fallbacks"]
    try:
        eng.compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, synthetic.to_sm_params(p),
                                 out.data_ptr())
        eng.synchronize()
    finally:
        eng.set_debug_flags(0)
        eng.set_stream(None)
    got = out.cpu().numpy()
    for i, (a, b) in enumerate(pairs):
        assert np.array_equal(got[i], ref_c.compute(a, b, p)), i
    assert eng.counters()["sweep_fallbacks"] == before + 3


@pytest.mark.parametrize("mode,cost,extra", [(5, 0, SWEEP8), (8, 1, SWEEP8)], ids=["sgbm5", "census8"])
def test_sweep_on_half_the_cus(mode, cost, extra):
    """A context restricted to half the CUs (hipExtStreamCreateWithCUMask):
    the sweeps size their co-resident launches from the CUs the stream
    reaches, so the full-size result is exact and nothing falls back."""
    import torch

    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    e = _lib.Engine(0)
    try:
        e.set_cu_mask(list(range(0, ncu, 2)))
        H, W, D = synthetic.CONFIGS["kitti"]
        left, right, _ = synthetic.random_dot_pair(H, W, D, seed=5)
        p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=mode)
        out = _run(e, left, right, p, extra)
        assert np.array_equal(out, ref_c.compute(left, right, p))
        assert e.counters()["sweep_fallbacks"] == 0
        e.set_cu_mask(None)
        assert np.array_equal(_run(e, left, right, p, extra), out)
    finally:
        e.close()


@pytest.mark.parametrize("mode,cost", [(5, 0), (8, 1)], ids=["sgbm5", "census8"])
def test_sweeps_too_wide_for_the_cus_run_per_direction(mode, cost):
    """On 4 CUs a KITTI pair's strips cannot all be co-resident: the library
    runs the per-direction engine instead (same maps, no device fallback)."""
    e = _lib.Engine(0)
    try:
        e.set_cu_mask([0, 1, 2, 3])
        H, W, D = synthetic.CONFIGS["kitti"]
        left, right, _ = synthetic.random_dot_pair(H, W, D, seed=6)
        p = dict(synthetic.headline_params(D) if cost else synthetic.parity_params(D), mode=mode)
        out = _run(e, left, right, p, SWEEP8)
        assert np.array_equal(out, ref_c.compute(left, right, p))
        assert e.counters()["sweep_fallbacks"] == 0
    finally:
        e.close()


def test_full_size_sweeps_do_not_fall_back(eng):
    H, W, D = synthetic.CONFIGS["kitti"]
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=6)
    before = eng.counters()["sweep_fallbacks"]
    for p, flags in ((synthetic.parity_params(D), SWEEP8), (synthetic.headline_params(D), SWEEP8)):
        assert np.array_equal(_run(eng, left, right, p, flags), ref_c.compute(left, right, p))
    assert eng.counters()["sweep_fallbacks"] == before


@pytest.mark.parametrize("kind", ["sgbm5", "census8", "sgbm8"])
@pytest.mark.parametrize("flags", [0, PERDIR])
def test_tsukuba_config1(eng, kind, flags):
    """BASELINE config 1: 384x288, D=16."""
    H, W, D = synthetic.CONFIGS["tsukuba"]
    left, right, gt = synthetic.random_dot_pair(H, W, D, seed=2)
    p = {"sgbm5": synthetic.parity_params(D), "census8": synthetic.headline_params(D),
         "sgbm8": dict(synthetic.parity_params(D), mode=8)}[kind]
    out = _run(eng, left, right, p, flags)
    assert np.array_equal(out, ref_c.compute(left, right, p))
    if kind == "sgbm5":  # the numpy restatement agrees too (config 1's plumbing check)
        assert np.array_equal(out, sgm_np.compute(left, right, p))
    valid = out >= 0
    assert valid.mean() > 0.7
    assert np.mean(np.abs(((out.astype(np.int64) + 8) >> 4) - gt)[valid] <= 1) > 0.9


@pytest.mark.slow
def test_middlebury_full_frame_bit_exact(eng):
    """BASELINE config 3 (2880x1988, D=256, census + 8 paths) on the whole frame: the
    default engine (one pair: per-direction), the fused sweeps forced (16384: the wide D = 256
    instance with 32-lane lines, sm_sweep.hpp wide_ncw), and two pairs in one device batch
    (the default engine there: the sweeps, two pairs per launch)."""
    import torch

    H, W, D = synthetic.CONFIGS["middlebury"]
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=9)
    p = synthetic.headline_params(D)
    exp = ref_c.compute(left, right, p)
    out = _run(eng, left, right, p)
    assert np.array_equal(out, exp), f"default: {np.sum(out != exp)} px differ"
    eng.set_debug_flags(16384)
    try:
        out = _run(eng, left, right, p)
    finally:
        eng.set_debug_flags(0)
    assert np.array_equal(out, exp), f"sweeps: {np.sum(out != exp)} px differ"
    # a two-pair batch of the same pair (a second oracle run would cost another full C run)
    L = torch.tensor(np.stack([left, left]), device="cuda")
    R = torch.tensor(np.stack([right, right]), device="cuda")
    o = torch.empty((2, H, W), dtype=torch.int16, device="cuda")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.compute_batch_device(L.data_ptr(), R.data_ptr(), 2, H * W, H, W, W, synthetic.to_sm_params(p),
                                 o.data_ptr())
        got = o.cpu().numpy()
    finally:
        eng.set_stream(None)
    assert np.array_equal(got[0], exp) and np.array_equal(got[1], exp)


def test_compute_disparity_settings_ini_full_kitti():
    """The reference surface at settings.ini values (window_size 5, D=160,
    blockSize 5, lambda 80000, sigma 1.2) on a full KITTI frame: left +
    right SGBM + WLS against the C port + numpy WLS run in the reference's
    order (stereo_vision/stereo_vision.py:148-182)."""
    import stereo_match_amd as sm

    s = dict(sm.DEFAULT_SETTINGS, window_size=5)
    H, W = synthetic.CONFIGS["kitti"][:2]
    D = s["num_disparities"]
    left, right, _ = synthetic.random_dot_pair(H, W, D, seed=77)
    displ, filt = sm.compute_disparity(left, right, s)
    hp = synthetic.parity_params(D, s["window_size"])
    lp = dict(hp, uniquenessRatio=0, disp12MaxDiff=1000000)
    exp_l = ref_c.compute(left, right, lp)
    exp_r = ref_c.compute(right, left, sgm_np.right_matcher_params(hp))
    assert np.array_equal(displ, exp_l)
    wp = dict(lmbda=80000.0, sigma=1.2, radius=(s["block_size"] + 1) // 2, min_disp=0, left_offset=D, right_offset=0)
    exp_f = wls_np.wls_filter(exp_l, left, exp_r, wp)
    assert np.array_equal(filt, exp_f), f"{np.sum(filt != exp_f)} px differ"


def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def test_rccl_gather_world1():
    """batch.gather_to_root over RCCL (backend "nccl" on ROCm), world size 1:
    int16 maps moved as raw bytes through dist.gather arrive byte-identical and
    in pair order."""
    import torch
    import torch.distributed as dist

    from stereo_match_amd.batch import gather_to_root

    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        g = torch.Generator(device="cpu").manual_seed(3)
        maps = torch.randint(-32768, 32767, (5, 37, 91), dtype=torch.int16, generator=g)
        out = gather_to_root(maps.cuda(), 5)
        torch.cuda.synchronize()
        assert out.dtype == torch.int16 and out.shape == (5, 37, 91)
        assert torch.equal(out.cpu(), maps)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("D", [64, 128])
def test_valid_result_flags_leave_compute_disparity_unchanged(eng, D):
    """Every debug flag documented as 'valid results' (include/stereo_match_amd.h)
    must leave the whole compute_disparity (both matchers + WLS) bit-identical,
    e.g. no flag may double as another kernel's timing ablation."""
    import stereo_match_amd as sm
    from stereo_match_amd import wls
    from stereo_match_amd.stereo_vision import matcher_from_settings

    s = dict(sm.DEFAULT_SETTINGS, window_size=5, num_disparities=D)
    H, W = 120, 420
    gl, gr, _ = synthetic.random_dot_pair(H, W, D, seed=D + 3)
    lm = matcher_from_settings(s)
    prm = lm.params()
    wf = wls.createDisparityWLSFilter(lm)
    wf.setLambda(s["lmbda"])
    wf.setSigmaColor(s["sigma"])
    wp = wf.params(H, W)
    ref = eng.compute_disparity(gl, gr, prm, wp)
    for f in (8, 64, 128, 256, 1 << 12, 1 << 13, 1 << 14, (1 << 14) | 128, (1 << 14) | 256, (1 << 14) | (1 << 19), 1 << 15,
              1 << 19, 1 << 20, (1 << 20) | (1 << 14), 1 << 21, 1 << 22, 1 << 23, 1 << 27, 1 << 30, 2 << 16):
        if f & ABLATION_FLAGS and not ablation_build():
            continue
        eng.set_debug_flags(f)
        try:
            got = eng.compute_disparity(gl, gr, prm, wp)
        finally:
            eng.set_debug_flags(0)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), f


def test_compute_disparity_on_a_caller_stream(eng):
    """After sm_set_stream the right matcher (twin context) still forks from and joins back
    into the caller's stream, in sequence (default) and side by side (flag 1 << 20)."""
    import torch

    import stereo_match_amd as sm
    from stereo_match_amd import wls
    from stereo_match_amd.stereo_vision import matcher_from_settings

    D = 64
    s = dict(sm.DEFAULT_SETTINGS, window_size=5, num_disparities=D)
    H, W = 96, 300
    gl, gr, _ = synthetic.random_dot_pair(H, W, D, seed=11)
    lm = matcher_from_settings(s)
    prm = lm.params()
    wf = wls.createDisparityWLSFilter(lm)
    wf.setLambda(s["lmbda"])
    wf.setSigmaColor(s["sigma"])
    wp = wf.params(H, W)
    ref = eng.compute_disparity(gl, gr, prm, wp)
    st = torch.cuda.Stream()
    eng.set_stream(st.cuda_stream)
    try:
        for f in (0, 1 << 20):
            eng.set_debug_flags(f)
            got = eng.compute_disparity(gl, gr, prm, wp)
            assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), f
    finally:
        eng.set_debug_flags(0)
        eng.set_stream(None)


def test_product_library_rejects_ablation_flags(eng):
    """The product library leaves the measured ablations out (SM_ABLATIONS=0)."""
    if ablation_build():
        pytest.skip("ablation build accepts them")
    for f in (32768, 128, 1 << 27, 32, 1 << 24, 1 << 31):
        with pytest.raises(_lib.SmError):
            eng.set_debug_flags(f)
    eng.set_debug_flags(0)
