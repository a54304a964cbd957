"""Repeatability diagnostic for compute_disparity: runs the batch-device call N times and
reports, per call, which of displ / dispr / filtered differ from the oracle chain (and
the WLS filter alone on fixed maps).  Test tooling (imports oracle/)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import stereo_match_amd as sm  # noqa: E402
from oracle import ref_c, sgm_np, wls_np  # noqa: E402
from stereo_match_amd import _lib, synthetic, wls  # noqa: E402
from stereo_match_amd.stereo_vision import matcher_from_settings  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
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
    L = torch.tensor(gl, device="cuda")
    R = torch.tensor(gr, device="cuda")
    dl = torch.empty((H, W), dtype=torch.int16, device="cuda")
    dr = torch.empty_like(dl)
    fo = torch.empty_like(dl)
    outs = []
    for i in range(N):
        eng.compute_disparity_batch_device(L.data_ptr(), R.data_ptr(), 1, H * W, H, W, W, prm, wp, dl.data_ptr(),
                                           dr.data_ptr(), fo.data_ptr())
        eng.synchronize()
        outs.append((dl.cpu().numpy(), dr.cpu().numpy(), fo.cpu().numpy()))
    # WLS alone on the first call's maps
    wl = []
    for i in range(N):
        wl.append(eng.wls_filter(outs[0][0], gl, outs[0][1], wp))
    a0 = outs[0]
    for i, o in enumerate(outs):
        print(f"D={D} call {i}: displ {int((o[0] != a0[0]).sum())} dispr {int((o[1] != a0[1]).sum())} "
              f"filt {int((o[2] != a0[2]).sum())} px differ from call 0; "
              f"wls-only {int((wl[i] != wl[0]).sum())}; wls-only vs fused {int((wl[i] != o[2]).sum())}", flush=True)
    eng.close()
