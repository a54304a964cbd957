"""Timing ablations of the WLS kernels (results are wrong under flags != 0):
1 << 28 skips the FGS sweeps, 1 << 29 skips the FGS global loads/stores."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from stereo_match_amd import _lib, synthetic
    H, W, D = synthetic.CONFIGS["kitti"]
    P = 8
    ls, rs = zip(*[synthetic.random_dot_pair(H, W, D, seed=i)[:2] for i in range(P)])
    dL = torch.tensor(np.stack(ls), device="cuda")
    dR = torch.tensor(np.stack(rs), device="cuda")
    outs = [torch.empty((P, H, W), dtype=torch.int16, device="cuda") for _ in range(3)]
    eng = _lib.Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    prm = synthetic.to_sm_params(synthetic.parity_params(D))
    wp = _lib.wls_default_params(prm)
    wp.lambda_, wp.sigma_color = 80000.0, 1.2
    eng.compute_disparity_batch_device(dL.data_ptr(), dR.data_ptr(), P, H * W, H, W, W, prm, wp,
                                       *(o.data_ptr() for o in outs))
    torch.cuda.synchronize()
    for flags in [0, 1 << 28, 1 << 29, 3 << 28, 0]:
        eng.set_debug_flags(flags)
        eng.set_timing(True)
        eng.reset_timing()
        for _ in range(3):
            eng.wls_filter_batch_device(outs[0].data_ptr(), outs[1].data_ptr(), dL.data_ptr(), P, H * W, W, H, W,
                                        wp, outs[2].data_ptr())
        t = eng.timing()
        eng.set_timing(False)
        print(json.dumps({"flags": flags, "wls_us_per_pair": t["wls"][0] * 1e3 / t["wls"][2]}), flush=True)
    eng.set_debug_flags(0)


if __name__ == "__main__":
    main()
