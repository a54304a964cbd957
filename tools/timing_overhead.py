"""Wall time per call of the headline batch with the engine's stage timers on and off
(interleaved rounds in one process)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from stereo_match_amd import _lib, synthetic
    mode = sys.argv[1] if len(sys.argv) > 1 else "census8"
    H, W, D = synthetic.CONFIGS["kitti"]
    p = synthetic.headline_params(D) if mode == "census8" else synthetic.parity_params(D)
    prm = synthetic.to_sm_params(p)
    P = 8
    ls, rs = zip(*[synthetic.random_dot_pair(H, W, D, seed=i)[:2] for i in range(P)])
    dL = torch.tensor(np.stack(ls), device="cuda")
    dR = torch.tensor(np.stack(rs), device="cuda")
    out = torch.empty((P, H, W), dtype=torch.int16, device="cuda")
    eng = _lib.Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)

    def run(n):
        for _ in range(n):
            eng.compute_batch_device(dL.data_ptr(), dR.data_ptr(), P, H * W, H, W, W, prm, out.data_ptr())

    run(10)
    torch.cuda.synchronize()
    res = {True: [], False: []}
    for _ in range(4):
        for timing in (False, True):
            eng.set_timing(timing)
            eng.reset_timing()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(100)
            torch.cuda.synchronize()
            res[timing].append((time.perf_counter() - t0) / 100 / P * 1e6)
            if timing:
                eng.timing()
            eng.set_timing(False)
    for k, v in res.items():
        print(f"timing={k}: us per pair {np.median(v):.1f} ({', '.join(f'{x:.1f}' for x in v)})")


if __name__ == "__main__":
    main()
