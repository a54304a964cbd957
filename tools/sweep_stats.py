"""Where the fused sweeps' waves wait (SWEEP_STATS variant build, tools/build_variant.sh
stats -DSWEEP_STATS=1; run with STEREO_MATCH_AMD_LIB=var/lib_stats.so): KITTI census8,
8 pairs per launch, counters of sm_sweep.hpp per mode as fractions of the waves' lives."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from stereo_match_amd import _lib, synthetic  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "census8"
H, W, D = synthetic.CONFIGS["kitti"]
p = synthetic.headline_params(D) if mode == "census8" else synthetic.parity_params(D)
if mode == "sgbm8":
    p = dict(p, mode=8)
n = 8
pairs = [synthetic.random_dot_pair(H, W, D, seed=1000 + i)[:2] for i in range(n)]
L = torch.tensor(np.stack([a for a, _ in pairs]), device="cuda")
R = torch.tensor(np.stack([b for _, b in pairs]), device="cuda")
out = torch.empty((n, H, W), dtype=torch.int16, device="cuda")
eng = _lib.Engine(0)
sp = synthetic.to_sm_params(p)
for _ in range(3):
    eng.compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, sp, out.data_ptr())
eng.synchronize()
eng.debug_fetch(20)  # clear
reps = 5
eng.set_timing(True)
eng.reset_timing()
for _ in range(reps):
    eng.compute_batch_device(L.data_ptr(), R.data_ptr(), n, H * W, H, W, W, sp, out.data_ptr())
eng.synchronize()
raw = np.frombuffer(eng.debug_fetch(20), np.uint64).reshape(6, 8)
st = raw.astype(np.float64)
print({k: round(v[0] * 1e3 / max(v[2], 1), 1) for k, v in eng.timing().items() if v[1]})
ln = st[5]
if ln[4]:  # MODE 3's line waves (words 40..44)
    own_life = st[3][4]
    print(f"mode 3 lines: {int(ln[4])} line waves, life {ln[3] / ln[4] / reps:.0f} cyc/launch; wait_cons "
          f"{ln[1] / ln[3]:.3f}, barriers {ln[2] / ln[3]:.3f}; own waves in wait_lines {ln[0] / max(own_life, 1):.3f}")
for m in range(5):
    s = st[m]
    if s[5] == 0:
        continue
    print(f"mode {m}: compute waves {int(s[5])}, life {s[4] / s[5] / reps:.0f} cyc/launch; wait_row "
          f"{s[2] / s[4]:.3f}, block barriers {s[3] / s[4]:.3f}; poller life {s[6] / reps:.0f} total, "
          f"polls {s[0] / max(s[6], 1):.3f}, barriers {s[1] / max(s[6], 1):.3f}; "
          f"workgroups on XCC (linear id % 8): {int(raw[m][7]) & 0xFFFFFFFF} of {int(raw[m][7]) >> 32}")

x = np.frombuffer(eng.debug_fetch(21), np.uint8)
ids = [int(v) & 15 for v in x if v & 0x80]
print("XCC by linear workgroup id (first 80):", ids[:80])
print("count per XCC:", np.bincount(ids, minlength=8).tolist())

# hand-off latency: snapshot publish (producer) -> observed by the neighbour's poller
ts = np.frombuffer(eng.debug_fetch(22), np.uint64).reshape(2, 3, 65536).astype(np.int64)
nblk = -(-H // 4)
for m in range(3):
    pub, obs = ts[0, m], ts[1, m]
    ok = (pub > 0) & (obs > 0)
    if not ok.any():
        continue
    lat = (obs[ok] - pub[ok]) * 10  # s_memrealtime: 100 MHz
    P = pub[: (len(pub) // nblk) * nblk].reshape(-1, nblk)
    per = np.diff(P[(P > 0).all(1)], axis=1).ravel() * 10
    print(f"mode {m}: hand-off latency ns p10/50/90 {np.percentile(lat, [10, 50, 90]).round().tolist()} "
          f"(n={ok.sum()}); block period ns p50 {np.percentile(per, 50) if per.size else None}")
