#!/usr/bin/env python3
"""Benchmark: stereo pairs/s (+ Mpix·disp/s) on the BASELINE.json headline
workload — KITTI 1242×375, D=128, Census 9×7 + 8-path SGM, WTA + uniqueness
+ sub-pixel + left/right check + 3×3 median — on 1..8 MI355X, one process per
GPU.

``python bench.py --gpus N`` with N > 1 and no ``WORLD_SIZE`` in the
environment starts ``torch.distributed.run`` with N ranks as a CHILD process
(nothing here touches the GPU before that) and exits with its status; the
driver's own ``torch.distributed.run ... bench.py --gpus N`` lands directly in
the per-rank path.  ``--gpus`` must equal the world size.

A step = every rank runs the hot path over its block of ``--pairs-per-gpu``
synthetic pairs (``batch.shard_range`` of the global batch) already resident
in HBM, then (N > 1) the int16 disparity maps are gathered to rank 0 over
RCCL/xGMI (BASELINE config 4).  Weak scaling: per-GPU work is fixed as N
grows.  Timed region: barrier + device sync on both sides, K steps, max over
ranks; the gather's share is timed separately with events on the same stream.

Prints ONE JSON line on rank 0 (DESIGN.md §6 lists every field).  The
roofline figure follows SURVEY.md §8(d): the model's bytes attributable to
the dominant kernel (see ``model_stage_bytes``) over that kernel's average
launch time; the engine's own bytes are reported beside it.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "stereo pairs/sec + Mpix·disp/sec, KITTI 1242×375 D=128 SGM, 1/2/4/8 GPU"  # BASELINE.json metric
CONFIG_NAMES = {"tsukuba": "Tsukuba", "kitti": "KITTI", "middlebury": "Middlebury-v3 full-res",
                "mccnn": "KITTI-size mc-cnn cost volume"}


def metric_for(config: str) -> str:
    """BASELINE.json's metric string for its headline config (KITTI); the same
    wording with the workload named for the other configs."""
    if config == "kitti":
        return METRIC
    from stereo_match_amd import synthetic

    H, W, D = synthetic.CONFIGS[config]
    return f"stereo pairs/sec + Mpix·disp/sec, {CONFIG_NAMES[config]} {W}×{H} D={D} SGM, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=None, choices=["kitti", "middlebury", "tsukuba", "mccnn"],
                    help="default: kitti (mccnn for --mode volume8)")
    ap.add_argument("--mode", default="census8", choices=["census8", "sgbm5", "sgbm8", "volume8", "disparity5", "bm"],
                    help="census8 = headline; sgbm5 = OpenCV parity mode; sgbm8 = OpenCV cost + 8 paths; "
                         "volume8 = mc-cnn f32 cost volume; "
                         "disparity5 = the reference's whole compute_disparity (left + right SGBM + WLS); "
                         "bm = StereoBM(numDisparities=D, blockSize=21), the method='BM' matcher")
    ap.add_argument("--pairs-per-gpu", type=int, default=8)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group (RCCL on the GPU) and run the gather even at world size 1, "
                         "so the multi-rank code path runs on one GPU")
    ap.add_argument("--engine", default="auto", choices=["auto", "perdir", "sweep"],
                    help="auto: the library's default per configuration; perdir / sweep force one engine "
                         "(DESIGN.md §4)")
    ap.add_argument("--debug-flags", type=int, default=0,
                    help="sm_set_debug_flags value OR-ed into the engine flags (engine selection for A/B runs; "
                         "ablation-only flags need STEREO_MATCH_AMD_LIB=.../libstereo_match_amd_ablate.so)")
    ap.add_argument("--tune", default="",
                    help="launch-shape knobs for A/B measurements, e.g. ew_waves=1,ew_lanes=16 "
                         "(sm_set_tuning; every value gives the same disparities)")
    ap.add_argument("--cpu-baseline-pairs", type=int, default=8,
                    help="pairs timed on the host C port per thread (rank 0, N=1 only); 0 = skip")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the multi-core CPU baseline; 0 = the process's CPU share "
                         "(cpu_share(): OMP_NUM_THREADS where the pool sets it, else the affinity mask)")
    ap.add_argument("--host-surface-calls", type=int, default=20,
                    help="rank 0, N=1: timed calls of the reference surface compute_disparity (host numpy in/out, "
                         "settings.ini, KITTI size); 0 = skip")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    ap.add_argument("--valu-file", default=os.path.join(ROOT, "profiles", "valu_latest.json"))
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="rank-path self-test: main's own sharding / timing / gather / JSON code over gloo on CPU with "
                         "a stand-in step (no disparity computed, not a measurement)")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# launcher
# ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Run this script under torch.distributed.run with n ranks (a child
    process: the parent never initialises the GPU and never execs)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def source_hash() -> str:
    """Hash of the kernel + C-ABI sources (stamps PMC traffic files)."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "stereo_match_amd", "csrc", "*.hip"))
                   + glob.glob(os.path.join(ROOT, "stereo_match_amd", "csrc", "*.hpp"))
                   + glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def kernel_stage(name: str, names) -> "str | None":
    """The engine stage (sm_set_timing's names) a profiled kernel belongs to; ``names`` are
    all kernels of the profiled run (they tell the engine apart).  Shared by
    tools/traffic_summary.py and tools/valu_summary.py, which sum a stage's kernels."""
    targs = [t.strip() for t in name.split("<", 1)[1].split(">")[0].split(",")] if "<" in name else []
    sweep_modes = set()
    for n in names:
        if "k_sweep<" in n:
            sweep_modes.add([t.strip() for t in n.split("<", 1)[1].split(">")[0].split(",")][3])
    sweep = bool(sweep_modes) or any("k_sweep2<" in n for n in names)
    lines5 = "3" in sweep_modes and "4" not in sweep_modes  # in-sweep E/W lines, 5 paths: k_wta reads the partial
    # the guarded fallback instances (run only when a strip gave up): k_sgm_paths<..., FB>,
    # k_wta<DPL, LT, NT, FB, PART_ONLY>
    if "k_sgm_paths" in name and targs and targs[-1] == "true":
        return None
    if "k_wta<" in name and len(targs) >= 4 and targs[3] == "true":
        return None
    if "k_sweep2<" in name or "k_sweep<" in name:  # MODE 0 / 3: down sweep -> partial; 1 / 2 / 4: with WTA
        return "sweep" if targs[4 if "k_sweep2<" in name else 3] in ("0", "3") else "sweep_wta"
    if "k_ew_patch" in name or "k_ew<" in name or (sweep and "k_sgm_paths" in name):
        return "horizontal"
    if "k_sgm_paths" in name:
        return "paths"
    if "k_wta" in name or "k_row_wta" in name:
        return "sweep_wta" if lines5 else "wta"
    if "k_lr_rows" in name:
        return "wta"
    if any(c in name for c in ("k_census9x7", "k_census_cost8", "k_sgbm_prefilter", "k_sgbm_cost", "k_cost_volume_f32",
                               "k_vol_")):
        return "cost"
    return None


# ---------------------------------------------------------------------------
# SURVEY.md §8(d) byte model, attributed to the engine's stages
# ---------------------------------------------------------------------------
def model_pair_bytes(mode: str, H: int, W: int, D: int, P: int) -> int:
    """§8(d) algorithmic bytes per pair (per matcher call).  volume8: the bytes an engine must
    move for an f32 volume (read once, 4 B; the quantised u16 volume written, 2 B, and read
    per path, 2 B; S written and read, 4 B), not §8(d)'s 4 B per path, which credits f32
    re-reads no engine makes (round-4 verdict: a frac above 1)."""
    cells = H * W * D
    if mode == "volume8":
        return cells * (4 + 2 + 2 * P + 4)
    if mode == "bm":
        return H * W * (2 + 2 * 2 + 2 + 4)
    return cells * (1 + P + 4) + 2 * H * W + 2 * H * W * 2


def model_stage_bytes(stage: str, mode: str, H: int, W: int, D: int, P: int, sweep: bool, lines: bool = False) -> int:
    """Share of ``model_pair_bytes`` owned by one engine stage, per pair.

    Model terms per cell: cost volume written once (1 B; f32 volume read once,
    4 B), read once per path (P x 1 B; 4 B for f32), S written once and read
    once (2 + 2 B); per pixel: 2 images in (2 B), 2 int16 maps out (4 B).
    A stage owns the terms of the work it does: the cost stage the volume
    write and the image reads; each aggregation kernel the reads of the paths
    it aggregates (+ the S write when it completes S); the WTA stage the S
    read and the outputs.  Summed over the stages this is exactly
    ``model_pair_bytes``.  With the in-sweep E/W lines (``lines``) the down sweep aggregates
    five paths (S, SE, SW, E, W; at 5 paths it completes S), the patch pass owns no model
    bytes, and the WTA stage is the up sweep (8 paths) or the WTA kernel over S (5 paths).
    """
    cells, px = H * W * D, H * W
    if mode == "bm":
        return model_pair_bytes(mode, H, W, D, P) if stage in ("wta", "paths") else 0
    vol = mode == "volume8"
    cw, r = (4 + 2, 2) if vol else (1, 1)  # volume8: f32 read + u16 written; paths read u16
    io_in, io_out = (0, 0) if vol else (2, 4)
    if stage == "cost":
        return cells * cw + px * io_in
    if not sweep:
        if stage == "paths":
            return cells * (P * r + 2)
        if stage == "wta":
            return cells * 2 + px * io_out
        return 0
    if lines:  # down sweep with E/W lines -> partial; patch; up sweep + WTA (8) / WTA over S (5)
        if stage == "sweep":
            return cells * 5 * r + (cells * 2 if P == 5 else 0)
        if stage == "sweep_wta":
            return (cells * (3 * r + 2 + 2) if P == 8 else cells * 2) + px * io_out
        return 0
    # fused-sweep engine: E/W lines, [down sweep S+SE+SW -> partial], last sweep (+ S write/read) + WTA
    if stage == "horizontal":
        return cells * 2 * r
    if stage == "sweep":
        return cells * 3 * r if P == 8 else 0
    if stage == "sweep_wta":
        return cells * (3 * r + 2 + 2) + px * io_out
    return 0


# ---------------------------------------------------------------------------
# the rank path: one process per GPU (or a gloo stand-in on CPU)
# ---------------------------------------------------------------------------
class GpuWorkload:
    """The hot path on this rank's GPU: its block of synthetic pairs resident in
    HBM, one ``step`` = one engine call over the block (census8: cost, E/W and
    the two fused sweeps, LR check, median)."""

    backend = "nccl"

    def __init__(self, args, local_rank):
        import torch

        from stereo_match_amd import _lib, synthetic

        self.args, self.torch, self._lib, self.synthetic = args, torch, _lib, synthetic
        self.dev = torch.device("cuda", local_rank)
        torch.cuda.set_device(self.dev)
        self.local_rank = local_rank
        self.H, self.W, self.D = synthetic.CONFIGS[args.config]
        self.volume = args.mode == "volume8"
        self.full = args.mode == "disparity5"
        self.bm = args.mode == "bm"
        if args.mode == "census8":
            p = synthetic.headline_params(self.D)
        elif self.volume:
            p = synthetic.cost_volume_params(self.D)
        else:
            p = synthetic.parity_params(self.D)
            if args.mode == "sgbm8":  # OpenCV cost, 8 paths (MODE_HH)
                p = dict(p, mode=8)
        self.p = p
        self.prm = synthetic.to_sm_params(p)
        if self.bm:
            self.prm = _lib.SmBmParams()
            _lib.load().sm_bm_default_params(self.D, 21, self.prm)

    def init_dist(self):
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=self.dev)

    def setup(self, first, P):
        # the reference's own surface (one pair per call) is measured first, on a device that has
        # not just run the batch workload: the state a one-pair caller sees (after the 8-pair
        # bench the same calls measured 12 % slower on one box: 1.09 vs 0.97 ms)
        self.hs = None
        if (int(os.environ.get("WORLD_SIZE", "1")) == 1 and self.args.host_surface_calls > 0
                and self.args.config == "kitti"):
            self.hs = host_surface(self.args, self.local_rank)

        torch, synthetic, _lib = self.torch, self.synthetic, self._lib
        H, W, D, dev = self.H, self.W, self.D, self.dev
        self.P = P
        # synthetic inputs for this rank's block of pairs, resident in HBM before timing
        self.lefts, self.rights = [], []
        for i in range(first, first + P):
            l, r, _ = synthetic.random_dot_pair(H, W, D, seed=1000 + i)
            self.lefts.append(l)
            self.rights.append(r)
        self.dL = torch.tensor(np.stack(self.lefts), device=dev)
        self.dR = torch.tensor(np.stack(self.rights), device=dev)
        self.out = torch.empty((P, H, W), dtype=torch.int16, device=dev)
        self.dOutR = self.dFilt = self.wprm = None
        if self.full:  # compute_disparity: settings.ini lambda/sigma, createDisparityWLSFilter defaults
            self.dOutR = torch.empty_like(self.out)
            self.dFilt = torch.empty_like(self.out)
            self.wprm = _lib.wls_default_params(self.prm)
            self.wprm.lambda_, self.wprm.sigma_color = 80000.0, 1.2
        self.vols = None
        if self.volume:  # config C: (1, D, H, W) float32 cost per pair, resident in HBM
            self.vols = torch.empty((P, D, H, W), dtype=torch.float32, device=dev)
            for i in range(P):
                self.vols[i].copy_(torch.from_numpy(synthetic.absdiff_volume(self.lefts[i], self.rights[i], D)[0]))
        self.eng = _lib.Engine(self.local_rank)
        self.stream = torch.cuda.current_stream(dev)
        self.eng.set_stream(self.stream.cuda_stream)
        flags = {"auto": 0, "perdir": 4096, "sweep": 16384}[self.args.engine] | self.args.debug_flags
        if flags:
            self.eng.set_debug_flags(flags)
        for kv in filter(None, self.args.tune.split(",")):
            k, v = kv.split("=")
            self.eng.set_tuning(getattr(self.eng, "TUNE_" + k.upper()), int(v))

    def step(self, out=None):
        """One engine call over the block into ``out`` ([P, H, W] int16 on this GPU; default
        self.out; the overlapped gather hands in its double buffers)."""
        e, P, H, W, prm = self.eng, self.P, self.H, self.W, self.prm
        o = (self.out if out is None else out).data_ptr()
        if self.full:
            e.compute_disparity_batch_device(self.dL.data_ptr(), self.dR.data_ptr(), P, H * W, H, W, W, prm, self.wprm,
                                             o, self.dOutR.data_ptr(), self.dFilt.data_ptr())
        elif self.bm:
            e.bm_compute_batch_device(self.dL.data_ptr(), self.dR.data_ptr(), P, H * W, H, W, W, prm, o)
        elif self.volume:
            e.aggregate_cost_f32_device(self.vols.data_ptr(), P, self.D * H * W, self.D, H, W, prm, 0.0,
                                        self.synthetic.VOLUME_SCALE, o)
        else:
            e.compute_batch_device(self.dL.data_ptr(), self.dR.data_ptr(), P, H * W, H, W, W, prm, o)

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def marker(self):
        ev = self.torch.cuda.Event(enable_timing=True)
        ev.record(self.stream)
        return ev

    @staticmethod
    def span_ms(a, b):
        return a.elapsed_time(b)

    def reduce_tensor(self, vals):
        return self.torch.tensor(vals, device=self.dev, dtype=self.torch.float64)

    # untimed warmup; its second half (at least one step) with every stage timed: the per-stage
    # profile (stage_us_per_pair) and the choice of the dominant kernel come from it (the first
    # steps allocate the engine's buffers)
    def profile_begin(self):
        self.eng.synchronize()
        self.eng.set_timing(True)
        self.eng.reset_timing()
        self._c0 = self.eng.counters()

    def profile_end(self, n_prof):
        self.eng.synchronize()  # device-side failures (sweep hand-off timeouts) fail the run here
        self.sync()
        self.n_prof = n_prof
        self.profile = self.eng.timing()
        args = self.args
        self.sweep = self.profile["sweep_wta"][1] > 0  # fused-sweep engine ran (its stages have launches)
        # ... with the horizontal paths inside the down sweep (sm_get_counter SM_COUNTER_LINE_GROUPS)
        self.lines = self.sweep and self.eng.counters()["line_groups"] > self._c0["line_groups"]
        self.P_dirs = 5 if args.mode in ("sgbm5", "disparity5") else 8
        # strips per pair of the lines engine (SM_COUNTER_LINE_STRIPS over the profiled pairs)
        c1 = self.eng.counters()
        self.strips = (c1["line_strips"] - self._c0["line_strips"]) / max(1, n_prof * self.P) if self.lines else 0
        self.kern, cands = design_kernels(args, self.profile, self.H, self.W, self.D, self.p, self.P_dirs, self.sweep,
                                          self.bm, self.lines, self.strips)
        self.cands = cands
        # the dominant kernel is fixed per engine (the stage that moves the most bytes by design:
        # the WTA sweep, the per-direction path kernel), not picked by a timing race between
        # stages a few percent apart; every stage's own fraction is reported beside it
        self.dom = max(cands, key=lambda k: (self.kern[k][1], -cands.index(k)))

    def stage_fracs(self):
        """Every aggregation / WTA stage's own roofline fraction from the warmup profile (all
        stages timed there): SURVEY §8(d) bytes the stage owns per launch / its launch time."""
        out = {}
        for k in self.cands:
            ms, launches, pairs = self.profile[k]
            if launches <= 0:
                continue
            launch_s = ms / 1e3 / launches
            ppl = pairs / launches
            alg = model_stage_bytes(k, self.args.mode, self.H, self.W, self.D, self.P_dirs, self.sweep,
                                    self.lines) * ppl
            out[k] = {"kernel": self.kern[k][0], "avg_launch_us": launch_s * 1e6, "alg_bytes_per_launch": alg,
                      "frac": alg / launch_s / 1e9 / HBM_PEAK_GBS if launch_s > 0 else None,
                      "design_bytes_per_launch": self.kern[k][1] * ppl, "source": "warmup profile"}
        return out

    def timed_begin(self):
        # timed region: only the dominant kernel's stage records events (every timed stage
        # delays the stream, about 12 us per KITTI pair with all of them: include/stereo_match_amd.h)
        self.eng.set_timing(True, stages=[self.dom])
        self.eng.reset_timing()
        self._ct0 = self.eng.counters()

    def timed_end(self):
        self.eng.synchronize()
        self.stages = self.eng.timing()
        self.eng.set_timing(False)
        c1 = self.eng.counters()
        self.timed_counters = {k: c1[k] - self._ct0[k] for k in c1}

    def report(self, elapsed, K, gpairs, world):
        """The bench line's workload-specific fields (rank 0)."""
        args, H, W, D, P = self.args, self.H, self.W, self.D, self.P
        out0 = self.out[0].cpu().numpy()
        cells = H * W * D
        dom, kern, sweep, P_dirs = self.dom, self.kern, self.sweep, self.P_dirs
        dom_ms, dom_launches, dom_pairs = self.stages[dom]
        launch_s = dom_ms / 1e3 / max(dom_launches, 1)
        pairs_per_launch = dom_pairs / max(dom_launches, 1)
        alg_bytes = model_stage_bytes(dom, args.mode, H, W, D, P_dirs, sweep, self.lines) * pairs_per_launch
        design_bytes = kern[dom][1] * pairs_per_launch
        achieved = alg_bytes / launch_s / 1e9 if launch_s > 0 else None
        traffic, traffic_note = read_traffic(args, dom, kern[dom][0], pairs_per_launch, sweep)
        valu = read_valu(args, dom, pairs_per_launch, sweep, launch_s, H, W, D)
        survey_bytes = model_pair_bytes(args.mode, H, W, D, P_dirs) * (2 if self.full else 1)
        # this rank's wall time per pair over the timed region (every call's device work and
        # the gaps between its kernels; per reference pair in disparity5: 2 matchers + WLS)
        pair_s = elapsed / max(K * P, 1)
        line = {
            "dtype": {"census8": "u8", "sgbm5": "i16", "sgbm8": "i16", "volume8": "f32->u16", "disparity5": "i16+f32",
                      "bm": "i32"}[args.mode],
            "data": "synthetic random-dot pairs (no dataset in the image)"
                    + ("; f32 cost = 3x3-smoothed |L-R|/255 volume per pair" if self.volume else ""),
            # the timed region's engine counters: launch groups the guarded fallback recomputed,
            # in-sweep E/W segments the patch pass repaired (sm_get_counter)
            "counters": dict(self.timed_counters, ew_repairs_per_pair=self.timed_counters["ew_repairs"] / max(K * P, 1)),
            "config": {
                "engine": ("fused sweeps, E/W lines in the down sweep" if self.lines else "fused sweeps") if sweep
                          else "per-direction",
                "workload": f"{args.config} {W}x{H} D={D} "
                            + {"census8": "census9x7 + 8-path SGM", "sgbm5": "OpenCV-SGBM 5-path",
                               "sgbm8": "OpenCV-SGBM 8-path (MODE_HH)",
                               "volume8": "f32 cost volume (mc-cnn) + 8-path SGM",
                               "disparity5": "compute_disparity: left+right OpenCV-SGBM 5-path + WLS",
                               "bm": "OpenCV StereoBM blockSize 21 (X-Sobel prefilter)"}[args.mode],
                **({"tune": args.tune} if args.tune else {}),
            },
            "mpix_disp_per_s": gpairs * K / elapsed * cells / 1e6,
            "roofline": {
                "kernel": kern[dom][0],
                **(valu_roofline(valu, launch_s) if self.bm else hbm_roofline(achieved, valu)),
                "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes,
                "alg_model": "SURVEY §8d bytes owned by this stage (bench.model_stage_bytes)",
                "design_bytes_per_launch": design_bytes,
                "design_achieved_GBs": design_bytes / launch_s / 1e9 if launch_s > 0 else None,
                "traffic_over_alg": (traffic / alg_bytes) if traffic and alg_bytes else None,
                "traffic_note": traffic_note,
                "valu": valu,
                "pairs_per_launch": pairs_per_launch,
                "avg_launch_us": launch_s * 1e6,
                "dominant_rule": "fixed per engine: the stage with the most design bytes (fused sweeps: the WTA "
                                 "sweep; with the in-sweep E/W lines: the down sweep with its line waves; "
                                 "per-direction: the path kernel)",
                "stages": self.stage_fracs(),
            },
            "pipeline_roofline": {
                "model": "SURVEY §8d " + ("H·W·D·(4+2+2P+4) (f32 read once)" if self.volume
                                          else "H·W·(2+4+2+4) (no volume)" if self.bm
                                          else "H·W·D·(1+P+4)+I/O")
                         + (" x2 matchers" if self.full else "") + " per pair",
                "bytes_per_pair": survey_bytes,
                "wall_us_per_pair": pair_s * 1e6,
                "achieved_GBs": survey_bytes / pair_s / 1e9 if pair_s > 0 else None,
                # StereoBM streams no cost volume: its few bytes per pixel against HBM say nothing
                # (its ceiling is VALU issue, roofline.valu)
                "frac": None if self.bm else survey_bytes / pair_s / 1e9 / HBM_PEAK_GBS if pair_s > 0 else None,
                **({"frac_note": "none for StereoBM: no cost volume; VALU-bound (roofline)"} if self.bm else {}),
            },
            "stage_us_per_pair": {k: v[0] * 1e3 / max(v[2], 1) for k, v in self.profile.items()},
            "stage_profile": f"last {self.n_prof} warmup steps, every stage timed; the timed region times only "
                             f"the dominant kernel's stage",
            "valid_frac_pair0": float((out0 >= 0).mean()),
        }
        hs_pair = None
        if world == 1 and self.hs is not None:
            line["host_surface"], hs_pair = self.hs
        if world == 1 and args.cpu_baseline_pairs > 0:
            line["cpu_baseline"] = cpu_baseline(args, H, W, D, self.p, self.lefts, self.rights, out0, self.volume,
                                                self.full, hs_pair)
        return line


class StandInWorkload:
    """CPU stand-in for ``GpuWorkload`` (--selftest-cpu): the same rank path over
    gloo; the step widens the left images to int16 x16 (no disparity computed),
    so the gathered maps are known per pair index.  Not a measurement."""

    backend = "gloo"

    def __init__(self, args, local_rank):
        import torch

        from stereo_match_amd import synthetic

        self.torch, self.args = torch, args
        self.H, self.W, self.D = synthetic.CONFIGS[args.config]

    def init_dist(self):
        import torch.distributed as dist

        dist.init_process_group("gloo")

    def setup(self, first, P):
        torch = self.torch
        self.P = P
        self.dL = torch.stack([torch.full((self.H, self.W), i % 251, dtype=torch.uint8)
                               for i in range(first, first + P)]) if P else \
            torch.empty((0, self.H, self.W), dtype=torch.uint8)
        self.out = torch.empty((P, self.H, self.W), dtype=torch.int16)

    def expected(self, gpairs):
        torch = self.torch
        return torch.stack([torch.full((self.H, self.W), (i % 251) * 16, dtype=torch.int16) for i in range(gpairs)])

    def step(self, out=None):
        (self.out if out is None else out).copy_(self.dL.to(self.torch.int16) * 16)

    def sync(self):
        pass

    def marker(self):
        return time.perf_counter()

    @staticmethod
    def span_ms(a, b):
        return (b - a) * 1e3

    def reduce_tensor(self, vals):
        return self.torch.tensor(vals, dtype=self.torch.float64)

    def profile_begin(self):
        pass

    def profile_end(self, n_prof):
        pass

    def timed_begin(self):
        pass

    def timed_end(self):
        pass

    def report(self, elapsed, K, gpairs, world):
        return {"value": None, "dtype": None,
                "data": "rank-path self-test: gloo on CPU, stand-in step (no disparity computed, not a measurement)",
                "config": {"engine": "stand-in"}}


def main():
    args = parse()
    if args.config is None:
        args.config = "mccnn" if args.mode == "volume8" else "kitti"
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch N ranks for --gpus N)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    wl = (StandInWorkload if args.selftest_cpu else GpuWorkload)(args, local_rank)
    run_rank(args, wl, world, rank)


def run_rank(args, wl, world, rank):
    """One rank: shard, warm up, time K steps between barriers + device syncs,
    max over ranks, gather to rank 0, print the JSON line on rank 0.  The same
    code for the GPU workload and the CPU stand-in (--selftest-cpu)."""
    import torch
    import torch.distributed as dist

    from stereo_match_amd.batch import OverlappedGather, gather_to_root, shard_range

    dist_on = world > 1 or args.dist
    if dist_on:
        if world == 1 and "MASTER_ADDR" not in os.environ:  # --dist without a launcher: a one-rank group
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
        wl.init_dist()
    gpairs = args.pairs_per_gpu * world
    first, P = shard_range(gpairs, rank, world)
    wl.setup(first, P)
    gather = dist_on and not args.no_gather
    # step k computes into one of two buffers while step k-1's maps travel to rank 0 (rank 0
    # computes straight into its rows of the [gpairs, H, W] result: no concatenation)
    og = OverlappedGather(gpairs, P, wl.H, wl.W, torch.int16, wl.out.device) if gather else None
    nstep = [0]

    def step():
        k = nstep[0]
        nstep[0] += 1
        if og is None:
            wl.step()
            return
        wl.step(og.buffer(k))
        og.launch(k)

    n_prof = max(1, args.warmup // 2)
    for _ in range(args.warmup - n_prof):
        step()
    wl.profile_begin()
    for _ in range(n_prof):
        step()
    if og is not None:
        og.drain()
    wl.profile_end(n_prof)
    wl.timed_begin()
    if og is not None:
        og.reset_stats(timing=True)
    if dist_on:
        dist.barrier()
    wl.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if og is not None:
        og.drain()  # the last step's maps have reached rank 0 inside the timed region
    wl.sync()
    if dist_on:
        dist.barrier()
    t1 = time.perf_counter()
    wl.timed_end()
    elapsed = t1 - t0
    gather_ms = gather_exposed_ms = 0.0
    if og is not None:
        gather_ms, gather_exposed_ms = og.transfer_ms(), og.exposed_ms()
        og.reset_stats(timing=False)
    gather_ms_max, gather_exposed_max = gather_ms, gather_exposed_ms
    if dist_on:
        t = wl.reduce_tensor([elapsed, gather_ms, gather_exposed_ms])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, gather_ms_max, gather_exposed_max = float(t[0].item()), float(t[1].item()), float(t[2].item())
    gather_check = None
    if gather:  # untimed: one more overlapped step; check the maps arrived in pair order
        kf = nstep[0]
        step()
        og.drain()
        wl.step()  # the same block into wl.out (deterministic: equal to what was sent)
        wl.sync()
        # per-pair checksums (int64 -> 4 int16 words) travel to rank 0 too, so it checks every
        # rank's block, not only its own
        sums = wl.out.reshape(P, -1).to(torch.int64).sum(1).contiguous()
        gsums = gather_to_root(sums.view(torch.int16).view(P, 1, 4), gpairs)
        if rank == 0:
            gathered = og.result(kf)
            want = gathered.reshape(gpairs, -1).to(torch.int64).sum(1)
            gather_check = bool(torch.equal(gsums.reshape(gpairs, 4).contiguous().view(torch.int64).reshape(-1), want)
                                and torch.equal(gathered[first:first + P], wl.out))
            if isinstance(wl, StandInWorkload):
                gather_check = gather_check and bool(torch.equal(gathered, wl.expected(gpairs)))
    if rank == 0:
        K = args.steps
        line = {
            "metric": metric_for(args.config),
            "value": gpairs * K / elapsed,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
        }
        extra = wl.report(elapsed, K, gpairs, world)
        cfg = extra.pop("config", {})
        line.update(extra)
        line["config"] = dict(cfg, pairs_per_gpu=args.pairs_per_gpu, global_batch=gpairs, H=wl.H, W=wl.W, D=wl.D,
                              gather=gather, parallelism=f"pairs/dp{world}")
        if dist_on:
            line["distributed"] = {
                "backend": dist.get_backend(), "world_size": dist.get_world_size(),
                "gather": "point-to-point into rank 0's preallocated [pairs,H,W] maps (rank 0 computes into its "
                          "rows), double-buffered: step k's transfers on a side stream beside step k+1's compute",
                # the transfers' own duration on the side stream (rank 0: all receives of a step)
                "gather_ms_per_step_rank0": gather_ms / K, "gather_ms_per_step_max": gather_ms_max / K,
                # the part compute did not hide: the caller's stream waiting for a gather (incl. the drain)
                "gather_exposed_ms_per_step": gather_exposed_ms / K,
                "gather_exposed_ms_per_step_max": gather_exposed_max / K,
                "gather_bytes_to_root": (gpairs - P) * wl.H * wl.W * 2 if gather else 0,
                "gathered_in_pair_order": gather_check,
                "compute_ms_per_step": (elapsed * 1e3 - gather_exposed_max) / K,
            }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


def design_kernels(args, stages, H, W, D, p, P_dirs, sweep, bm, lines=False, strips=0):
    """The engine's own bytes per pair for each timed stage (what the kernels
    move by design), and the stages that can be the dominant kernel."""
    width1 = W - D  # minDisparity 0
    vol = H * width1 * D
    eb = 1 if args.mode == "census8" else 2  # bytes per path element
    if bm:  # SAD kernel reads the two prefiltered views, writes disparity (+ int32 cost)
        return {"paths": ("k_bm_sad (column sums in LDS + WTA)", H * W * (2 + 2 + 4)),
                "wta": ("k_bm_sad (column sums in LDS + WTA)", H * W * (2 + 2 + 4))}, ("wta",)
    if sweep and lines:
        rec_b = 8 * H * width1
        # boundary states of the E/W segments: 2 directions x (entering, far end) per strip and row
        # (strips per pair from SM_COUNTER_LINE_STRIPS; 36-column strips when not reported)
        st = 4 * D * eb * H * (round(strips) if strips else (width1 + 35) // 36)
        kern = {"sweep": ("k_sweep MODE 3 (S+SE+SW + in-kernel E/W lines -> partial)", vol * eb + 2 * vol + st),
                "horizontal": ("k_ew_patch (segment check + repairs)", st),
                "sweep_wta": ("k_sweep MODE 4 (N+NE+NW + partial + WTA)", vol * eb + 2 * vol + rec_b) if P_dirs == 8
                else ("k_wta over the partial", 2 * vol + 4 * H * W)}
        return kern, tuple(k for k in ("horizontal", "sweep", "sweep_wta") if stages[k][1] > 0)
    if sweep:
        rec_b = 8 * H * width1  # WTA winner record + sub-pixel inputs per pixel
        # E/W kernel (sm_api.hip ew_lanes): packed lines of 32 / 16 lanes where D % 64 / D % 32 == 0,
        # else 8-lane packed lines (u8 costs) or the per-direction row lines (u16)
        ew_lanes = 32 if D % 64 == 0 else 16 if D % 32 == 0 else 8 if eb == 1 else 0
        ew = f"k_ew ({ew_lanes}-lane packed E/W lines)" if ew_lanes else "k_sgm_paths (E/W row lines only)"
        kern = {"horizontal": (ew, 4 * vol * eb),
                "sweep": ("k_sweep down (S+SE+SW -> u16 partial)", vol * eb + 2 * vol),
                "sweep_wta": ("k_sweep " + ("up (N+NE+NW" if P_dirs == 8 else "down (S+SE+SW")
                              + " + E + W" + (" + partial" if P_dirs == 8 else "") + " + WTA)",
                              3 * vol * eb + (2 * vol if P_dirs == 8 else 0) + rec_b)}
        return kern, tuple(k for k in ("horizontal", "sweep", "sweep_wta") if stages[k][1] > 0)
    # per-direction engine: one path volume per direction written, cost volume read per direction
    kern = {"paths": ("k_sgm_paths (all directions)", 2 * P_dirs * vol * eb),
            "wta": ("k_wta", P_dirs * vol * eb + 2 * H * W)}
    return kern, ("paths", "wta")


# VALU issue ceiling of the chip: 1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction
VALU_PEAK_GINSTR = 1024 * 2.4 / 4


def hbm_roofline(achieved, valu):
    """The dominant kernel's HBM roofline (achieved = SURVEY §8(d) bytes / launch time) and the
    ceiling that binds it: ``bound`` names VALU when the kernel's VALU issue fraction (SQ counters,
    read_valu) exceeds its HBM fraction.  achieved / peak / frac stay the HBM figures; both
    fractions are quoted."""
    f_hbm = achieved / HBM_PEAK_GBS if achieved else None
    f_valu = valu.get("frac") if isinstance(valu, dict) else None
    binding = "valu" if f_valu is not None and f_hbm is not None and f_valu > f_hbm else "hbm"
    return {"bound": binding, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": f_hbm,
            "frac_hbm": f_hbm, "frac_valu": f_valu,
            "bound_note": "achieved/peak/frac: SURVEY §8(d) bytes against HBM; bound = the larger of the HBM "
                          "and VALU-issue fractions (frac_valu = SQ_INSTS_VALU x 4 cycles over the launch, "
                          "roofline.valu)" + ("" if f_valu is not None else "; no VALU counter file: HBM assumed")}


def valu_roofline(valu, launch_s):
    """StereoBM (no cost volume: the SAD window sums are VALU work): the dominant kernel against
    the VALU issue ceiling, from the SQ_INSTS_VALU counter file (tools/valu.sh --mode bm)."""
    insts = valu.get("insts_per_launch") if isinstance(valu, dict) else None
    ach = insts / launch_s / 1e9 if insts and launch_s > 0 else None
    return {"bound": "valu", "achieved": ach, "peak": VALU_PEAK_GINSTR, "unit": "G wave64 VALU instr/s",
            "frac": ach / VALU_PEAK_GINSTR if ach else None,
            "bound_note": "StereoBM has no cost volume to stream; its SAD sums are VALU work, so the frac is "
                          "SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x the launch's cycles at 2.4 GHz)"
                          + ("" if ach else " (no VALU counter file for this mode: unmeasured)")}


def read_traffic(args, dom, kernel_label, pairs_per_launch, sweep):
    """HBM bytes per launch of the dominant kernel from a PMC summary
    (tools/traffic.sh), used only when it was collected on the same sources,
    configuration, mode and engine as this run."""
    if not os.path.exists(args.traffic_file):
        return None, "no traffic file"
    try:
        with open(args.traffic_file) as f:
            tr = json.load(f)
    except (OSError, ValueError):
        return None, "unreadable traffic file"
    want = {"config": args.config, "mode": args.mode, "engine": "sweep" if sweep else "perdir",
            "src_sha16": source_hash(), "pairs_per_launch": pairs_per_launch}
    for k, v in want.items():
        if tr.get(k) != v:
            return None, f"traffic file {os.path.relpath(args.traffic_file, ROOT)} is for {k}={tr.get(k)!r}, " \
                         f"this run has {v!r}: dropped"
    st = tr.get("stages", {}).get(dom)
    if not st:
        return None, f"traffic file has no stage {dom!r}"
    return st.get("hbm_bytes_per_launch"), f"PMC FETCH_SIZE/WRITE_SIZE, {os.path.relpath(args.traffic_file, ROOT)}"


def read_valu(args, dom, pairs_per_launch, sweep, launch_s, H, W, D, path=None):
    """VALU issue of the dominant kernel from the SQ-counter summary
    (tools/valu.sh -> profiles/valu_latest.json), used only when it was collected
    on the same sources, configuration, mode, engine and launch size as this run.
    ``frac`` = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x the profiled launch's
    cycles); ``frac_live`` divides by this run's launch time at 2.4 GHz."""
    path = path or args.valu_file
    if not os.path.exists(path):
        return {"note": "no VALU counter file"}
    try:
        with open(path) as f:
            vs = json.load(f)
    except (OSError, ValueError):
        return {"note": "unreadable VALU counter file"}
    want = {"config": args.config, "mode": args.mode, "engine": "sweep" if sweep else "perdir",
            "src_sha16": source_hash(), "pairs_per_launch": pairs_per_launch}
    for k, v in want.items():
        if vs.get(k) != v:
            return {"note": f"VALU file {os.path.relpath(path, ROOT)} is for {k}={vs.get(k)!r}, this run has {v!r}: "
                            f"dropped"}
    st = vs.get("stages", {}).get(dom)
    if not st:
        return {"note": f"VALU file has no stage {dom!r}"}
    insts = st["sq_insts_valu"]
    cyc = vs["issue_cycles_per_instr"]
    cells = H * (W - D) * D * pairs_per_launch  # minDisparity 0: width1 = W - D
    return {
        "bound": "valu",
        "insts_per_launch": insts,
        "issue_cycles_per_instr": cyc,
        "frac": st.get("valu_issue_frac"),
        "frac_live": insts * cyc / (vs["simds"] * launch_s * 2.4e9) if launch_s > 0 else None,
        "wave_insts_per_cell": insts / cells,
        "lane_ops_per_cell": insts * 64 / cells,
        "wait_any_frac": st.get("wait_any_frac"),
        "note": f"SQ_INSTS_VALU, {os.path.relpath(path, ROOT)} (tools/valu.sh)",
    }


def host_surface(args, device):
    """The reference's own surface (stereo_vision/stereo_vision.py:132-184):
    ``compute_disparity(gray_l, gray_r, settings)`` with host numpy in and
    out, one pair per call, settings.ini values (window_size 5 -> P1 600 /
    P2 2400, numDisparities 160, blockSize 5, lambda 80000, sigma 1.2) at KITTI
    size: left SGBM + right SGBM + WLS, each call synchronous.  Also the
    one-call C-ABI form (sm_compute_disparity) with its host<->device copies
    timed apart."""
    from stereo_match_amd import _lib, compute_disparity, settings, synthetic

    s = dict(settings.DEFAULT_SETTINGS, window_size=5)  # /root/reference/settings.ini:3-23
    H, W = synthetic.CONFIGS["kitti"][:2]
    D = s["num_disparities"]
    gl, gr, _ = synthetic.random_dot_pair(H, W, D, seed=77)
    n = args.host_surface_calls
    e = _lib.engine(device)
    for _ in range(2):
        compute_disparity(gl, gr, s, device=device)
    e.set_timing(True)
    e.reset_timing()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        displ, filt = compute_disparity(gl, gr, s, device=device)
        ts.append(time.perf_counter() - t0)
    st = e.timing()
    e.set_timing(False)
    # one-call C-ABI form
    from stereo_match_amd.stereo_vision import matcher_from_settings
    from stereo_match_amd import wls as _wls
    lm = matcher_from_settings(s, device=device)
    prm = lm.params()  # before createDisparityWLSFilter mutates the matcher (sm_compute_disparity applies it)
    wf = _wls.createDisparityWLSFilter(lm)
    wf.setLambda(s["lmbda"])
    wf.setSigmaColor(s["sigma"])
    wp = wf.params(H, W)
    e.compute_disparity(gl, gr, prm, wp)
    # device time per call: only the call's own span is timed (each timed stage puts events in the
    # stream, which delays the kernels behind them: include/stereo_match_amd.h sm_set_timing)
    e.set_timing(True, stages=["call", "h2d", "d2h"])
    e.reset_timing()
    ts1 = []
    for _ in range(n):
        t0 = time.perf_counter()
        d1, f1 = e.compute_disparity(gl, gr, prm, wp)
        ts1.append(time.perf_counter() - t0)
    st1 = e.timing()
    # the stage breakdown from a second series with every stage timed (slower by the events)
    e.set_timing(True)
    e.reset_timing()
    for _ in range(n):
        e.compute_disparity(gl, gr, prm, wp)
    st2 = e.timing()
    e.set_timing(False)
    med, med1 = float(np.median(ts)), float(np.median(ts1))
    return {
        "what": "stereo_match_amd.compute_disparity(gray_l, gray_r, settings) = reference "
                "stereo_vision.py:132-184: left + right SGBM (5 paths) + WLS, host numpy in/out, one pair per call",
        "workload": f"kitti {W}x{H} D={D} settings.ini (window_size 5, blockSize 5, lambda 80000, sigma 1.2)",
        "calls": n,
        "value": 1.0 / med, "unit": "pairs/s", "ms_per_call_median": med * 1e3,
        "ms_per_call_mean": float(np.mean(ts)) * 1e3,
        "h2d_ms_per_call": st["h2d"][0] / n, "d2h_ms_per_call": st["d2h"][0] / n,
        # the Python surface runs through the one-call ABI for 2-D uint8 numpy pairs (DESIGN.md
        # §4.5; its three-call form for other inputs: left, right, WLS, whose device spans add up)
        "device_ms_per_call": (st["call"][0] if st["call"][0] > 0 else st["total"][0] + st["wls"][0]) / n,
        "device_ms_note": "all stages timed (their events delay the kernels); one_call_abi times the call alone",
        "wls_ms_per_call": st["wls"][0] / n,
        "one_call_abi": {"entry": "sm_compute_disparity", "value": 1.0 / med1, "ms_per_call_median": med1 * 1e3,
                         "h2d_ms_per_call": st1["h2d"][0] / n, "d2h_ms_per_call": st1["d2h"][0] / n,
                         "device_ms_per_call": st1["call"][0] / n,
                         "device_ms_note": "SM_STAGE_CALL alone timed (no per-stage events inside the call)",
                         "wls_ms_per_call": st2["wls"][0] / n,
                         "stage_us_per_call_all_timed": {k: v[0] * 1e3 / n for k, v in st2.items() if v[0] > 0},
                         "same_as_python_surface": bool(np.array_equal(d1, displ) and np.array_equal(f1, filt))},
    }, (gl, gr, s, displ, filt)


def cpu_baseline(args, H, W, D, p, lefts, rights, out0, volume, full=False, hs=None):
    """The C restatement (oracle/sgm_ref.c, -O3) on a bounded sample of the
    same workload: ``--cpu-threads`` host threads each running
    ``--cpu-baseline-pairs`` pairs concurrently (ctypes releases the GIL; the
    port is single-threaded per pair, the pairs are independent), plus the
    one-thread rate.  Also re-checks pair 0 bit for bit; the numpy oracle on
    Tsukuba (BASELINE.md CPU plan step 2); and the host-surface pair
    ``hs`` = (left, right, settings, displ, filtered) through the C port +
    numpy WLS."""
    import threading

    from oracle import ref_c, sgm_np, wls_np
    from stereo_match_amd import synthetic

    n = args.cpu_baseline_pairs
    share, share_src = cpu_share()
    T = max(1, args.cpu_threads or share)
    if volume:
        n = max(1, n // 4)  # ~4x the work per pair (D=192, u16 volume, cost quantisation)
        vol0 = synthetic.absdiff_volume(lefts[0], rights[0], D)[0]

        def one(i):
            return ref_c.compute_volume(vol0, p, 0.0, synthetic.VOLUME_SCALE)
    elif args.mode == "bm":  # numpy restatement (vectorised over pixels, loops over d)
        from oracle import bm_np
        bp = dict(numDisparities=D, blockSize=21)
        n = max(1, n // 4)

        def one(i):
            return bm_np.stereo_bm(lefts[i % len(lefts)], rights[i % len(rights)], bp)
    elif full:  # compute_disparity: C port for both matchers + the numpy WLS restatement
        lp = dict(p, uniquenessRatio=0, disp12MaxDiff=1000000)
        rp = sgm_np.right_matcher_params(p)
        wp = _wls_oracle_params(p, D)
        n = max(1, n // 4)

        def one(i):
            a, b = lefts[i % len(lefts)], rights[i % len(rights)]
            dl = ref_c.compute(a, b, lp)
            wls_np.wls_filter(dl, a, ref_c.compute(b, a, rp), wp)
            return dl
    else:
        def one(i):
            return ref_c.compute(lefts[i % len(lefts)], rights[i % len(rights)], p)
    ref_c.load()
    # one thread
    n1 = max(1, n // 2)
    t0 = time.perf_counter()
    first = one(0)
    for i in range(1, n1):
        one(i)
    dt1 = time.perf_counter() - t0

    def worker(k):
        for i in range(n):
            one(k * n + i)

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(T)]
    t0 = time.perf_counter()
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    dtT = time.perf_counter() - t0
    what = "f32 cost volumes" if volume else ("pairs (left+right C port + numpy WLS)" if full else "pairs")
    out = {
        "value": T * n / dtT,
        "unit": "pairs/s",
        "cores": T,
        "kind": "port",
        "sample": f"{T} threads x {n} {W}x{H} D={D} {what}, oracle/sgm_ref.c -O3 (one pair per thread at a "
                  f"time), {dtT:.1f} s wall",
        "single_thread": {"value": n1 / dt1, "unit": "pairs/s", "cores": 1, "sample": f"{n1} {what}, {dt1:.1f} s"},
        "mpix_disp_per_s": T * n * H * W * D / dtT / 1e6,
        "host_cpus_visible": os.cpu_count(),
        "affinity_cpus": len(os.sched_getaffinity(0)),
        "cpu_share": share,
        "cores_rule": f"--cpu-threads {args.cpu_threads}" if args.cpu_threads else
                      f"the process's CPU share, {share_src}: the GPU pool gives one GPU's job 16 host CPUs and "
                      f"sets OMP_NUM_THREADS to that share, while os.cpu_count() and the affinity mask show the "
                      f"whole machine",
        "gpu_matches_port_pair0": bool(np.array_equal(first, out0)),
    }
    # BASELINE.md CPU plan step 2: the numpy oracle on Tsukuba (config 1), median of 5 after 1 warm-up
    tl, tr, _ = synthetic.random_dot_pair(*synthetic.CONFIGS["tsukuba"], seed=5)
    tp = synthetic.parity_params(16)
    sgm_np.compute(tl, tr, tp)
    tt = []
    for _ in range(5):
        t0 = time.perf_counter()
        sgm_np.compute(tl, tr, tp)
        tt.append(time.perf_counter() - t0)
    out["numpy_tsukuba"] = {"value": 1.0 / float(np.median(tt)), "unit": "pairs/s", "cores": 1,
                            "sample": "oracle/sgm_np.py, 384x288 D=16 OpenCV-SGBM 5-path (settings.ini), "
                                      "median of 5 after 1 warm-up"}
    if hs is not None:  # host surface: the same pair through the C port (both matchers) + numpy WLS
        gl, gr, s, displ, filt = hs
        Dh = s["num_disparities"]
        hp = synthetic.parity_params(Dh, s["window_size"])
        lp = dict(hp, uniquenessRatio=0, disp12MaxDiff=1000000)
        t0 = time.perf_counter()
        dl = ref_c.compute(gl, gr, lp)
        dr = ref_c.compute(gr, gl, sgm_np.right_matcher_params(hp))
        fl = wls_np.wls_filter(dl, gl, dr, _wls_oracle_params(hp, Dh))
        dt = time.perf_counter() - t0
        out["host_surface_port"] = {
            "value": 1.0 / dt, "unit": "pairs/s", "cores": 1,
            "sample": f"1 KITTI pair D={Dh}: oracle/sgm_ref.c left + right + oracle/wls_np.py WLS, {dt:.1f} s",
            "gpu_matches_port": bool(np.array_equal(dl, displ) and np.array_equal(fl, filt)),
        }
    return out


def cpu_share():
    """Host threads this job may use: OMP_NUM_THREADS where the environment sets it (the GPU pool
    sets it to the job's CPU share), else the CPUs in this process's affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env), f"OMP_NUM_THREADS={env}"
    n = len(os.sched_getaffinity(0))
    return n, f"affinity mask ({n} CPUs)"


def _wls_oracle_params(p, D):
    """createDisparityWLSFilter(left) defaults for the numpy WLS restatement."""
    return dict(lmbda=80000.0, sigma=1.2, radius=(p["blockSize"] + 1) // 2, min_disp=p["minDisparity"],
                left_offset=max(0, p["minDisparity"] + D), right_offset=max(0, -p["minDisparity"]))


if __name__ == "__main__":
    main()
