#!/usr/bin/env python3
"""Benchmark: stereo pairs/s (+ Mpix·disp/s) on the BASELINE.json headline
workload — KITTI 1242×375, D=128, Census 9×7 + 8-path SGM, WTA + uniqueness
+ sub-pixel + left/right check + 3×3 median — on 1..8 MI355X, one process per
GPU (launched by torch.distributed.run for N > 1).

A step = every rank runs the hot path over its batch of ``--pairs-per-gpu``
synthetic pairs already resident in HBM, then (N > 1) the int16 disparity
maps are gathered to rank 0 over RCCL/xGMI (BASELINE config 4).  Weak
scaling: per-GPU work is fixed as N grows.  Timed region: barrier +
device sync on both sides, K steps, max over ranks.

Prints ONE JSON line on rank 0 (see DESIGN.md §6 for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=["kitti", "middlebury", "tsukuba", "mccnn"],
                    help="default: kitti (mccnn for --mode volume8)")
    ap.add_argument("--mode", default="census8", choices=["census8", "sgbm5", "sgbm8", "volume8", "disparity5", "bm"],
                    help="census8 = headline; sgbm5 = OpenCV parity mode; sgbm8 = OpenCV cost + 8 paths; "
                         "volume8 = mc-cnn f32 cost volume; "
                         "disparity5 = the reference's whole compute_disparity (left + right SGBM + WLS); "
                         "bm = StereoBM(numDisparities=D, blockSize=21), the method='BM' matcher")
    ap.add_argument("--pairs-per-gpu", type=int, default=8)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--row", action="store_true",
                    help="experimental fused row kernel (E/W paths + WTA) instead of k_wta (D %% 64 == 0)")
    ap.add_argument("--engine", default="auto", choices=["auto", "perdir", "sweep"],
                    help="auto: fused sweeps for 5 paths, per-direction volumes for 8 paths (measured faster); "
                         "perdir / sweep force one engine (DESIGN.md §4)")
    ap.add_argument("--cpu-baseline-pairs", type=int, default=8,
                    help="pairs timed on the host C port per thread (rank 0, N=1 only); 0 = skip")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads for the multi-core CPU baseline (the box's CPU share is 16)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    return ap.parse_args()


def main():
    args = parse()
    if args.config is None:
        args.config = "mccnn" if args.mode == "volume8" else "kitti"
    import torch
    import torch.distributed as dist

    from stereo_match_amd import _lib, synthetic
    from stereo_match_amd.batch import gather_to_root

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    H, W, D = synthetic.CONFIGS[args.config]
    volume = args.mode == "volume8"
    full = args.mode == "disparity5"
    bm = args.mode == "bm"
    if args.mode == "census8":
        p = synthetic.headline_params(D)
    elif volume:
        p = synthetic.cost_volume_params(D)
    else:
        p = synthetic.parity_params(D)
        if args.mode == "sgbm8":  # OpenCV cost, 8 paths (MODE_HH)
            p = dict(p, mode=8)
    prm = synthetic.to_sm_params(p)
    if bm:
        prm = _lib.SmBmParams()
        _lib.load().sm_bm_default_params(D, 21, prm)
    P = args.pairs_per_gpu
    gpairs = P * world

    # synthetic inputs for this rank's pairs, resident in HBM before timing
    lefts, rights = [], []
    for i in range(rank * P, rank * P + P):
        l, r, _ = synthetic.random_dot_pair(H, W, D, seed=1000 + i)
        lefts.append(l)
        rights.append(r)
    dL = torch.tensor(np.stack(lefts), device=dev)
    dR = torch.tensor(np.stack(rights), device=dev)
    dOut = torch.empty((P, H, W), dtype=torch.int16, device=dev)
    dOutR = dFilt = wprm = None
    if full:  # compute_disparity: settings.ini lambda/sigma, createDisparityWLSFilter defaults
        dOutR = torch.empty_like(dOut)
        dFilt = torch.empty_like(dOut)
        wprm = _lib.wls_default_params(prm)
        wprm.lambda_, wprm.sigma_color = 80000.0, 1.2
    vols = None
    if volume:  # config C: (1, D, H, W) float32 cost per pair, resident in HBM
        vols = torch.empty((P, D, H, W), dtype=torch.float32, device=dev)
        for i in range(P):
            vols[i].copy_(torch.from_numpy(synthetic.absdiff_volume(lefts[i], rights[i], D)[0]))

    eng = _lib.Engine(local_rank)
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    flags = 32 if args.row else 0
    flags |= {"auto": 0, "perdir": 4096, "sweep": 16384}[args.engine]
    if flags:
        eng.set_debug_flags(flags)

    def step():
        if full:
            eng.compute_disparity_batch_device(dL.data_ptr(), dR.data_ptr(), P, H * W, H, W, W, prm, wprm,
                                               dOut.data_ptr(), dOutR.data_ptr(), dFilt.data_ptr())
        elif bm:
            eng.bm_compute_batch_device(dL.data_ptr(), dR.data_ptr(), P, H * W, H, W, W, prm, dOut.data_ptr())
        elif volume:
            eng.aggregate_cost_f32_device(vols.data_ptr(), P, D * H * W, D, H, W, prm, 0.0, synthetic.VOLUME_SCALE,
                                          dOut.data_ptr())
        else:
            eng.compute_batch_device(dL.data_ptr(), dR.data_ptr(), P, H * W, H, W, W, prm, dOut.data_ptr())
        if world > 1 and not args.no_gather:
            gather_to_root(dOut, gpairs)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.set_timing(True)
    eng.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    stages = eng.timing()
    eng.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # correctness spot check of the last step (cheap, outside the timed region)
    out0 = dOut[0].cpu().numpy()
    valid_frac = float((out0 >= 0).mean())

    if rank == 0:
        K = args.steps
        pairs_total = gpairs * K
        value = pairs_total / elapsed
        cells = H * W * D
        width1 = W - D
        vol = H * width1 * D
        P_dirs = 5 if args.mode in ("sgbm5", "disparity5") else 8
        eb = 1 if args.mode == "census8" else 2  # bytes per path element
        row_mode = args.row and D % 64 == 0  # both horizontal paths fused into the row/WTA kernel
        # census mode: the path kernel reads the precomputed u8 Hamming cost volume
        # once per direction (k_census_cost8), like the u16 cost volume in SGBM mode
        census_b = 0
        if row_mode:
            # paths launch: vertical family only; row kernel: E (+W) paths + WTA
            paths_bytes = (P_dirs - 2) * vol * eb + (census_b or (P_dirs - 2) * vol * eb)
            wta_bytes = vol * eb + (P_dirs - 1) * vol * eb + (census_b or 2 * vol * 2) + 2 * H * W
            wta_name = "k_row_wta (E/W paths + WTA + disp2/LR, one wave per row)"
        else:
            paths_bytes = P_dirs * vol * eb + (census_b or P_dirs * vol * eb)
            wta_bytes = P_dirs * vol * eb + 2 * H * W
            wta_name = "k_wta"
        if bm:  # SAD kernel reads the two prefiltered views, writes disparity (+ int32 cost)
            wta_name, wta_bytes = "k_bm_sad (column sums in LDS + WTA)", H * W * (2 + 2 + 4)
        kern = {"paths": ("k_sgm_paths (vertical family)" if row_mode else "k_sgm_paths (all directions)",
                          paths_bytes),
                "wta": (wta_name, wta_bytes)}
        cands = ("paths", "wta")
        if stages["sweep_wta"][1] > 0:  # fused-sweep engine (sm_sweep.hpp): its kernels have stages of their own
            rec_b = 8 * H * width1  # WTA winner record + sub-pixel inputs per pixel
            kern = {"horizontal": ("k_sgm_paths (E/W lines only)", 4 * vol * eb),
                    "sweep": ("k_sweep down (S+SE+SW -> u16 partial)", vol * eb + 2 * vol),
                    "sweep_wta": ("k_sweep " + ("up (N+NE+NW" if P_dirs == 8 else "down (S+SE+SW")
                                  + " + E + W" + (" + partial" if P_dirs == 8 else "") + " + WTA)",
                                  3 * vol * eb + (2 * vol if P_dirs == 8 else 0) + rec_b)}
            cands = tuple(k for k in ("horizontal", "sweep", "sweep_wta") if stages[k][1] > 0)
        # dominant kernel = the stage with the largest device time
        dom = max(cands, key=lambda k: stages[k][0])
        dom_ms, dom_launches, dom_pairs = stages[dom]
        paths_avg_s = dom_ms / 1e3 / max(dom_launches, 1)
        pairs_per_launch = dom_pairs / max(dom_launches, 1)
        alg_bytes_paths = kern[dom][1] * pairs_per_launch
        achieved = alg_bytes_paths / paths_avg_s / 1e9 if paths_avg_s > 0 else None
        traffic = None
        if os.path.exists(args.traffic_file):
            try:
                with open(args.traffic_file) as f:
                    tr = json.load(f)
                if tr.get("config") == args.config and tr.get("mode") == args.mode:
                    st = tr.get("stages", {}).get(dom, {})
                    # per launch of the same pairs-per-launch as this run
                    if st and tr.get("pairs_per_launch", pairs_per_launch) == pairs_per_launch:
                        traffic = st.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        # SURVEY.md §8(d) whole-pipeline model: H·W·D·(1+P+4) + 2HW + 4HW per pair
        # (mc-cnn f32 volume: H·W·D·(4·P + 8))
        if volume:
            survey_bytes = cells * (4 * P_dirs + 8)
        elif bm:  # no volume: images in, prefiltered views, disparity + cost out
            survey_bytes = H * W * (2 + 2 * 2 + 2 + 4)
        elif full:  # two matcher runs (left, right) per pair; WLS traffic is O(H·W)
            survey_bytes = 2 * (cells * (1 + P_dirs + 4) + 2 * H * W + 4 * H * W)
        else:
            survey_bytes = cells * (1 + P_dirs + 4) + 2 * H * W + 4 * H * W
        tot_ms, _, tot_pairs = stages["total"]
        pair_s = tot_ms / 1e3 / max(tot_pairs, 1)
        if full:  # per reference pair: two matcher calls + the WLS filter
            pair_s = (tot_ms + stages["wls"][0]) / 1e3 / max(stages["wls"][2], 1)
        line = {
            "metric": "stereo pairs/sec + Mpix·disp/sec, KITTI 1242×375 D=128 SGM, 1/2/4/8 GPU",
            "value": value,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"census8": "u8", "sgbm5": "i16", "sgbm8": "i16", "volume8": "f32->u16", "disparity5": "i16+f32",
                      "bm": "i32"}[args.mode],
            "data": "synthetic random-dot pairs (no dataset in the image)"
                    + ("; f32 cost = 3x3-smoothed |L-R|/255 volume per pair" if volume else ""),
            "config": {
                "engine": {"auto": "per-direction (census 8 paths) / fused sweeps (otherwise)", "perdir": "per-direction",
                           "sweep": "fused sweeps"}[args.engine],
                "workload": f"{args.config} {W}x{H} D={D} "
                            + {"census8": "census9x7 + 8-path SGM", "sgbm5": "OpenCV-SGBM 5-path",
                               "sgbm8": "OpenCV-SGBM 8-path (MODE_HH)",
                               "volume8": "f32 cost volume (mc-cnn) + 8-path SGM",
                               "disparity5": "compute_disparity: left+right OpenCV-SGBM 5-path + WLS",
                               "bm": "OpenCV StereoBM blockSize 21 (X-Sobel prefilter)"}[args.mode],
                "pairs_per_gpu": P, "global_batch": gpairs, "H": H, "W": W, "D": D,
                "gather": world > 1 and not args.no_gather, "parallelism": f"pairs/dp{world}",
            },
            "mpix_disp_per_s": value * cells / 1e6,
            "roofline": {
                "kernel": kern[dom][0],
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes_paths,
                "pairs_per_launch": pairs_per_launch,
                "avg_launch_us": paths_avg_s * 1e6,
            },
            "pipeline_roofline": {
                "model": "SURVEY §8d " + ("H·W·D·(4P+8)" if volume else "H·W·(2+4+2+4) (no volume)" if bm
                                          else "H·W·D·(1+P+4)+I/O")
                         + (" x2 matchers" if full else "") + " per pair",
                "bytes_per_pair": survey_bytes,
                "device_us_per_pair": pair_s * 1e6,
                "achieved_GBs": survey_bytes / pair_s / 1e9 if pair_s > 0 else None,
                "frac": survey_bytes / pair_s / 1e9 / HBM_PEAK_GBS if pair_s > 0 else None,
            },
            "stage_us_per_pair": {k: v[0] * 1e3 / max(v[2], 1) for k, v in stages.items()},
            "valid_frac_pair0": valid_frac,
        }
        if world == 1 and args.cpu_baseline_pairs > 0:
            line["cpu_baseline"] = cpu_baseline(args, H, W, D, p, lefts, rights, out0, volume, full)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(args, H, W, D, p, lefts, rights, out0, volume, full=False):
    """The C restatement (oracle/sgm_ref.c, -O3) on a bounded sample of the
    same workload: ``--cpu-threads`` host threads each running
    ``--cpu-baseline-pairs`` pairs concurrently (ctypes releases the GIL; the
    port is single-threaded per pair, the pairs are independent), plus the
    one-thread rate.  Also re-checks pair 0 bit for bit."""
    import threading

    from oracle import ref_c
    from stereo_match_amd import synthetic

    n = args.cpu_baseline_pairs
    T = max(1, args.cpu_threads)
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
        from oracle import sgm_np, wls_np
        lp = dict(p, uniquenessRatio=0, disp12MaxDiff=1000000)
        rp = sgm_np.right_matcher_params(p)
        wp = dict(lmbda=80000.0, sigma=1.2, radius=(p["blockSize"] + 1) // 2, min_disp=p["minDisparity"],
                  left_offset=max(0, p["minDisparity"] + D), right_offset=max(0, -p["minDisparity"]))
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
    return {
        "value": T * n / dtT,
        "unit": "pairs/s",
        "cores": T,
        "kind": "port",
        "sample": f"{T} threads x {n} {W}x{H} D={D} {what}, oracle/sgm_ref.c -O3 (one pair per thread at a "
                  f"time), {dtT:.1f} s wall",
        "single_thread": {"value": n1 / dt1, "unit": "pairs/s", "cores": 1, "sample": f"{n1} {what}, {dt1:.1f} s"},
        "mpix_disp_per_s": T * n * H * W * D / dtT / 1e6,
        "host_cpus_visible": os.cpu_count(),
        "gpu_matches_port_pair0": bool(np.array_equal(first, out0)),
    }


if __name__ == "__main__":
    main()
