"""ctypes loader for oracle/libsgm_ref.so (the C restatement).

TEST INFRASTRUCTURE ONLY — see oracle/sgm_np.py for the parity status
("parity unpinned") and the import rule (tests/, smoke(), bench cpu_baseline).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libsgm_ref.so")


class SgmRefParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "min_disparity", "num_disparities", "block_size", "P1", "P2",
        "disp12_max_diff", "uniqueness_ratio", "pre_filter_cap",
        "speckle_window_size", "speckle_range", "cost_kind", "npaths")]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        build()  # make: no-op when libsgm_ref.so is up to date
        lib = ctypes.CDLL(_LIB)
        lib.sgm_ref_compute.restype = ctypes.c_int
        lib.sgm_ref_compute.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.POINTER(SgmRefParams), ctypes.c_void_p,
                                        ctypes.c_int]
        lib.sgm_ref_compute_wta.restype = ctypes.c_int
        lib.sgm_ref_compute_wta.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.POINTER(SgmRefParams), ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int]
        lib.sgm_ref_compute_cn.restype = ctypes.c_int
        lib.sgm_ref_compute_cn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.POINTER(SgmRefParams),
                                           ctypes.c_void_p, ctypes.c_int]
        lib.sgm_ref_cost_volume_cn.restype = ctypes.c_int
        lib.sgm_ref_cost_volume_cn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.POINTER(SgmRefParams),
                                               ctypes.c_void_p, ctypes.c_void_p]
        lib.sgm_ref_compute_volume.restype = ctypes.c_int
        lib.sgm_ref_compute_volume.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(SgmRefParams), ctypes.c_float, ctypes.c_float,
                                               ctypes.c_void_p, ctypes.c_int]
        lib.sgm_ref_census9x7.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p]
        lib.sgm_ref_median3.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _lib = lib
    return _lib


def make_params(p: dict) -> SgmRefParams:
    return SgmRefParams(
        int(p.get("minDisparity", 0)), int(p.get("numDisparities", 16)), int(p.get("blockSize", 3)),
        int(p.get("P1", 0)), int(p.get("P2", 0)), int(p.get("disp12MaxDiff", 0)),
        int(p.get("uniquenessRatio", 0)), int(p.get("preFilterCap", 0)),
        int(p.get("speckleWindowSize", 0)), int(p.get("speckleRange", 0)),
        int(p.get("cost", 0)), int(p.get("mode", 5)))


def compute(left: np.ndarray, right: np.ndarray, params: dict, median: bool = True) -> np.ndarray:
    """uint8 [H, W] gray or [H, W, 3] BGR pairs (OpenCV's x86 SIMD arithmetic, sgm_ref.c header)."""
    lib = load()
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    if left.shape != right.shape or left.ndim not in (2, 3) or (left.ndim == 3 and left.shape[2] != 3):
        raise ValueError("left/right must be same-size uint8 [H, W] or [H, W, 3]")
    H, W = left.shape[:2]
    cn = 1 if left.ndim == 2 else 3
    out = np.empty((H, W), np.int16)
    prm = make_params(params)
    rc = lib.sgm_ref_compute_cn(left.ctypes.data, right.ctypes.data, H, W, W * cn, cn, ctypes.byref(prm),
                                out.ctypes.data, int(bool(median)))
    if rc != 0:
        raise ValueError(f"sgm_ref_compute failed ({rc})")
    return out


def compute_many(pairs, params: dict, threads: int = 8, median: bool = True):
    """compute() over a list of (left, right) pairs on host threads (ctypes releases the GIL
    during the call; the port is single-threaded per pair): the batch tests' checker for every
    pair of a launch group."""
    from concurrent.futures import ThreadPoolExecutor

    load()
    with ThreadPoolExecutor(max_workers=max(1, min(threads, len(pairs)))) as ex:
        return list(ex.map(lambda lr: compute(lr[0], lr[1], params, median), pairs))


def compute_wta(left: np.ndarray, right: np.ndarray, params: dict, median: bool = True):
    """(disparity int16 [H, W], integer WTA index int16 [H, W]) of a gray pair: the index is
    OpenCV's bestDisp in [0, D) where the pixel passes the uniqueness test, -1 elsewhere
    (before the sub-pixel step, the disp12MaxDiff check and the median)."""
    lib = load()
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    if left.shape != right.shape or left.ndim != 2:
        raise ValueError("left/right must be same-size uint8 [H, W]")
    H, W = left.shape
    out = np.empty((H, W), np.int16)
    wta = np.empty((H, W), np.int16)
    prm = make_params(params)
    rc = lib.sgm_ref_compute_wta(left.ctypes.data, right.ctypes.data, H, W, W, ctypes.byref(prm), out.ctypes.data,
                                 wta.ctypes.data, int(bool(median)))
    if rc != 0:
        raise ValueError(f"sgm_ref_compute_wta failed ({rc})")
    return out, wta


def cost_volume(left: np.ndarray, right: np.ndarray, params: dict) -> np.ndarray:
    """OpenCV's int16 cost rows C[H][width1][D] (P2 seed included; SGBM cost only)."""
    lib = load()
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    H, W = left.shape[:2]
    cn = 1 if left.ndim == 2 else 3
    minD, D = int(params.get("minDisparity", 0)), int(params.get("numDisparities", 16))
    width1 = W + min(minD, 0) - max(minD + D, 0)
    C = np.zeros((H, max(width1, 0), D), np.int16)
    out = np.empty((H, W), np.int16)
    rc = lib.sgm_ref_cost_volume_cn(left.ctypes.data, right.ctypes.data, H, W, W * cn, cn,
                                    ctypes.byref(make_params(params)), C.ctypes.data, out.ctypes.data)
    if rc != 0:
        raise ValueError(f"sgm_ref_cost_volume_cn failed ({rc})")
    return C


def compute_volume(vol: np.ndarray, params: dict, offset: float = 0.0, scale: float = 1.0,
                   median: bool = True) -> np.ndarray:
    """SGM over a d-major float32 cost volume [D][H][W] (or [1][D][H][W])."""
    lib = load()
    v = np.ascontiguousarray(vol, np.float32)
    if v.ndim == 4:
        v = v[0]
    D, H, W = v.shape
    if D != int(params.get("numDisparities", 16)):
        raise ValueError("volume planes != numDisparities")
    out = np.empty((H, W), np.int16)
    prm = make_params(dict(params, cost=2))
    rc = lib.sgm_ref_compute_volume(v.ctypes.data, H, W, ctypes.byref(prm), float(offset), float(scale),
                                    out.ctypes.data, int(bool(median)))
    if rc != 0:
        raise ValueError(f"sgm_ref_compute_volume failed ({rc})")
    return out


def census(img: np.ndarray) -> np.ndarray:
    lib = load()
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    out = np.empty((H, W), np.uint64)
    lib.sgm_ref_census9x7(img.ctypes.data, H, W, W, out.ctypes.data)
    return out
