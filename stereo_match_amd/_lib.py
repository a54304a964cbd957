"""ctypes binding of ``libstereo_match_amd.so`` (C-ABI: include/stereo_match_amd.h).

The product path has NO CPU fallback: if the in-tree HIP library is missing,
``load()`` raises ``ImportError`` with the build command.  Nothing here
imports ``oracle/``.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# STEREO_MATCH_AMD_LIB: alternative build of the same library (kernel experiments only)
LIB_PATH = os.environ.get("STEREO_MATCH_AMD_LIB") or os.path.join(_HERE, "libstereo_match_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "stereo_match_amd.h")

SM_OK, SM_E_ARG, SM_E_HIP, SM_E_UNSUPPORTED = 0, -1, -2, -4
SM_COST_SGBM, SM_COST_CENSUS, SM_COST_VOLUME = 0, 1, 2
SM_MODE_SGBM, SM_MODE_HH = 5, 8
TIMING_ONLY = 0x40000000  # include/stereo_match_amd.h SM_TIMING_ONLY
STAGES = ("cost", "paths", "wta", "median", "total", "wls", "speckle", "horizontal", "sweep", "sweep_wta", "h2d",
          "d2h", "fallback", "call")


class SmParams(ctypes.Structure):
    """Mirror of ``struct sm_params`` (field order must match the header)."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "min_disparity", "num_disparities", "block_size", "P1", "P2",
        "disp12_max_diff", "uniqueness_ratio", "pre_filter_cap",
        "speckle_window_size", "speckle_range", "cost_kind", "mode")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class SmWlsParams(ctypes.Structure):
    """Mirror of ``struct sm_wls_params``."""
    _fields_ = [("lambda_", ctypes.c_double), ("sigma_color", ctypes.c_double)] + [
        (n, ctypes.c_int) for n in (
            "lrc_thresh", "depth_discontinuity_radius", "use_confidence", "min_disp", "left_offset",
            "right_offset", "top_offset", "bottom_offset", "num_iter")] + [
        ("lambda_attenuation", ctypes.c_float), ("roll_off", ctypes.c_float)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class SmBmParams(ctypes.Structure):
    """Mirror of ``struct sm_bm_params``."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "min_disparity", "num_disparities", "block_size", "pre_filter_type", "pre_filter_size",
        "pre_filter_cap", "texture_threshold", "uniqueness_ratio", "speckle_window_size", "speckle_range",
        "disp12_max_diff")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


ABI_VERSION = 3  # include/stereo_match_amd.h SM_ABI_VERSION this binding is written against

_c = ctypes
_SIGS = {
    "sm_version": (_c.c_char_p, []),
    "sm_abi_version": (_c.c_int, []),
    "sm_create": (_c.c_int, [_c.c_int, _c.POINTER(_c.c_void_p)]),
    "sm_destroy": (None, [_c.c_void_p]),
    "sm_set_stream": (_c.c_int, [_c.c_void_p, _c.c_void_p]),
    "sm_reset_stream": (_c.c_int, [_c.c_void_p]),
    "sm_compute": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                              _c.POINTER(SmParams), _c.c_void_p, _c.c_void_p]),
    "sm_compute_wta_batch_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_size_t,
                                               _c.c_int, _c.c_int, _c.c_int, _c.POINTER(SmParams), _c.c_void_p,
                                               _c.c_void_p]),
    "sm_compute_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                     _c.POINTER(SmParams), _c.c_void_p]),
    "sm_compute_batch_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_size_t,
                                           _c.c_int, _c.c_int, _c.c_int, _c.POINTER(SmParams), _c.c_void_p]),
    "sm_compute_cn": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                 _c.POINTER(SmParams), _c.c_void_p]),
    "sm_compute_batch_device_cn": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_size_t,
                                              _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.POINTER(SmParams),
                                              _c.c_void_p]),
    "sm_aggregate_cost_f32": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                         _c.POINTER(SmParams), _c.c_float, _c.c_float, _c.c_void_p]),
    "sm_aggregate_cost_f32_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_size_t, _c.c_int,
                                                _c.c_int, _c.c_int, _c.POINTER(SmParams), _c.c_float,
                                                _c.c_float, _c.c_void_p]),
    "sm_wls_default_params": (_c.c_int, [_c.POINTER(SmParams), _c.POINTER(SmWlsParams)]),
    "sm_wls_filter": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                 _c.POINTER(SmWlsParams), _c.c_void_p]),
    "sm_wls_filter_batch_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int,
                                              _c.c_size_t, _c.c_int, _c.c_int, _c.c_int, _c.POINTER(SmWlsParams),
                                              _c.c_void_p]),
    "sm_compute_disparity": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                        _c.POINTER(SmParams), _c.POINTER(SmWlsParams), _c.c_void_p, _c.c_void_p]),
    "sm_compute_disparity_batch_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_size_t,
                                                     _c.c_int, _c.c_int, _c.c_int, _c.POINTER(SmParams),
                                                     _c.POINTER(SmWlsParams), _c.c_void_p, _c.c_void_p,
                                                     _c.c_void_p]),
    "sm_filter_speckles": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int]),
    "sm_filter_speckles_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                             _c.c_int, _c.c_int]),
    "sm_reproject_image_to_3d": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                            _c.c_void_p, _c.c_int, _c.c_void_p]),
    "sm_reproject_image_to_3d_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                                   _c.c_void_p, _c.c_int, _c.c_void_p]),
    "sm_bm_default_params": (_c.c_int, [_c.c_int, _c.c_int, _c.POINTER(SmBmParams)]),
    "sm_bm_right_matcher_params": (_c.c_int, [_c.POINTER(SmBmParams), _c.POINTER(SmBmParams)]),
    "sm_bm_compute": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                 _c.POINTER(SmBmParams), _c.c_void_p]),
    "sm_bm_compute_batch_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_size_t,
                                              _c.c_int, _c.c_int, _c.c_int, _c.POINTER(SmBmParams), _c.c_void_p]),
    "sm_compute_batch": (_c.c_int, [_c.POINTER(_c.c_void_p), _c.c_int, _c.POINTER(_c.c_void_p),
                                    _c.POINTER(_c.c_void_p), _c.c_int, _c.c_int, _c.c_int, _c.POINTER(SmParams),
                                    _c.c_void_p]),
    "sm_right_matcher_params": (_c.c_int, [_c.POINTER(SmParams), _c.POINTER(SmParams)]),
    "sm_synchronize": (_c.c_int, [_c.c_void_p]),
    "sm_get_counters": (_c.c_int, [_c.c_void_p, _c.POINTER(_c.c_longlong)]),
    "sm_get_counter": (_c.c_int, [_c.c_void_p, _c.c_int, _c.POINTER(_c.c_longlong)]),
    "sm_set_cu_mask": (_c.c_int, [_c.c_void_p, _c.POINTER(_c.c_uint32), _c.c_int]),
    "sm_set_timing": (_c.c_int, [_c.c_void_p, _c.c_int]),
    "sm_get_timing": (_c.c_int, [_c.c_void_p, _c.c_int, _c.POINTER(_c.c_double), _c.POINTER(_c.c_longlong),
                                 _c.POINTER(_c.c_longlong)]),
    "sm_reset_timing": (_c.c_int, [_c.c_void_p]),
    "sm_set_debug_flags": (_c.c_int, [_c.c_void_p, _c.c_int]),
    "sm_set_tuning": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_int]),
    "sm_debug_fetch": (_c.c_longlong, [_c.c_void_p, _c.c_int, _c.c_void_p, _c.c_size_t]),
    "sm_last_error": (_c.c_char_p, [_c.c_void_p]),
}

_lib = None
_lock = threading.Lock()


def wls_default_params(left: SmParams) -> SmWlsParams:
    """sm_wls_default_params: the filter createDisparityWLSFilter(left) builds."""
    out = SmWlsParams()
    rc = load().sm_wls_default_params(ctypes.byref(left), ctypes.byref(out))
    if rc != SM_OK:
        _raise(rc, None)
    return out


def volume_scale(scale) -> float:
    """The C-ABI's scale argument for an external cost volume: "auto" -> 0.0 (the window derived
    per pair on the device), else the explicit float (NaN is refused: it would quantise every
    cell to NaN; the C-ABI itself treats NaN like 0)."""
    if isinstance(scale, str):
        if scale != "auto":
            raise ValueError(f"scale must be a number or 'auto', not {scale!r}")
        return 0.0
    if scale is None:
        raise ValueError("scale=None is ambiguous: pass 'auto' for the per-pair window or a number")
    s = float(scale)
    if s != s:
        raise ValueError("scale is NaN: pass 'auto' for the per-pair window")
    return s


def header_symbols(path: str = HEADER_PATH):
    """Function names declared in include/stereo_match_amd.h."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(sm_\w+)\s*\(", text, flags=re.M)))


def _init_torch_hip_first():
    """torch wheels bundle their own libamdhip64; our library links ROCm's.
    Both runtimes can live in one process, but on the MI355X boxes torch's
    reports "No HIP GPUs are available" if ROCm's was initialised first.  So
    when torch is installed, bring its runtime up before ours (device
    enumeration only; no context is created on any device)."""
    try:
        import torch
    except Exception:  # torch absent: nothing to order
        return
    try:
        if getattr(torch.version, "hip", None):
            torch.cuda.is_available()
    except Exception:
        pass


def load():
    """Load the HIP library (fails loudly if it has not been built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C stereo_match_amd/csrc` "
                "(or python -c 'import __graft_entry__ as g; g.build()'). "
                "There is no CPU fallback.")
        _init_torch_hip_first()
        lib = ctypes.CDLL(LIB_PATH)
        # the version check comes before any other symbol is bound: a library built for an
        # older ABI may lack symbols this binding declares (AttributeError otherwise)
        if not hasattr(lib, "sm_abi_version"):
            raise ImportError(f"{LIB_PATH} predates the versioned C-ABI (no sm_abi_version), this binding needs "
                              f"version {ABI_VERSION}: rebuild it with `make -C stereo_match_amd/csrc`")
        lib.sm_abi_version.restype = ctypes.c_int
        lib.sm_abi_version.argtypes = []
        abi = lib.sm_abi_version()
        if abi != ABI_VERSION:
            raise ImportError(f"{LIB_PATH} has C-ABI version {abi}, this binding needs {ABI_VERSION}: rebuild it "
                              "with `make -C stereo_match_amd/csrc`")
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                raise ImportError(f"{LIB_PATH} (C-ABI {abi}) does not export {name}: rebuild it with "
                                  "`make -C stereo_match_amd/csrc`")
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


class SmError(RuntimeError):
    """Raised for SM_E_HIP / SM_E_UNSUPPORTED (OpenCV would raise cv2.error)."""

    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _raise(code: int, ctx):
    lib = load()
    msg = (lib.sm_last_error(ctx) or b"").decode(errors="replace")
    if code == SM_E_ARG:
        raise ValueError(msg)
    raise SmError(code, msg)


class Engine:
    """One sm_ctx bound to one HIP device (not thread-safe; one per thread)."""

    def __init__(self, device: int = 0):
        lib = load()
        h = ctypes.c_void_p()
        rc = lib.sm_create(int(device), ctypes.byref(h))
        if rc != SM_OK:
            _raise(rc, None)
        self._lib = lib
        self.ctx = h
        self.device = device

    def close(self):
        if getattr(self, "ctx", None):
            self._lib.sm_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != SM_OK:
            _raise(rc, self.ctx)

    def set_stream(self, stream_handle):
        """Enqueue on this hipStream_t handle (0 = the null stream, e.g. torch's
        default stream); None = back to the context's own stream."""
        if stream_handle is None:
            self._check(self._lib.sm_reset_stream(self.ctx))
        else:
            self._check(self._lib.sm_set_stream(self.ctx, ctypes.c_void_p(int(stream_handle))))

    # -- host arrays -------------------------------------------------------
    def compute(self, left: np.ndarray, right: np.ndarray, params: SmParams) -> np.ndarray:
        """uint8 [H, W] gray or [H, W, 3] BGR pairs -> int16 [H, W] disparity x16."""
        left = np.ascontiguousarray(left)
        right = np.ascontiguousarray(right)
        H, W = left.shape[:2]
        cn = 1 if left.ndim == 2 else left.shape[2]
        out = np.empty((H, W), np.int16)
        self._check(self._lib.sm_compute_cn(self.ctx, left.ctypes.data, right.ctypes.data, H, W, W * cn, cn,
                                            ctypes.byref(params), out.ctypes.data))
        return out

    def compute_wta(self, left: np.ndarray, right: np.ndarray, params: SmParams):
        """Gray pair -> (int16 [H, W] disparity x16, int16 [H, W] integer WTA index): the
        index is OpenCV's bestDisp in [0, D) where the uniqueness test passes, -1 elsewhere,
        before the sub-pixel step, the LR check and the median (sm_compute's wta_out)."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        if left.ndim != 2:
            raise ValueError("compute_wta takes gray [H, W] images")
        H, W = left.shape
        out = np.empty((H, W), np.int16)
        wta = np.empty((H, W), np.int16)
        self._check(self._lib.sm_compute(self.ctx, left.ctypes.data, right.ctypes.data, H, W, W,
                                         ctypes.byref(params), out.ctypes.data, wta.ctypes.data))
        return out, wta

    # -- device pointers (e.g. torch tensors' data_ptr()) -------------------
    def compute_wta_batch_device(self, d_left: int, d_right: int, npairs: int, pair_stride: int, H: int, W: int,
                                 stride: int, params: SmParams, d_out: int, d_wta: int):
        self._check(self._lib.sm_compute_wta_batch_device(
            self.ctx, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right), npairs, pair_stride, H, W, stride,
            ctypes.byref(params), ctypes.c_void_p(d_out), ctypes.c_void_p(d_wta)))

    def compute_device(self, d_left: int, d_right: int, H: int, W: int, stride: int, params: SmParams,
                       d_out: int):
        self._check(self._lib.sm_compute_device(self.ctx, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right),
                                                H, W, stride, ctypes.byref(params), ctypes.c_void_p(d_out)))

    def compute_batch_device(self, d_left: int, d_right: int, npairs: int, pair_stride: int, H: int, W: int,
                             stride: int, params: SmParams, d_out: int, channels: int = 1):
        self._check(self._lib.sm_compute_batch_device_cn(
            self.ctx, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right), npairs, pair_stride, H, W, stride,
            channels, ctypes.byref(params), ctypes.c_void_p(d_out)))

    # -- external cost volume (mc-cnn) ----------------------------------------
    def aggregate_cost_f32(self, vol: np.ndarray, params: SmParams, offset: float = 0.0,
                           scale=1.0) -> np.ndarray:
        """SGM over a float32 d-major cost volume [D][H][W] (or [1][D][H][W]).  scale "auto"
        (opt-in): the quantisation window from the volume's own finite range, per pair
        (include/stereo_match_amd.h: scale 0 at the C-ABI); default: the explicit window
        offset 0, scale 1."""
        scale = volume_scale(scale)
        v = np.ascontiguousarray(vol, np.float32)
        if v.ndim == 4:
            if v.shape[0] != 1:
                raise ValueError("expected a (1, D, H, W) volume")
            v = v[0]
        if v.ndim != 3:
            raise ValueError("expected a (D, H, W) float32 volume")
        D, H, W = v.shape
        out = np.empty((H, W), np.int16)
        self._check(self._lib.sm_aggregate_cost_f32(self.ctx, v.ctypes.data, D, H, W, ctypes.byref(params),
                                                    float(offset), float(scale), out.ctypes.data))
        return out

    def aggregate_cost_f32_device(self, d_cost: int, npairs: int, pair_stride_elems: int, D: int, H: int,
                                  W: int, params: SmParams, offset: float, scale, d_out: int):
        self._check(self._lib.sm_aggregate_cost_f32_device(
            self.ctx, ctypes.c_void_p(d_cost), npairs, pair_stride_elems, D, H, W, ctypes.byref(params),
            float(offset), volume_scale(scale), ctypes.c_void_p(d_out)))

    # -- WLS post-filter --------------------------------------------------------
    def wls_filter(self, displ: np.ndarray, guide: np.ndarray, dispr, params: "SmWlsParams") -> np.ndarray:
        displ = np.ascontiguousarray(displ, np.int16)
        guide = np.ascontiguousarray(guide, np.uint8)
        H, W = displ.shape
        if guide.shape != (H, W):
            raise ValueError("guide must be a gray (uint8) image of the disparity map's size")
        ptr_r = None
        if dispr is not None:
            dispr = np.ascontiguousarray(dispr, np.int16)
            if dispr.shape != (H, W):
                raise ValueError("right disparity map must match the left one")
            ptr_r = dispr.ctypes.data
        out = np.empty((H, W), np.int16)
        self._check(self._lib.sm_wls_filter(self.ctx, displ.ctypes.data, ptr_r, guide.ctypes.data, W, H, W,
                                            ctypes.byref(params), out.ctypes.data))
        return out

    def wls_filter_batch_device(self, d_displ: int, d_dispr, d_guide: int, npairs: int, guide_pair_stride: int,
                                guide_stride: int, H: int, W: int, params: "SmWlsParams", d_out: int):
        self._check(self._lib.sm_wls_filter_batch_device(
            self.ctx, ctypes.c_void_p(d_displ), ctypes.c_void_p(d_dispr or 0) if d_dispr else None,
            ctypes.c_void_p(d_guide), npairs, guide_pair_stride, guide_stride, H, W, ctypes.byref(params),
            ctypes.c_void_p(d_out)))

    def compute_disparity(self, left: np.ndarray, right: np.ndarray, params: SmParams, wls: "SmWlsParams"):
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        H, W = left.shape
        displ = np.empty((H, W), np.int16)
        filt = np.empty((H, W), np.int16)
        self._check(self._lib.sm_compute_disparity(self.ctx, left.ctypes.data, right.ctypes.data, H, W, W,
                                                   ctypes.byref(params), ctypes.byref(wls), displ.ctypes.data,
                                                   filt.ctypes.data))
        return displ, filt

    def compute_disparity_batch_device(self, d_left: int, d_right: int, npairs: int, pair_stride: int, H: int,
                                       W: int, stride: int, params: SmParams, wls: "SmWlsParams", d_displ: int,
                                       d_dispr: int, d_filtered: int):
        self._check(self._lib.sm_compute_disparity_batch_device(
            self.ctx, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right), npairs, pair_stride, H, W, stride,
            ctypes.byref(params), ctypes.byref(wls), ctypes.c_void_p(d_displ), ctypes.c_void_p(d_dispr),
            ctypes.c_void_p(d_filtered)))

    # -- speckle filter -------------------------------------------------------
    def filter_speckles(self, img: np.ndarray, new_val: int, max_speckle_size: int, max_diff: int) -> np.ndarray:
        """cv::filterSpeckles on a copy of an int16 map (returns the filtered map)."""
        out = np.array(img, dtype=np.int16, order="C", copy=True)
        if out.ndim != 2:
            raise ValueError("expected a 2-D int16 map")
        H, W = out.shape
        self._check(self._lib.sm_filter_speckles(self.ctx, out.ctypes.data, H, W, int(new_val),
                                                 int(max_speckle_size), int(max_diff)))
        return out

    def filter_speckles_device(self, d_img: int, nimg: int, H: int, W: int, new_val: int, max_speckle_size: int,
                               max_diff: int):
        self._check(self._lib.sm_filter_speckles_device(self.ctx, ctypes.c_void_p(d_img), nimg, H, W, int(new_val),
                                                        int(max_speckle_size), int(max_diff)))

    # -- 3-D reprojection ---------------------------------------------------------
    def reproject(self, disp: np.ndarray, Q: np.ndarray, handle_missing: bool = False) -> np.ndarray:
        d = np.ascontiguousarray(disp)
        kind = {np.dtype(np.int16): 0, np.dtype(np.float32): 1}.get(d.dtype)
        if kind is None or d.ndim != 2:
            raise ValueError("disparity must be a 2-D int16 or float32 array")
        Qd = np.ascontiguousarray(np.asarray(Q, np.float64).reshape(16))
        H, W = d.shape
        out = np.empty((H, W, 3), np.float32)
        self._check(self._lib.sm_reproject_image_to_3d(self.ctx, d.ctypes.data, kind, H, W, Qd.ctypes.data,
                                                       int(bool(handle_missing)), out.ctypes.data))
        return out

    def reproject_device(self, d_disp: int, kind: int, nimg: int, H: int, W: int, Q: np.ndarray,
                         handle_missing: bool, d_xyz: int):
        Qd = np.ascontiguousarray(np.asarray(Q, np.float64).reshape(16))
        self._check(self._lib.sm_reproject_image_to_3d_device(self.ctx, ctypes.c_void_p(d_disp), kind, nimg, H, W,
                                                              Qd.ctypes.data, int(bool(handle_missing)),
                                                              ctypes.c_void_p(d_xyz)))

    # -- StereoBM -------------------------------------------------------------------
    def bm_compute(self, left: np.ndarray, right: np.ndarray, params: "SmBmParams") -> np.ndarray:
        left = np.ascontiguousarray(left)
        right = np.ascontiguousarray(right)
        H, W = left.shape
        out = np.empty((H, W), np.int16)
        self._check(self._lib.sm_bm_compute(self.ctx, left.ctypes.data, right.ctypes.data, H, W, W,
                                            ctypes.byref(params), out.ctypes.data))
        return out

    def bm_compute_batch_device(self, d_left: int, d_right: int, npairs: int, pair_stride: int, H: int, W: int,
                                stride: int, params: "SmBmParams", d_out: int):
        self._check(self._lib.sm_bm_compute_batch_device(
            self.ctx, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right), npairs, pair_stride, H, W, stride,
            ctypes.byref(params), ctypes.c_void_p(d_out)))

    def synchronize(self):
        self._check(self._lib.sm_synchronize(self.ctx))

    COUNTERS = ("sweep_fallbacks", "ew_repairs", "volume_clamped", "volume_nan", "line_groups",
                "ew_open", "band_repairs", "band_open", "band_groups", "line_strips")  # SM_COUNTER_*

    def counters(self) -> dict:
        """Counters since the engine was created (include/stereo_match_amd.h SM_COUNTER_*):
        sweep_fallbacks (launch groups the guarded fallback recomputed), ew_repairs (in-sweep
        E/W strip segments the patch pass recomputed), volume_clamped / volume_nan (external
        cost-volume cells clamped by the quantisation window / NaN), line_groups (launch groups
        whose E/W paths ran inside the down sweep), ew_open (of the ew_repairs, segments whose
        recomputation had not met the speculative values by the strip's end), band_repairs /
        band_open / band_groups (the row-band engine's repaired chains, chains that crossed a
        boundary, launch groups), line_strips (strips x pairs of the line_groups)."""
        out = {}
        n = ctypes.c_longlong()
        for i, name in enumerate(self.COUNTERS):
            self._check(self._lib.sm_get_counter(self.ctx, i, ctypes.byref(n)))
            out[name] = n.value
        return out

    def set_cu_mask(self, cus):
        """Restrict the context's streams to the CU indices in ``cus`` (None: all)."""
        if cus is None:
            self._check(self._lib.sm_set_cu_mask(self.ctx, None, 0))
            return
        nwords = (max(cus) // 32 + 1) if cus else 1
        words = (ctypes.c_uint32 * nwords)()
        for c in cus:
            words[c // 32] |= 1 << (c % 32)
        self._check(self._lib.sm_set_cu_mask(self.ctx, words, nwords))

    # -- timing ---------------------------------------------------------------
    def set_timing(self, on, stages=None):
        """on: every stage; with ``stages`` (names from STAGES) only those stages
        record events (each timed stage delays the stream a little)."""
        v = int(bool(on))
        if on and stages is not None:
            v = TIMING_ONLY
            for name in stages:
                v |= 1 << STAGES.index(name)
        self._check(self._lib.sm_set_timing(self.ctx, v))

    def reset_timing(self):
        self._check(self._lib.sm_reset_timing(self.ctx))

    def timing(self) -> dict:
        """{stage: (total_ms, launches, pairs)}"""
        out = {}
        for i, name in enumerate(STAGES):
            ms = ctypes.c_double()
            n = ctypes.c_longlong()
            np_ = ctypes.c_longlong()
            self._check(self._lib.sm_get_timing(self.ctx, i, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(np_)))
            out[name] = (ms.value, n.value, np_.value)
        return out

    # -- debug ------------------------------------------------------------------
    def set_debug_flags(self, flags: int):
        """Timing ablations only (results become wrong); 0 = normal."""
        self._check(self._lib.sm_set_debug_flags(self.ctx, int(flags)))

    TUNE_EW_LANES, TUNE_SWEEP_NCW, TUNE_EW_WAVES, TUNE_EW_PRIO, TUNE_EW_WARMUP, TUNE_SWEEP_LINES = 1, 2, 3, 4, 5, 6
    TUNE_EW_GUESS = 7
    TUNE_BANDS, TUNE_BAND_WARMUP, TUNE_BAND_GUESS, TUNE_COST_WGS, TUNE_LR_STAGGER, TUNE_SWEEP_XCD = 8, 9, 10, 11, 12, 13

    def set_tuning(self, key: int, value: int):
        """Launch-shape knob (include/stereo_match_amd.h sm_set_tuning); 0 = automatic."""
        self._check(self._lib.sm_set_tuning(self.ctx, int(key), int(value)))

    def debug_fetch(self, what: int) -> bytes:
        n = self._lib.sm_debug_fetch(self.ctx, what, None, 0)
        if n < 0:
            _raise(int(n), self.ctx)
        buf = (ctypes.c_char * max(int(n), 1))()
        r = self._lib.sm_debug_fetch(self.ctx, what, buf, int(n))
        if r < 0:
            _raise(int(r), self.ctx)
        return bytes(buf)[:int(n)]


def right_matcher_params(p: SmParams) -> SmParams:
    lib = load()
    out = SmParams()
    rc = lib.sm_right_matcher_params(ctypes.byref(p), ctypes.byref(out))
    if rc != SM_OK:
        _raise(rc, None)
    return out


def compute_batch(engines, lefts, rights, params: SmParams) -> np.ndarray:
    """sm_compute_batch over several Engines (one per device): host pairs in,
    int16 [n, H, W] out; pairs sharded contiguously across the engines."""
    lib = load()
    n = len(lefts)
    if n != len(rights):
        raise ValueError("lefts and rights differ in length")
    if n == 0:
        return np.empty((0, 0, 0), np.int16)
    L = [np.ascontiguousarray(a, np.uint8) for a in lefts]
    R = [np.ascontiguousarray(b, np.uint8) for b in rights]
    H, W = L[0].shape
    if any(a.shape != (H, W) for a in L + R):
        raise ValueError("all images must have the same shape")
    out = np.empty((n, H, W), np.int16)
    ctxs = (ctypes.c_void_p * len(engines))(*[e.ctx for e in engines])
    lp = (ctypes.c_void_p * n)(*[a.ctypes.data for a in L])
    rp = (ctypes.c_void_p * n)(*[b.ctypes.data for b in R])
    rc = lib.sm_compute_batch(ctxs, len(engines), lp, rp, n, H, W, ctypes.byref(params), out.ctypes.data)
    if rc != SM_OK:
        _raise(rc, None)
    return out


_engines: dict = {}


def engine(device: int = 0) -> Engine:
    """Per-(thread, device) cached engine."""
    key = (threading.get_ident(), device)
    e = _engines.get(key)
    if e is None:
        e = _engines[key] = Engine(device)
    return e
