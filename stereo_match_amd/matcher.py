"""OpenCV-compatible matcher objects backed by the gfx950 engine.

Mirrors the surface the reference scripts use:

* ``cv2.StereoSGBM_create(...)`` / ``.compute(left, right)`` —
  ``stereo_vision/stereo_vision.py:153-163,178``, ``disparity_test.py:165,191``,
  ``try_try.py:69,81``, ``mapTo3D_mc_cnn.py:81``.
* ``cv2.ximgproc.createRightMatcher(left_matcher)`` —
  ``stereo_vision/stereo_vision.py:171``.

Return contract is OpenCV's: a fresh C-contiguous ``int16[H, W]`` holding
disparity × 16, invalid pixels = ``(minDisparity - 1) * 16``.  Bad
arguments raise ``ValueError`` (OpenCV raises ``cv2.error`` from CV_Assert);
configurations the GPU path does not reproduce raise ``SmError``.

Extension (north-star mode, no OpenCV counterpart): ``cost="census"``
selects the 9×7 census + Hamming cost; ``mode=STEREO_SGBM_MODE_HH`` selects
8 paths.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import SmError, SmParams

# cv2.StereoSGBM mode constants
STEREO_SGBM_MODE_SGBM = 0
STEREO_SGBM_MODE_HH = 1
STEREO_SGBM_MODE_SGBM_3WAY = 2
STEREO_SGBM_MODE_HH4 = 3

_COSTS = {"sgbm": _lib.SM_COST_SGBM, "census": _lib.SM_COST_CENSUS}


def _is_torch_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


class StereoSGBM:
    """cv2.StereoSGBM work-alike (same kwargs, getters/setters, compute)."""

    def __init__(self, minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0, disp12MaxDiff=0,
                 preFilterCap=0, uniquenessRatio=0, speckleWindowSize=0, speckleRange=0,
                 mode=STEREO_SGBM_MODE_SGBM, cost="sgbm", device=0):
        self.minDisparity = int(minDisparity)
        self.numDisparities = int(numDisparities)
        self.blockSize = int(blockSize)
        self.P1 = int(P1)
        self.P2 = int(P2)
        self.disp12MaxDiff = int(disp12MaxDiff)
        self.preFilterCap = int(preFilterCap)
        self.uniquenessRatio = int(uniquenessRatio)
        self.speckleWindowSize = int(speckleWindowSize)
        self.speckleRange = int(speckleRange)
        self.mode = int(mode)
        if cost not in _COSTS:
            raise ValueError(f"cost must be one of {sorted(_COSTS)}")
        self.cost = cost
        self.device = int(device)

    # --- cv::StereoMatcher / cv::StereoSGBM accessors --------------------
    def getMinDisparity(self): return self.minDisparity
    def setMinDisparity(self, v): self.minDisparity = int(v)
    def getNumDisparities(self): return self.numDisparities
    def setNumDisparities(self, v): self.numDisparities = int(v)
    def getBlockSize(self): return self.blockSize
    def setBlockSize(self, v): self.blockSize = int(v)
    def getP1(self): return self.P1
    def setP1(self, v): self.P1 = int(v)
    def getP2(self): return self.P2
    def setP2(self, v): self.P2 = int(v)
    def getDisp12MaxDiff(self): return self.disp12MaxDiff
    def setDisp12MaxDiff(self, v): self.disp12MaxDiff = int(v)
    def getPreFilterCap(self): return self.preFilterCap
    def setPreFilterCap(self, v): self.preFilterCap = int(v)
    def getUniquenessRatio(self): return self.uniquenessRatio
    def setUniquenessRatio(self, v): self.uniquenessRatio = int(v)
    def getSpeckleWindowSize(self): return self.speckleWindowSize
    def setSpeckleWindowSize(self, v): self.speckleWindowSize = int(v)
    def getSpeckleRange(self): return self.speckleRange
    def setSpeckleRange(self, v): self.speckleRange = int(v)
    def getMode(self): return self.mode
    def setMode(self, v): self.mode = int(v)

    def params(self) -> SmParams:
        if self.mode == STEREO_SGBM_MODE_SGBM:
            paths = _lib.SM_MODE_SGBM
        elif self.mode == STEREO_SGBM_MODE_HH:
            paths = _lib.SM_MODE_HH
        else:
            raise SmError(_lib.SM_E_UNSUPPORTED,
                          f"StereoSGBM mode {self.mode} (3WAY/HH4) is not implemented on the GPU path")
        return SmParams(self.minDisparity, self.numDisparities, self.blockSize, self.P1, self.P2,
                        self.disp12MaxDiff, self.uniquenessRatio, self.preFilterCap,
                        self.speckleWindowSize, self.speckleRange, _COSTS[self.cost], paths)

    def compute(self, left, right, disparity=None):
        """StereoSGBM::compute.  numpy in → numpy out (synchronous);
        torch CUDA tensors in → torch int16 tensor out on the same device
        (enqueued on torch's current stream)."""
        prm = self.params()
        if _is_torch_cuda(left) or _is_torch_cuda(right):
            return _compute_torch(left, right, prm)
        left = np.asarray(left)
        right = np.asarray(right)
        _check_pair(left, right, colour=True)
        out = _lib.engine(self.device).compute(left, right, prm)
        if disparity is not None:
            np.copyto(disparity, out)
            return disparity
        return out

    def computeFromCost(self, cost, offset: float = 0.0, scale=1.0):
        """SGM over an external matching-cost volume (mc-cnn).

        ``cost``: float32 ``(1, D, H, W)`` or ``(D, H, W)``, d-major — the
        memmap ``mapTo3D_mc_cnn.py:71`` opens (``np.memmap`` works as is) —
        with ``D == numDisparities``; plane d is the cost of left x against
        right x − (minDisparity + d).  Costs are quantised
        ``rint((c + offset) * scale)`` to [0, 4095] (NaN → 4095), then the
        same paths / WTA / LR / median as :meth:`compute` run (``mode`` picks
        5 or 8 paths; ``blockSize``/``preFilterCap`` are unused).  The window
        is explicit by default (``offset`` 0, ``scale`` 1).  ``scale="auto"``
        (opt-in) derives it per pair on the device from the volume's own finite
        range (offset = -min, scale = 4095 / (max - min)), so nothing is
        clamped; P1 / P2 are in the quantised units either way, so under
        "auto" the smoothing strength follows each frame's own cost range (it
        differs between the pairs of a batch and along a video, and one large
        finite outlier compresses every other cost into a few levels): pass a
        fixed window for consistent smoothing.  Cells that were clamped or NaN
        are counted (``_lib.engine().counters()``).  numpy in → int16 numpy
        out; a torch CUDA float32 tensor in → int16 CUDA tensor (torch's
        current stream)."""
        scale = _lib.volume_scale(scale)
        prm = self.params()
        prm.cost_kind = _lib.SM_COST_VOLUME
        if _is_torch_cuda(cost):
            import torch

            if cost.dtype != torch.float32:
                raise ValueError("cost volume must be float32")
            v = cost.contiguous()
            if v.dim() == 4:
                v = v[0]
            D, H, W = v.shape
            out = torch.empty((H, W), dtype=torch.int16, device=v.device)
            eng = _lib.engine(v.device.index or 0)
            eng.set_stream(torch.cuda.current_stream(v.device).cuda_stream)
            eng.aggregate_cost_f32_device(v.data_ptr(), 1, D * H * W, D, H, W, prm, offset, scale, out.data_ptr())
            return out
        v = np.asarray(cost)
        if v.dtype != np.float32:
            raise ValueError("cost volume must be float32")
        return _lib.engine(self.device).aggregate_cost_f32(v, prm, offset, scale)


def _check_pair(left, right, colour=False):
    """OpenCV's asserts: same size and type, CV_8U; StereoSGBM takes 1 or 3
    channels (try_try.py:56-57,81 passes cv2.imread BGR images), StereoBM gray."""
    if left.shape != right.shape or left.dtype != right.dtype:
        raise ValueError("left and right images must have the same size and type")
    if left.dtype != np.uint8:
        raise ValueError("images must be CV_8U (uint8)")
    if left.ndim not in (2, 3) or left.size == 0:
        raise ValueError("images must be non-empty 2-D arrays")
    if left.ndim == 3 and colour and left.shape[2] == 1:
        return
    if left.ndim == 3 and not (colour and left.shape[2] == 3):
        raise ValueError("images must be gray (H, W)" + (" or BGR (H, W, 3)" if colour else ""))


def _compute_torch(left, right, prm: SmParams):
    import torch

    if left.shape != right.shape or left.dtype != torch.uint8 or right.dtype != torch.uint8:
        raise ValueError("left/right must be same-shape torch.uint8 tensors")
    if left.dim() != 2 or left.device != right.device:
        raise ValueError("left/right must be 2-D tensors on the same device")
    left = left.contiguous()
    right = right.contiguous()
    H, W = left.shape
    out = torch.empty((H, W), dtype=torch.int16, device=left.device)
    eng = _lib.engine(left.device.index or 0)
    eng.set_stream(torch.cuda.current_stream(left.device).cuda_stream)
    eng.compute_device(left.data_ptr(), right.data_ptr(), H, W, W, prm, out.data_ptr())
    return out


def StereoSGBM_create(minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0, disp12MaxDiff=0,
                      preFilterCap=0, uniquenessRatio=0, speckleWindowSize=0, speckleRange=0,
                      mode=STEREO_SGBM_MODE_SGBM, cost="sgbm", device=0):
    """cv2.StereoSGBM_create (reference: stereo_vision/stereo_vision.py:153)."""
    return StereoSGBM(minDisparity, numDisparities, blockSize, P1, P2, disp12MaxDiff, preFilterCap,
                      uniquenessRatio, speckleWindowSize, speckleRange, mode, cost, device)


PREFILTER_NORMALIZED_RESPONSE = 0
PREFILTER_XSOBEL = 1


class StereoBM:
    """cv2.StereoBM work-alike (``cv2.StereoBM_create(numDisparities, blockSize)``,
    reference: stereo_vision/stereo_vision.py:164-166).  The X-Sobel prefilter
    (the default) is implemented; NORMALIZED_RESPONSE raises SmError."""

    def __init__(self, numDisparities=0, blockSize=21, device=0):
        self.minDisparity = 0
        self.numDisparities = int(numDisparities)
        self.blockSize = int(blockSize)
        self.preFilterType = PREFILTER_XSOBEL
        self.preFilterSize = 9
        self.preFilterCap = 31
        self.textureThreshold = 10
        self.uniquenessRatio = 15
        self.speckleWindowSize = 0
        self.speckleRange = 0
        self.disp12MaxDiff = -1
        self.device = int(device)

    def getMinDisparity(self): return self.minDisparity
    def setMinDisparity(self, v): self.minDisparity = int(v)
    def getNumDisparities(self): return self.numDisparities
    def setNumDisparities(self, v): self.numDisparities = int(v)
    def getBlockSize(self): return self.blockSize
    def setBlockSize(self, v): self.blockSize = int(v)
    def getPreFilterType(self): return self.preFilterType
    def setPreFilterType(self, v): self.preFilterType = int(v)
    def getPreFilterSize(self): return self.preFilterSize
    def setPreFilterSize(self, v): self.preFilterSize = int(v)
    def getPreFilterCap(self): return self.preFilterCap
    def setPreFilterCap(self, v): self.preFilterCap = int(v)
    def getTextureThreshold(self): return self.textureThreshold
    def setTextureThreshold(self, v): self.textureThreshold = int(v)
    def getUniquenessRatio(self): return self.uniquenessRatio
    def setUniquenessRatio(self, v): self.uniquenessRatio = int(v)
    def getSpeckleWindowSize(self): return self.speckleWindowSize
    def setSpeckleWindowSize(self, v): self.speckleWindowSize = int(v)
    def getSpeckleRange(self): return self.speckleRange
    def setSpeckleRange(self, v): self.speckleRange = int(v)
    def getDisp12MaxDiff(self): return self.disp12MaxDiff
    def setDisp12MaxDiff(self, v): self.disp12MaxDiff = int(v)

    def params(self) -> "_lib.SmBmParams":
        return _lib.SmBmParams(self.minDisparity, self.numDisparities, self.blockSize, self.preFilterType,
                               self.preFilterSize, self.preFilterCap, self.textureThreshold, self.uniquenessRatio,
                               self.speckleWindowSize, self.speckleRange, self.disp12MaxDiff)

    def compute(self, left, right, disparity=None):
        """StereoBM::compute: numpy in → int16 numpy out; torch CUDA uint8
        tensors → int16 CUDA tensor (torch's current stream)."""
        prm = self.params()
        if _is_torch_cuda(left) or _is_torch_cuda(right):
            import torch

            if left.shape != right.shape or left.dtype != torch.uint8 or left.dim() != 2:
                raise ValueError("left/right must be same-shape 2-D torch.uint8 tensors")
            left, right = left.contiguous(), right.contiguous()
            H, W = left.shape
            out = torch.empty((H, W), dtype=torch.int16, device=left.device)
            eng = _lib.engine(left.device.index or 0)
            eng.set_stream(torch.cuda.current_stream(left.device).cuda_stream)
            eng.bm_compute_batch_device(left.data_ptr(), right.data_ptr(), 1, H * W, H, W, W, prm, out.data_ptr())
            return out
        left = np.asarray(left)
        right = np.asarray(right)
        _check_pair(left, right)
        out = _lib.engine(self.device).bm_compute(left, right, prm)
        if disparity is not None:
            np.copyto(disparity, out)
            return disparity
        return out


def StereoBM_create(numDisparities=0, blockSize=21, device=0):
    """cv2.StereoBM_create (reference: stereo_vision/stereo_vision.py:165)."""
    return StereoBM(numDisparities, blockSize, device)


def createRightMatcher(matcher_left):
    """cv2.ximgproc.createRightMatcher (reference: stereo_vision/stereo_vision.py:171).

    StereoSGBM: minDisparity = -(minD + numD) + 1, uniquenessRatio 0,
    disp12MaxDiff 1e6, speckleWindowSize 0; P1, P2, mode, preFilterCap and
    blockSize copied.  StereoBM: a fresh StereoBM(numD, blockSize) with that
    minDisparity, textureThreshold 0, uniquenessRatio 0, disp12MaxDiff 1e6,
    speckleWindowSize 0.
    """
    if isinstance(matcher_left, StereoBM):
        r = StereoBM(matcher_left.numDisparities, matcher_left.blockSize, matcher_left.device)
        r.setMinDisparity(-(matcher_left.minDisparity + matcher_left.numDisparities) + 1)
        r.setTextureThreshold(0)
        r.setUniquenessRatio(0)
        r.setDisp12MaxDiff(1000000)
        r.setSpeckleWindowSize(0)
        return r
    if not isinstance(matcher_left, StereoSGBM):
        raise SmError(_lib.SM_E_UNSUPPORTED, "createRightMatcher: only StereoSGBM / StereoBM matchers are implemented")
    m = matcher_left
    return StereoSGBM(minDisparity=-(m.minDisparity + m.numDisparities) + 1, numDisparities=m.numDisparities,
                      blockSize=m.blockSize, P1=m.P1, P2=m.P2, disp12MaxDiff=1000000,
                      preFilterCap=m.preFilterCap, uniquenessRatio=0, speckleWindowSize=0,
                      speckleRange=m.speckleRange, mode=m.mode, cost=m.cost, device=m.device)


def filterSpeckles(img, newVal, maxSpeckleSize, maxDiff, buf=None, device=0):
    """cv2.filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) — in place on an
    int16 numpy map (returns ``(img, buf)`` like the cv2 binding) or on a torch
    CUDA int16 tensor (torch's current stream)."""
    if _is_torch_cuda(img):
        import torch

        if img.dtype != torch.int16 or img.dim() != 2 or not img.is_contiguous():
            raise ValueError("expected a contiguous 2-D int16 tensor")
        eng = _lib.engine(img.device.index or 0)
        eng.set_stream(torch.cuda.current_stream(img.device).cuda_stream)
        eng.filter_speckles_device(img.data_ptr(), 1, img.shape[0], img.shape[1], newVal, maxSpeckleSize, maxDiff)
        return img, buf
    a = np.asarray(img)
    if a.dtype != np.int16 or a.ndim != 2:
        raise SmError(_lib.SM_E_UNSUPPORTED, "filterSpeckles: only CV_16SC1 maps are implemented on the GPU path")
    a[...] = _lib.engine(device).filter_speckles(a, newVal, maxSpeckleSize, maxDiff)
    return a, buf
