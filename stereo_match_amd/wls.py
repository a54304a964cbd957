"""``cv2.ximgproc.createDisparityWLSFilter`` work-alike (next scope row).

Reference use: ``stereo_vision/stereo_vision.py:172-175,182``.

Parity-relevant side effect reproduced here: upstream ximgproc's
``createDisparityWLSFilter(matcher_left)`` MUTATES the matcher it is given —
``setDisp12MaxDiff(1000000)``, ``setSpeckleWindowSize(0)`` and, for
StereoSGBM, ``setUniquenessRatio(0)`` — and the reference calls it (:172)
before ``left_matcher.compute`` (:178).  So the reference's ``displ`` is
produced with the LR check and the uniqueness test disabled, whatever
``settings.ini`` says.  ``compute_disparity`` keeps the reference's call
order, so it inherits exactly that behaviour.

``filter`` runs on the GPU through ``sm_wls_filter`` (kernels in
``csrc/sm_wls.hpp``): LR-consistency × depth-discontinuity confidence, then
the fast global smoother (3 iterations of row/column tridiagonal solves)
over ``conf·disp`` and ``conf``, divided and rounded to int16.  Semantics and
parity status: ``oracle/wls_np.py`` (parity unpinned — ximgproc is not in
the image).  There is no CPU path.
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib
from ._lib import SM_E_UNSUPPORTED, SmError, SmWlsParams


class DisparityWLSFilter:
    def __init__(self, use_confidence=True, left_offset=0, right_offset=0, top_offset=0, bottom_offset=0,
                 min_disp=0):
        self.use_confidence = bool(use_confidence)
        self.left_offset, self.right_offset = left_offset, right_offset
        self.top_offset, self.bottom_offset = top_offset, bottom_offset
        self.min_disp = min_disp
        self.lmbda = 8000.0
        self.sigma_color = 1.0
        self.lrc_thresh = 24
        self.depth_discontinuity_radius = 5
        self.num_iter = 3
        self.lambda_attenuation = 0.25
        self.roll_off = 0.001
        self.device = 0
        self._roi = None

    def setLambda(self, v): self.lmbda = float(v)
    def getLambda(self): return self.lmbda
    def setSigmaColor(self, v): self.sigma_color = float(v)
    def getSigmaColor(self): return self.sigma_color
    def setLRCthresh(self, v): self.lrc_thresh = int(v)
    def getLRCthresh(self): return self.lrc_thresh
    def setDepthDiscontinuityRadius(self, v): self.depth_discontinuity_radius = int(v)
    def getDepthDiscontinuityRadius(self): return self.depth_discontinuity_radius

    def getROI(self):
        return self._roi

    def params(self, H: int, W: int, ROI=None) -> SmWlsParams:
        lo, ro, to, bo = self.left_offset, self.right_offset, self.top_offset, self.bottom_offset
        if ROI is not None and len(ROI) == 4 and ROI[2] * ROI[3] != 0:  # user ROI (x, y, w, h)
            x, y, w, h = (int(v) for v in ROI)
            lo, to, ro, bo = x, y, W - x - w, H - y - h
        self._roi = (lo, to, W - lo - ro, H - to - bo)
        return SmWlsParams(float(self.lmbda), float(self.sigma_color), int(self.lrc_thresh),
                           int(self.depth_discontinuity_radius), int(self.use_confidence), int(self.min_disp),
                           int(lo), int(ro), int(to), int(bo), int(self.num_iter),
                           float(self.lambda_attenuation), float(self.roll_off))

    def filter(self, disparity_map_left, left_view, filtered_disparity_map=None, disparity_map_right=None,
               ROI=None, right_view=None):
        """DisparityWLSFilter::filter (reference: stereo_vision/stereo_vision.py:182).
        numpy in → numpy int16 out (synchronous); torch CUDA tensors in →
        int16 CUDA tensor (torch's current stream)."""
        dl = disparity_map_left
        if getattr(dl, "ndim", 0) != 2:
            raise ValueError("disparity_map_left must be a 2-D int16 map")
        if getattr(left_view, "ndim", 0) == 3:
            raise SmError(SM_E_UNSUPPORTED, "colour guide images are not implemented on the GPU path; "
                          "the reference passes gray_l (stereo_vision.py:182)")
        if tuple(left_view.shape) != tuple(dl.shape):
            raise SmError(SM_E_UNSUPPORTED, "disparity map and guide must have the same size "
                          "(the resize_factor path is not implemented)")
        if self.use_confidence and disparity_map_right is None:
            raise ValueError("this filter uses confidence: pass disparity_map_right")
        H, W = dl.shape
        prm = self.params(H, W, ROI)
        if _is_torch_cuda(dl):
            import torch

            if dl.dtype != torch.int16 or left_view.dtype != torch.uint8:
                raise ValueError("expected int16 disparity and uint8 guide tensors")
            dl = dl.contiguous()
            g = left_view.contiguous()
            dr = disparity_map_right.contiguous() if disparity_map_right is not None else None
            out = torch.empty((H, W), dtype=torch.int16, device=dl.device)
            eng = _lib.engine(dl.device.index or 0)
            eng.set_stream(torch.cuda.current_stream(dl.device).cuda_stream)
            eng.wls_filter_batch_device(dl.data_ptr(), dr.data_ptr() if dr is not None else None, g.data_ptr(),
                                        1, H * W, W, H, W, prm, out.data_ptr())
            res = out
        else:
            dl = np.asarray(dl)
            if dl.dtype != np.int16:
                raise ValueError("disparity_map_left must be CV_16S (int16)")
            g = np.asarray(left_view)
            if g.dtype != np.uint8:
                raise ValueError("left_view must be CV_8U (uint8)")
            dr = None if disparity_map_right is None else np.asarray(disparity_map_right)
            if dr is not None and (dr.dtype != np.int16 or dr.shape != dl.shape):
                raise ValueError("disparity_map_right must be an int16 map of the same size")
            res = _lib.engine(self.device).wls_filter(dl, g, dr, prm)
        if filtered_disparity_map is not None:
            filtered_disparity_map[...] = res
            return filtered_disparity_map
        return res


def _is_torch_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def createDisparityWLSFilter(matcher_left):
    """ximgproc::createDisparityWLSFilter — mutates ``matcher_left`` like upstream
    (disp12MaxDiff 1e6, speckleWindowSize 0; StereoBM also textureThreshold 0 and
    uniquenessRatio 0; StereoSGBM uniquenessRatio 0) and sets the valid-ROI
    offsets (BM: + blockSize/2 on every side) and the discontinuity radius
    (BM: ceil(0.33*blockSize), SGBM: ceil(0.5*blockSize))."""
    from .matcher import StereoBM

    matcher_left.setDisp12MaxDiff(1000000)
    matcher_left.setSpeckleWindowSize(0)
    min_disp = matcher_left.getMinDisparity()
    num_disp = matcher_left.getNumDisparities()
    wsize = matcher_left.getBlockSize()
    wsize2 = wsize // 2
    if isinstance(matcher_left, StereoBM):
        matcher_left.setTextureThreshold(0)
        matcher_left.setUniquenessRatio(0)
        f = DisparityWLSFilter(True, max(0, min_disp + num_disp) + wsize2, max(0, -min_disp) + wsize2, wsize2,
                               wsize2, min_disp)
        f.setDepthDiscontinuityRadius(int(math.ceil(0.33 * wsize)))
        f.device = getattr(matcher_left, "device", 0)
        return f
    matcher_left.setUniquenessRatio(0)
    f = DisparityWLSFilter(True, max(0, min_disp + num_disp), max(0, -min_disp), 0, 0, min_disp)
    f.setDepthDiscontinuityRadius(int(math.ceil(0.5 * wsize)))
    f.device = getattr(matcher_left, "device", 0)
    return f


def createDisparityWLSFilterGeneric(use_confidence):
    return DisparityWLSFilter(bool(use_confidence))
