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

The WLS smoothing itself (fast global smoother over the confidence map) is
the first "next" row of DESIGN.md §8.  Until it lands on the GPU,
``filter`` raises ``SmError(SM_E_UNSUPPORTED)`` instead of running anything
on the CPU.
"""
from __future__ import annotations

import math

from ._lib import SM_E_UNSUPPORTED, SmError


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

    def setLambda(self, v): self.lmbda = float(v)
    def getLambda(self): return self.lmbda
    def setSigmaColor(self, v): self.sigma_color = float(v)
    def getSigmaColor(self): return self.sigma_color
    def setLRCthresh(self, v): self.lrc_thresh = int(v)
    def getLRCthresh(self): return self.lrc_thresh
    def setDepthDiscontinuityRadius(self, v): self.depth_discontinuity_radius = int(v)
    def getDepthDiscontinuityRadius(self): return self.depth_discontinuity_radius

    def filter(self, disparity_map_left, left_view, filtered_disparity_map=None, disparity_map_right=None,
               ROI=None, right_view=None):
        raise SmError(SM_E_UNSUPPORTED, "DisparityWLSFilter.filter is not implemented on the GPU path yet "
                      "(DESIGN.md §8, next row 1)")


def createDisparityWLSFilter(matcher_left):
    """ximgproc::createDisparityWLSFilter — mutates ``matcher_left`` like upstream."""
    matcher_left.setDisp12MaxDiff(1000000)
    matcher_left.setSpeckleWindowSize(0)
    matcher_left.setUniquenessRatio(0)
    min_disp = matcher_left.getMinDisparity()
    num_disp = matcher_left.getNumDisparities()
    wsize = matcher_left.getBlockSize()
    f = DisparityWLSFilter(True, max(0, min_disp + num_disp), max(0, -min_disp), 0, 0, min_disp)
    f.setDepthDiscontinuityRadius(int(math.ceil(0.5 * wsize)))
    return f


def createDisparityWLSFilterGeneric(use_confidence):
    return DisparityWLSFilter(bool(use_confidence))
