"""stereo_match_amd — MI355X-native drop-in for the ocean1100/stereo_match hot path.

Public surface (mirrors the reference / OpenCV names the reference uses):

* :func:`compute_disparity` — ``stereo_vision/stereo_vision.py:132``
* :func:`StereoSGBM_create`, :func:`createRightMatcher` — the cv2 /
  cv2.ximgproc calls at ``stereo_vision/stereo_vision.py:153,171``
* :func:`parse_config_file` — ``disparity_calculation.py:75``

All compute runs in ``libstereo_match_amd.so`` (HIP, gfx950) through the
C-ABI in ``include/stereo_match_amd.h``; there is no CPU fallback.
"""
from .matcher import (STEREO_SGBM_MODE_HH, STEREO_SGBM_MODE_HH4, STEREO_SGBM_MODE_SGBM,
                      STEREO_SGBM_MODE_SGBM_3WAY, StereoSGBM, StereoSGBM_create, createRightMatcher,
                      filterSpeckles, StereoBM, StereoBM_create)
from .settings import DEFAULT_SETTINGS, parse_config_file
from .stereo_vision import compute_disparity, matcher_from_settings
from ._lib import SmError
from .reproject import project_points_3D, reprojectImageTo3D, write_ply

__all__ = [
    "compute_disparity", "matcher_from_settings", "StereoSGBM", "StereoSGBM_create", "createRightMatcher",
    "STEREO_SGBM_MODE_SGBM", "STEREO_SGBM_MODE_HH", "STEREO_SGBM_MODE_SGBM_3WAY", "STEREO_SGBM_MODE_HH4",
    "parse_config_file", "DEFAULT_SETTINGS", "SmError", "filterSpeckles", "reprojectImageTo3D",
    "project_points_3D", "write_ply", "StereoBM", "StereoBM_create",
]
__version__ = "0.1.0"
