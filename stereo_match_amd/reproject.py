"""3-D reprojection and point-cloud output.

* :func:`reprojectImageTo3D` — ``cv2.reprojectImageTo3D(disp, Q, ddepth=CV_32F)``
  as the reference calls it (``disparity_calculation.py:302``,
  ``mapTo3D_mc_cnn.py:124``), on the GPU (``sm_reproject_image_to_3d``).
* :func:`project_points_3D` — ``stereo_vision/stereo_vision.py:187-210``,
  including its unconditional ``/ 16`` (its ``dtype is not np.float32``
  test is always true).
* :func:`write_ply` — ``io_functions.py:28-44`` / ``mapTo3D.py:59``: the same
  ASCII PLY header and ``'%f %f %f %d %d %d '`` rows.
"""
from __future__ import annotations

import numpy as np

from . import _lib

PLY_HEADER = '''ply
format ascii 1.0
element vertex %(vert_num)d
property float x
property float y
property float z
property uchar red
property uchar green
property uchar blue
end_header
'''


def _is_torch_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def reprojectImageTo3D(disparity, Q, _3dImage=None, handleMissingValues=False, ddepth=-1, device=0):
    """float32 ``[H, W, 3]`` points.  ``disparity``: int16 or float32 (numpy, or
    a torch CUDA tensor → CUDA tensor on torch's current stream).  Only
    ``ddepth`` -1 / CV_32F (5) is implemented (what the reference uses)."""
    if ddepth not in (-1, 5):
        raise _lib.SmError(_lib.SM_E_UNSUPPORTED, "reprojectImageTo3D: only ddepth=CV_32F is implemented")
    Qd = np.ascontiguousarray(np.asarray(Q, np.float64).reshape(4, 4))
    if _is_torch_cuda(disparity):
        import torch

        t = disparity.contiguous()
        kind = {torch.int16: 0, torch.float32: 1}.get(t.dtype)
        if kind is None or t.dim() != 2:
            raise ValueError("disparity must be a 2-D int16 or float32 tensor")
        H, W = t.shape
        out = torch.empty((H, W, 3), dtype=torch.float32, device=t.device)
        eng = _lib.engine(t.device.index or 0)
        eng.set_stream(torch.cuda.current_stream(t.device).cuda_stream)
        eng.reproject_device(t.data_ptr(), kind, 1, H, W, Qd, handleMissingValues, out.data_ptr())
        return out
    d = np.asarray(disparity)
    if d.ndim != 2 or d.dtype not in (np.int16, np.float32):
        raise ValueError("disparity must be a 2-D int16 or float32 array")
    out = _lib.engine(device).reproject(d, Qd, handleMissingValues)
    if _3dImage is not None:
        _3dImage[...] = out
        return _3dImage
    return out


def project_points_3D(disparity, Q):
    """stereo_vision.project_points_3D: ``disparity.astype(float32) / 16`` (always,
    as the reference's identity test is always true), Q as float32."""
    d = np.asarray(disparity).astype(np.float32) / np.float32(16.0)
    return reprojectImageTo3D(d, np.asarray(Q).astype(np.float32))


def write_ply(fn, verts, colors):
    """io_functions.write_ply: ASCII PLY with float xyz and uchar rgb."""
    verts = np.asarray(verts).reshape(-1, 3)
    colors = np.asarray(colors).reshape(-1, 3)
    verts = np.hstack([verts, colors])
    with open(fn, 'wb') as f:
        f.write((PLY_HEADER % dict(vert_num=len(verts))).encode('utf-8'))
        np.savetxt(f, verts, fmt='%f %f %f %d %d %d ')
