"""Host-side logic of the drop-in (no GPU compute): settings parsing,
matcher construction, argument checks, the C-ABI symbol table."""
import ctypes
import os

import numpy as np
import pytest

import stereo_match_amd as sm
from stereo_match_amd import _lib, matcher, settings, wls
from stereo_match_amd.stereo_vision import matcher_from_settings


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = _lib.header_symbols()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert lib.sm_version().startswith(b"stereo_match_amd")


def test_soname_names_a_loadable_file():
    """A C program linked with -lstereo_match_amd records DT_NEEDED = the soname: that file
    must exist beside the library (the Makefile's symlink) and be the same library."""
    import subprocess

    path = _lib.LIB_PATH
    dyn = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    import re
    m = re.search(r"Library soname: \[([^\]]+)\]", dyn)
    assert m, dyn
    soname = m.group(1)
    assert soname.endswith(".so.%d" % _lib.ABI_VERSION)
    target = os.path.join(os.path.dirname(path), soname)
    assert os.path.exists(target), target
    assert os.path.samefile(os.path.realpath(target), os.path.realpath(path))
    lib = ctypes.CDLL(target)
    lib.sm_abi_version.restype = ctypes.c_int
    assert lib.sm_abi_version() == _lib.ABI_VERSION


def test_c_abi_struct_matches_header():
    text = open(_lib.HEADER_PATH).read()
    body = text[text.index("typedef struct sm_params"):text.index("} sm_params;")]
    import re
    body = re.sub(r"/\*.*?\*/", "", body.split("{", 1)[1], flags=re.S)
    fields = [n.strip() for decl in body.split(";") if decl.strip()
              for n in decl.strip()[len("int"):].split(",")]
    assert [f for f, _ in _lib.SmParams._fields_] == fields


def test_right_matcher_params_via_abi():
    p = _lib.SmParams(0, 160, 5, 600, 2400, 1, 15, 63, 0, 2, 0, 5)
    r = _lib.right_matcher_params(p)
    assert (r.min_disparity, r.num_disparities, r.uniqueness_ratio, r.disp12_max_diff,
            r.speckle_window_size) == (-159, 160, 0, 1000000, 0)
    assert (r.P1, r.P2, r.block_size, r.pre_filter_cap, r.mode) == (600, 2400, 5, 63, 5)


def test_parse_config_file(tmp_path):
    assert settings.parse_config_file(None) == settings.DEFAULT_SETTINGS
    assert settings.parse_config_file(str(tmp_path / "missing.ini")) == settings.DEFAULT_SETTINGS
    ini = tmp_path / "settings.ini"
    ini.write_text("[disparity]\nwindow_size = 5\nmin_disparity = 0\nnum_disparities = 160\nblock_size = 5\n"
                   "disp12_max_diff = 1\nuniqueness_ratio = 15\nspeckle_window_size = 0\nspeckle_range=2\n"
                   "pre_filter_cap = 63\nlmbda = 80000\nsigma = 1.2\ncost = census\npaths = 8\n")
    s = settings.parse_config_file(str(ini))
    assert s["window_size"] == 5 and s["num_disparities"] == 160 and s["sigma"] == 1.2
    assert s["cost"] == "census" and s["paths"] == 8 and s["mode"] == "P"


def test_matcher_from_settings_p1_p2():
    s = dict(settings.DEFAULT_SETTINGS, window_size=5)
    m = matcher_from_settings(s)
    assert (m.getP1(), m.getP2()) == (600, 2400)
    assert m.getNumDisparities() == 160 and m.getBlockSize() == 5 and m.getMode() == sm.STEREO_SGBM_MODE_SGBM
    m3 = matcher_from_settings(settings.DEFAULT_SETTINGS)
    assert (m3.getP1(), m3.getP2()) == (216, 864)
    assert matcher_from_settings(dict(s, paths=8, cost="census")).params().mode == 8


def test_method_errors_like_reference():
    with pytest.raises(RuntimeError, match="Method not supported"):
        matcher_from_settings(settings.DEFAULT_SETTINGS, method="ELAS")
    bm = matcher_from_settings(settings.DEFAULT_SETTINGS, method="BM")
    assert isinstance(bm, sm.StereoBM)
    assert (bm.getNumDisparities(), bm.getBlockSize(), bm.getTextureThreshold(), bm.getDisp12MaxDiff()) == \
        (160, 5, 10, -1)


def test_bm_right_matcher_and_wls_mutation():
    bm = sm.StereoBM_create(numDisparities=64, blockSize=15)
    r = sm.createRightMatcher(bm)
    assert (r.getMinDisparity(), r.getTextureThreshold(), r.getUniquenessRatio(), r.getDisp12MaxDiff()) == \
        (-63, 0, 0, 1000000)
    f = wls.createDisparityWLSFilter(bm)
    assert (bm.getTextureThreshold(), bm.getUniquenessRatio(), bm.getDisp12MaxDiff()) == (0, 0, 1000000)
    assert (f.left_offset, f.right_offset, f.top_offset, f.bottom_offset) == (64 + 7, 7, 7, 7)
    assert f.getDepthDiscontinuityRadius() == 5  # ceil(0.33 * 15)


def test_create_right_matcher():
    m = sm.StereoSGBM_create(minDisparity=3, numDisparities=64, blockSize=7, P1=10, P2=50,
                             disp12MaxDiff=2, uniquenessRatio=9, preFilterCap=31, mode=sm.STEREO_SGBM_MODE_HH)
    r = sm.createRightMatcher(m)
    assert r.getMinDisparity() == -(3 + 64) + 1 and r.getNumDisparities() == 64
    assert (r.getUniquenessRatio(), r.getDisp12MaxDiff(), r.getSpeckleWindowSize()) == (0, 1000000, 0)
    assert (r.getP1(), r.getP2(), r.getBlockSize(), r.getPreFilterCap(), r.getMode()) == (10, 50, 7, 31, 1)


def test_wls_factory_mutates_left_matcher_like_ximgproc():
    m = sm.StereoSGBM_create(numDisparities=160, blockSize=5, disp12MaxDiff=1, uniquenessRatio=15,
                             speckleWindowSize=100)
    f = wls.createDisparityWLSFilter(m)
    assert (m.getDisp12MaxDiff(), m.getSpeckleWindowSize(), m.getUniquenessRatio()) == (1000000, 0, 0)
    assert f.getDepthDiscontinuityRadius() == 3 and f.left_offset == 160 and f.right_offset == 0


@pytest.mark.parametrize("left,right,exc", [
    (np.zeros((4, 40), np.uint8), np.zeros((4, 41), np.uint8), ValueError),
    (np.zeros((4, 40), np.uint16), np.zeros((4, 40), np.uint16), ValueError),
    (np.zeros((0, 40), np.uint8), np.zeros((0, 40), np.uint8), ValueError),
    (np.zeros((4, 40, 2), np.uint8), np.zeros((4, 40, 2), np.uint8), ValueError),  # gray or BGR only
    (np.zeros((0, 40, 1), np.uint8), np.zeros((0, 40, 1), np.uint8), ValueError),  # empty single-channel 3-D
    (np.zeros((4, 40, 3, 1), np.uint8), np.zeros((4, 40, 3, 1), np.uint8), ValueError),
])
def test_bad_inputs_raise_before_gpu(left, right, exc):
    with pytest.raises(exc):
        sm.StereoSGBM_create().compute(left, right)


def test_unsupported_modes_raise():
    with pytest.raises(sm.SmError):
        sm.StereoSGBM_create(mode=sm.STEREO_SGBM_MODE_SGBM_3WAY).params()
    with pytest.raises(ValueError):
        sm.StereoSGBM_create(cost="sad")


def test_product_package_never_imports_oracle():
    root = os.path.dirname(sm.__file__)
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.replace("oracle/", "").split("\n")[0:0] or True
                assert "import oracle" not in src and "from oracle" not in src, f


def test_write_ply_matches_reference_format(tmp_path):
    """io_functions.write_ply format: header + '%f %f %f %d %d %d ' rows."""
    from stereo_match_amd.reproject import write_ply

    v = np.array([[1.5, -2.25, 3.0], [0.0, 1e-7, 10000.0]], np.float32)
    c = np.array([[255, 0, 7], [1, 2, 3]], np.uint8)
    fn = tmp_path / "p.ply"
    write_ply(str(fn), v, c)
    text = fn.read_text()
    assert text.startswith("ply\nformat ascii 1.0\nelement vertex 2\nproperty float x\n")
    assert text.endswith("end_header\n1.500000 -2.250000 3.000000 255 0 7 \n0.000000 0.000000 10000.000000 1 2 3 \n")


def test_reproject_oracle_known_answer():
    from oracle import reproject_np

    # Q of disparity_calculation.py:295-298 (f = 1164, c = (640, 360))
    Q = np.float32([[1, 0, 0, -640], [0, -1, 0, 360], [0, 0, 0, -1164], [0, 0, 1, 0]])
    d = np.zeros((3, 4), np.int16)
    d[1, 2] = 32
    p = reproject_np.reproject_image_to_3d(d, Q)
    # X = (x - 640)/d, Y = (360 - y)/d, Z = -1164/d
    assert np.allclose(p[1, 2], [(2 - 640) / 32, (360 - 1) / 32, -1164 / 32])
    assert np.isinf(p[0, 0, 2])
    pm = reproject_np.reproject_image_to_3d(d, Q, handle_missing=True)
    assert pm[0, 0, 2] == 10000.0 and pm[1, 2, 2] == p[1, 2, 2]


def test_volume_scale_argument():
    """the automatic quantisation window is opt-in ("auto" -> 0 at the C-ABI); NaN and
    None are refused on the Python surface; numbers pass through."""
    assert _lib.volume_scale("auto") == 0.0
    assert _lib.volume_scale(4000) == 4000.0
    assert _lib.volume_scale(1.0) == 1.0
    for bad in (float("nan"), None, "automatic"):
        with pytest.raises(ValueError):
            _lib.volume_scale(bad)
    import inspect
    assert inspect.signature(sm.StereoSGBM.computeFromCost).parameters["scale"].default == 1.0
