import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# sm_set_debug_flags bits only the ablation build accepts (sm_api.hip kAblationFlags)
ABLATION_FLAGS = 1 | 2 | 4 | 16 | 32 | 128 | (1 << 27) | 32768 | (7 << 24) | (1 << 28) | (1 << 29) | (1 << 31)


def ablation_build() -> bool:
    """True when the loaded library is the ablation build (make ablation)."""
    from stereo_match_amd import _lib

    return b"ablation" in (_lib.load().sm_version() or b"")


def skip_unless_ablation(flags: int):
    """Tests of measured ablations run only against libstereo_match_amd_ablate.so
    (STEREO_MATCH_AMD_LIB); the product library rejects their flags."""
    if flags & ABLATION_FLAGS and not ablation_build():
        pytest.skip("ablation build only (make -C stereo_match_amd/csrc ablation)")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size parity cases (seconds each)")


@pytest.fixture(scope="session")
def golden_cases():
    import glob
    import json

    import numpy as np

    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        if os.path.basename(path).startswith(("vol_", "wls_")):
            continue
        z = np.load(path, allow_pickle=False)
        out.append((os.path.basename(path)[:-4], z["left"], z["right"], json.loads(str(z["params"])),
                    z["expected"], z["raw"]))
    assert out, "no golden fixtures (run tests/golden/make_golden.py)"
    return out


@pytest.fixture(scope="session")
def golden_volume_cases():
    """(name, vol f32 [D,H,W], params, offset, scale, expected, raw) — mc-cnn mode."""
    import glob
    import json

    import numpy as np

    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "vol_*.npz"))):
        z = np.load(path, allow_pickle=False)
        out.append((os.path.basename(path)[:-4], z["vol"], json.loads(str(z["params"])), float(z["offset"]),
                    float(z["scale"]), z["expected"], z["raw"]))
    assert out, "no volume fixtures (run tests/golden/make_golden.py)"
    return out


@pytest.fixture(scope="session")
def golden_wls_cases():
    """(name, displ, dispr or None, guide, wls params, expected) — WLS post-filter."""
    import glob
    import json

    import numpy as np

    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "wls_*.npz"))):
        z = np.load(path, allow_pickle=False)
        out.append((os.path.basename(path)[:-4], z["displ"], z["dispr"] if "dispr" in z.files else None,
                    z["guide"], json.loads(str(z["params"])), z["expected"]))
    assert out, "no WLS fixtures (run tests/golden/make_golden.py)"
    return out
