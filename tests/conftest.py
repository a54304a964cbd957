import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


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
        z = np.load(path, allow_pickle=False)
        out.append((os.path.basename(path)[:-4], z["left"], z["right"], json.loads(str(z["params"])),
                    z["expected"], z["raw"]))
    assert out, "no golden fixtures (run tests/golden/make_golden.py)"
    return out
