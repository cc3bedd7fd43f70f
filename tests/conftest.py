import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "map-anything_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP library + device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="session")
def synthetic_sd():
    from mapanything.models.mapanything.spec import canonical_spec
    from mapanything.utils.synthetic import synthetic_state_dict

    return synthetic_state_dict(canonical_spec())


@pytest.fixture(scope="session")
def golden():
    def load(name):
        with np.load(os.path.join(GOLDEN, f"golden_{name}.npz")) as z:
            return {k: z[k] for k in z.files}

    return load
