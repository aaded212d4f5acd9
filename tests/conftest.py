import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: full-size CPU oracle cases")


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "small_manifest.json")) as f:
        man = json.load(f)
    with open(os.path.join(d, "digests.json")) as f:
        dig = json.load(f)
    gold = np.load(os.path.join(d, "small_goldens.npz"))
    return {"manifest": man, "digests": dig, "gold": gold}


def load_manifest(name):
    import json
    with open(os.path.join(ROOT, "feddct_amd", "manifests", name + ".json")) as f:
        return json.load(f)
