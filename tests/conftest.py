import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        # decompressed once into a dict: indexing an NpzFile re-reads the member on every access
        if name not in cache:
            with np.load(os.path.join(GOLDEN, name)) as z:
                cache[name] = {k: z[k] for k in z.files}
        return cache[name]
    return load
