import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    from hsfft_testlib import GOLDEN
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        meta = json.load(f)
    data = np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False)
    return meta, data
