import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# tests/dev/: parity of the development build's measured-slower variants -- collected only when
# asked for (HSFFT_DEV_TESTS=1, with HSFFT_LIB_PATH pointing at lib/libhsfft_dev.so)
collect_ignore_glob = [] if os.environ.get("HSFFT_DEV_TESTS") == "1" else ["dev/*"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


def pytest_sessionfinish(session, exitstatus):
    """hsfft_finalize() before the test process exits, where the library was loaded and a GPU is
    present: every device object the library holds is released while the runtime is intact"""
    mod = sys.modules.get("hsfft")
    if mod is None or getattr(mod, "_lib", None) is None:
        return
    try:
        if mod.device_count() > 0:
            mod.lib().hsfft_finalize()
    except Exception:  # teardown must not turn a finished session into an error
        pass


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    from hsfft_testlib import GOLDEN
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        meta = json.load(f)
    data = np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False)
    return meta, data
