import os
import sys

# bench.py's queue configuration (bench.py:35), set before anything initialises HIP, so the
# concurrency tests (test_pipeline_gpu.py::test_concurrent_registered_tiles_equal_isolated)
# run the four-tile, eight-stream schedule the bench line is measured on, not HIP's default 4
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("HRF_HW_QUEUES", "16")

import pytest  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhrf.so on the device)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)

    return load


@pytest.fixture(scope="session")
def orc():
    import oracle as O

    O.build()
    return O
