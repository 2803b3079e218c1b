import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src")
for p in (ROOT, SRC):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


# GPU tests that start rank processes go first: they must be started by a process that has not touched
# the GPU yet (test_distributed.py), whatever order the other test files would run in
_FIRST = ("test_bench_launches_ranks_and_sums_counts", "test_two_rank_sharded_decode_on_gpu")


def pytest_collection_modifyitems(config, items):
    first = [it for it in items if it.name in _FIRST]
    items[:] = sorted(first, key=lambda it: _FIRST.index(it.name)) + [it for it in items if it.name not in _FIRST]


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))

    return load
