"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, C-ABI symbol export,
gloo multi-process DP. `-m gpu` runs on the MI355X box: HIP kernels through the C-ABI vs the
oracle / torch references.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "video-generation-for-human-avatars_amd")
for p in (PKG_ROOT, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
