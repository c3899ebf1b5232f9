import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "yolo-continuous_amd")
GOLD = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and the built HIP library")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLD, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def g1():
    return dict(np.load(os.path.join(GOLD, "g1_ops.npz")))


@pytest.fixture(scope="session")
def g2():
    return dict(np.load(os.path.join(GOLD, "g2_nets.npz")))


@pytest.fixture(scope="session")
def g3():
    return dict(np.load(os.path.join(GOLD, "g3_post.npz")))


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")
