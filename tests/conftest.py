"""Test configuration.

Markers:
  gpu   -- needs an MI355X (run with `pytest -m gpu` on the GPU box); everything
           else runs on CPU (`pytest -m "not gpu"`).
The oracle (oracle/, test infrastructure) and the product's Python packages
(gym-ignition_amd/python) are put on sys.path here.
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

MODELS = os.path.join(ROOT, "gym-ignition_amd", "models")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X GPU (HIP kernels)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def cartpole_file():
    return os.path.join(MODELS, "cartpole.urdf")


@pytest.fixture(scope="session")
def pendulum_file():
    return os.path.join(MODELS, "pendulum.urdf")


@pytest.fixture(scope="session")
def require_gpu():
    if not gpu_available():
        pytest.fail("this test needs a GPU: run it on the MI355X box (pytest -m gpu)")


@pytest.fixture(scope="session")
def panda_file():
    return os.path.join(MODELS, "panda.urdf")
