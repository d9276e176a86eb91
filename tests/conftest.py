import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (runs the HIP path)")


def _ensure_built():
    lib = os.path.join(ROOT, "cubed_amd", "libcubed_amd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", ROOT, "-j8", "cubed_amd/libcubed_amd.so"], check=True)
    ref = os.path.join(ROOT, "oracle", "_ref", "liboracle.so")
    if not os.path.exists(ref):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session")
def built():
    _ensure_built()
    return True


@pytest.fixture(scope="session")
def gpu_executor():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    _ensure_built()
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    return GpuDagExecutor("cuda:0")


@pytest.fixture
def dry():
    from dryrun import DryExecutor

    return DryExecutor()
