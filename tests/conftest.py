"""pytest configuration: the `gpu` marker, repo paths, and lazily built helpers."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "narwhal-tusk_amd")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


def pytest_collection_finish(session):
    """PyTorch-ROCm wheels bundle their own HIP/HSA runtime next to the system
    ROCm one libntcrypto links.  Two runtimes in one process work when torch's
    is initialised first; torch's first HIP init AFTER libntcrypto has mapped
    tens of GB fails ("No HIP GPUs are available").  GPU tests that use torch
    device buffers would then depend on file order, so a session that
    selected GPU tests initialises torch's runtime before any of them runs
    ("PyTorch in the same process")."""
    if not any(item.get_closest_marker("gpu") for item in session.items):
        return
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()
        assert torch.cuda.is_initialized(), "torch's HIP runtime must start before libntcrypto's nt_init"


@pytest.fixture(scope="session")
def oracle():
    import _oracle
    return _oracle.load()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
