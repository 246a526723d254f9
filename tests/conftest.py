import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def engine():
    """One HIP context for the whole GPU session (tests must not fall back to the CPU)."""
    import seqalib_amd
    eng = seqalib_amd.Engine(0)
    yield eng
    eng.close()


@pytest.fixture(autouse=True)
def _batch_kernels(request, monkeypatch):
    """Modules that test the batch kernels (BATCH_KERNELS = True) keep their small host calls off
    the small-call kernel (SEQALIB_TINY=0, sa_tiny.hip); a test may set it back.  The small-call
    kernel has its own tests (test_gpu_tiny.py) and runs by default everywhere else."""
    if getattr(request.module, "BATCH_KERNELS", False):
        monkeypatch.setenv("SEQALIB_TINY", "0")
