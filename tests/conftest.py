"""Shared pytest configuration.

Markers:
  gpu   - needs an MI355X (HIP device); the driver runs ``pytest -m gpu`` on a GPU box and ``-m "not gpu"`` on CPU.
  slow  - multi-second end-to-end scenarios (still part of the default CPU run).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# a crash inside the library prints the faulting thread's native frames before Python's faulthandler runs (and
# SIGUSR2 dumps every thread of a hung test); the library reads this when it initialises
os.environ.setdefault("PCCL_DEBUG_BACKTRACE_SIGNAL", "1")
os.environ["PYTHONPATH"] = ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU (HIP backend)")
    config.addinivalue_line("markers", "slow: long-running end-to-end scenario")


@pytest.fixture(scope="session")
def hip():
    """Skips unless a HIP device is present *and* the HIP plugin is loaded (fails loudly if the plugin is missing)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pccl_amd.ops import kernels as K
    assert K.hip_device_count() > 0, "GPU present but libpccl_hip.so did not load"
    return torch.device("cuda:0")
