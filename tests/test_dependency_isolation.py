"""numpy-only and torch-only usage (reference python/tests/{numpy_only_tests,pytorch_only_tests}, run in CI with
the other package uninstalled): the package imports and works with either library blocked."""
import subprocess
import sys

import pytest

from pccl_amd.utils.launch import REPO_ROOT

SCRIPT = r"""
import sys
sys.modules[{blocked!r}] = None          # make `import {blocked}` raise ImportError
sys.path.insert(0, {root!r})
import pccl_amd as pccl
from pccl_amd.utils import local_master, run_threaded_peers
{make}

def fn(rank, comm):
    x = make(rank)
    comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)
    return float(x[0])

with local_master() as addr:
    res = run_threaded_peers(2, fn, address=addr)
assert res == [3.0, 3.0], res

# a lone peer gets TooFewPeers
def alone(rank, comm):
    try:
        comm.all_reduce(make(0), make(0), op=pccl.ReduceOp.SUM, tag=0)
    except pccl.PCCLError as e:
        return e.result
with local_master() as addr:
    assert run_threaded_peers(1, alone, address=addr) == [pccl.Result.TOO_FEW_PEERS]
print("OK")
"""


@pytest.mark.parametrize("blocked,make", [
    ("torch", "import numpy as np\ndef make(r): return np.full(1000, r + 1, dtype=np.float32)"),
    ("numpy", "import torch\ndef make(r): return torch.full((1000,), float(r + 1))"),
])
def test_single_library_install(blocked, make):
    code = SCRIPT.format(blocked=blocked, root=REPO_ROOT, make=make)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
