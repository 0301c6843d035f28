"""bench.py's RCCL yardstick (extra.multi_gpu_table.rccl) runs only on the driver's multi-GPU node, where one rank per
GPU is possible. Its code path - an RCCL group next to the gloo default group, warm-up, timed all-reduces of every
size, the max over the job - is exercised here with one rank on one GPU, in a child process (its own default group)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, types
sys.path.insert(0, sys.argv[1])
import torch
import torch.distributed as dist
import bench
dist.init_process_group("gloo", rank=0, world_size=1)
job = bench.Job.__new__(bench.Job)
job.torch, job.dist, job.dev, job.world = torch, dist, torch.device("cuda:0"), 1
a = types.SimpleNamespace(steps=3, warmup=1)
print(json.dumps(bench.rccl_reference(job, a, 64 << 20)))
dist.destroy_process_group()
"""


@pytest.mark.gpu
def test_rccl_yardstick_runs_with_one_rank(hip):
    from pccl_amd.utils import free_port
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert "error" not in res, res
    assert res["ranks"] == 1 and all(f"{m}MiB" in res for m in (1, 16)), res
