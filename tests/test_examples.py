"""The nanoGPT examples (DDP over PCCL, sync / async / quantized DiLoCo) run end to end with two peer processes
and finish with identical model state on both peers (tiny preset, CPU; GPU variants marked gpu)."""
import json
import os
import subprocess

import pytest

from pccl_amd.utils import local_master, spawn_python

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "nanogpt")


def _run(script, extra, device="cpu", world=2, timeout=300):
    base = ["--preset", "tiny", "--device", device, "--batch-size", "4", "--dtype",
            "float32" if device == "cpu" else "bfloat16"]
    with local_master() as addr:
        procs = [spawn_python([os.path.join(EX, script), "--master", addr, *base, *extra],
                              env={"OMP_NUM_THREADS": "2"}, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for _ in range(world)]
        outs = [p.communicate(timeout=timeout) for p in procs]
    done = []
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
        done.append(lines[-1])
    return done


def test_train_pccl_ddp():
    res = _run("train_pccl.py", ["--max-iters", "6"])
    assert all(r["done"] and r["iter"] == 6 for r in res)
    assert res[0]["param_sum"] == res[1]["param_sum"]


@pytest.mark.parametrize("extra", [[], ["--async-outer"], ["--quantize", "uint8"], ["--outer-momentum", "0.9",
                                                                                       "--nesterov"]])
def test_diloco(extra):
    res = _run("sync_diloco.py", ["--max-iters", "12", "--inner-steps", "3", *extra])
    assert res[0]["outer_sum"] == res[1]["outer_sum"]
    assert res[0]["outer_steps"] == 4


@pytest.mark.gpu
def test_train_pccl_ddp_gpu(hip):
    res = _run("train_pccl.py", ["--max-iters", "6"], device="cuda")
    assert res[0]["param_sum"] == res[1]["param_sum"]


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--async-outer"], ["--quantize", "fp8"]])
def test_diloco_gpu(hip, extra):
    res = _run("sync_diloco.py", ["--max-iters", "12", "--inner-steps", "3", *extra], device="cuda")
    assert res[0]["outer_sum"] == res[1]["outer_sum"]
