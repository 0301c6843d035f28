"""The nanoGPT examples (DDP over PCCL, sync / async / quantized DiLoCo) run end to end with two peer processes
and finish with identical model state on both peers (tiny preset, CPU; GPU variants marked gpu)."""
import json
import os
import subprocess
import sys

import pytest

from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, spawn_python

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "nanogpt")


def _run(script, extra, device="cpu", world=2, timeout=300):
    base = ["--preset", "tiny", "--device", device, "--batch-size", "4", "--dtype",
            "float32" if device == "cpu" else "bfloat16"]
    with local_master() as addr:
        procs = [spawn_python([os.path.join(EX, script), "--master", addr, *base, *extra],
                              env={"OMP_NUM_THREADS": "2"}, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for _ in range(world)]
        try:
            outs = communicate_all(procs, timeout, DIAG_SIGNALS)
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
    done = []
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
        done.append(lines[-1])
    return done


@pytest.mark.parametrize("extra", [[], ["--overlap", "--grad-accum", "2"]])
def test_train_pccl_ddp(extra):
    res = _run("train_pccl.py", ["--max-iters", "6", *extra])
    assert all(r["done"] and r["iter"] == 6 for r in res)
    assert res[0]["param_sum"] == res[1]["param_sum"]


@pytest.mark.parametrize("extra", [[], ["--async-outer"], ["--quantize", "uint8"], ["--outer-momentum", "0.9",
                                                                                       "--nesterov"]])
def test_diloco(extra):
    res = _run("sync_diloco.py", ["--max-iters", "12", "--inner-steps", "3", *extra])
    assert res[0]["outer_sum"] == res[1]["outer_sum"]
    assert res[0]["outer_steps"] == 4


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--overlap"]])
def test_train_pccl_ddp_gpu(hip, extra):
    res = _run("train_pccl.py", ["--max-iters", "6", *extra], device="cuda")
    assert res[0]["param_sum"] == res[1]["param_sum"]


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--async-outer"], ["--quantize", "fp8"]])
def test_diloco_gpu(hip, extra):
    res = _run("sync_diloco.py", ["--max-iters", "12", "--inner-steps", "3", *extra], device="cuda")
    assert res[0]["outer_sum"] == res[1]["outer_sum"]


def test_diloco_fsdp_two_nodes():
    """Two simulated nodes (torchrun x 2, gloo FSDP2 with 2 ranks each) x PCCL peer group per local rank."""
    from pccl_amd.utils import free_ports
    ports = free_ports(2)
    with local_master() as addr:
        nodes = [spawn_python(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
                               "127.0.0.1", "--master-port", str(ports[k]), os.path.join(EX, "sync_diloco_fsdp.py"),
                               "--preset", "tiny", "--device", "cpu", "--dtype", "float32",
                               "--batch-size", "2", "--max-iters", "6", "--inner-steps", "3", "--seed", str(1337 + k)],
                              env={"OMP_NUM_THREADS": "1", "PCCL_MASTER": addr}, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True)
                 for k in range(2)]
        try:
            outs = communicate_all(nodes, 300, DIAG_SIGNALS)
        finally:
            for p in nodes:
                if p.poll() is None:
                    p.kill()
    done = {}
    for p, (o, e) in zip(nodes, outs):
        assert p.returncode == 0, e[-3000:]
        for ln in o.splitlines():
            if ln.startswith("{") and '"done"' in ln:
                r = json.loads(ln)
                done.setdefault(r["group"], []).append(r)
    assert sorted(done) == [0, 1]
    for g, rs in done.items():
        assert len(rs) == 2 and rs[0]["outer_sum"] == rs[1]["outer_sum"] and rs[0]["outer_steps"] == 2, rs


def test_prepare_data_and_rccl_baseline(tmp_path):
    """Data prep -> uint16 memmap; the plain-DDP (RCCL/gloo) baseline trainer runs on it under torchrun."""
    from pccl_amd.utils import free_port
    r = subprocess.run([sys.executable, os.path.join(EX, "prepare_data.py"), "--out-dir", str(tmp_path),
                        "--synthetic-bytes", "200000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    p = spawn_python(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
                      "127.0.0.1", "--master-port", str(free_port()), os.path.join(EX, "train_rccl.py"), "--preset",
                      "tiny", "--device", "cpu", "--dtype", "float32", "--max-iters", "3", "--batch-size", "2",
                      "--data", str(tmp_path / "train.bin")], env={"OMP_NUM_THREADS": "1"},
                     stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    o, e = p.communicate(timeout=300)
    assert p.returncode == 0, e[-3000:]
    assert len([ln for ln in o.splitlines() if ln.startswith('{"iter"')]) == 3
