"""MNIST data-parallel end-to-end: separate peer processes, world 2 / 3 / 2+1 late joiner
(reference python/tests/end_to_end/mnist_ddp/mnist_ddp_e2e_test.py). Beyond the reference's exit-code check we
assert that every peer ends with bit-identical parameters and that the loss went down."""
import json
import os
import subprocess
import time

import pytest

from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, spawn_python

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEER = os.path.join(ROOT, "examples", "mnist_ddp", "mnist_peer.py")


def _run(world, device="cpu", steps=60, late_joiner=False, timeout=150):
    with local_master() as addr:
        procs = []
        n0 = world - 1 if late_joiner else world
        # a late joiner arrives mid-run; otherwise every peer waits for the whole world before training (no peer
        # may finish the run before the last one has even registered)
        extra = ["--min-world", str(world)] if late_joiner else ["--start-world", str(world)]
        for r in range(n0):
            procs.append(spawn_python([PEER, "--master", addr, "--rank", str(r), "--device", device, "--max-steps",
                                       str(steps), *extra], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
        if late_joiner:
            time.sleep(1.5)
            assert all(p.poll() is None for p in procs), "a peer exited before the late joiner arrived"
            procs.append(spawn_python([PEER, "--master", addr, "--rank", str(world - 1), "--device", device,
                                       "--max-steps", str(steps)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
        try:
            outs = communicate_all(procs, timeout, DIAG_SIGNALS)
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
    res = []
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-4000:]
        res.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    return res


def _check(res, steps):
    assert len({r["hash"] for r in res}) == 1, res
    assert all(r["revision"] == steps for r in res), res
    full = [r for r in res if r["steps_here"] >= steps // 2]
    assert full and all(r["loss_last"] < r["loss_first"] for r in full), res


@pytest.mark.parametrize("world", [2, 3])
def test_mnist_ddp(world):
    _check(_run(world), 60)


def test_mnist_ddp_late_joiner():
    res = _run(3, late_joiner=True)
    _check(res, 60)
    assert res[-1]["steps_here"] < 60  # the joiner picked up a run in progress


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_mnist_ddp_gpu(hip, world):
    _check(_run(world, device="cuda"), 60)


@pytest.mark.gpu
def test_mnist_ddp_gpu_late_joiner(hip):
    _check(_run(3, device="cuda", late_joiner=True), 60)


DILOCO_PEER = os.path.join(ROOT, "examples", "mnist_diloco", "mnist_diloco_peer.py")


def _run_diloco(world, device="cpu", late_joiner=False):
    with local_master() as addr:
        procs = []
        n0 = world - 1 if late_joiner else world
        # a late joiner arrives mid-run; otherwise every peer waits for the whole world before training (no peer
        # may finish the run before the last one has even registered)
        extra = ["--min-world", str(world)] if late_joiner else ["--start-world", str(world)]
        for r in range(n0):
            procs.append(spawn_python([DILOCO_PEER, "--master", addr, "--rank", str(r), "--device", device, *extra],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        if late_joiner:
            time.sleep(2.0)
            procs.append(spawn_python([DILOCO_PEER, "--master", addr, "--rank", str(world - 1), "--device", device],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        try:
            outs = communicate_all(procs, 300, DIAG_SIGNALS)
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
    res = []
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        res.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    assert len({r["hash"] for r in res}) == 1, res
    assert all(r["outer_steps"] == 10 for r in res)
    return res


def test_mnist_diloco():
    res = _run_diloco(2)
    assert all(r["loss_last"] < r["loss_first"] for r in res)


def test_mnist_diloco_late_joiner():
    _run_diloco(3, late_joiner=True)


@pytest.mark.gpu
def test_mnist_diloco_gpu(hip):
    _run_diloco(2, device="cuda")
