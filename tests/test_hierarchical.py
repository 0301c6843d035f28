"""Hierarchical all-reduce across hosts (xGMI/IPC inside each host, one TCP device ring per local rank across
hosts). Several hosts are simulated on one machine with PCCL_HOST_TOKEN: the master groups peers by token, hands
every peer its inter-host ring partners (extra P2P connections) and the host layout, and an op runs hierarchically
only if every participant announces the capability (device buffers + host-local IPC arena + partner connections).

CPU: the extra connections and layout must not disturb the flat host ring. GPU: every process shares cuda:0, each
simulated host's peers rendezvous in their own IPC arena, and results must be exact for sum / avg / max, in-place
and out-of-place, with uint8 quantization on the inter-host stage."""
import json
import os
import subprocess

import pytest

import pccl_amd as pccl
from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, spawn_python

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "workers", "allreduce_peer.py")


def _run(hosts, per_host, device, extra=(), n=(1 << 20) + 37, dtype="f32", steps=3, per_rank=None):
    world = hosts * per_host
    with local_master() as addr:
        procs = []
        for r in range(world):
            args = [WORKER, addr, str(world), str(r), "--n", str(n), "--dtype", dtype, "--device", device,
                    "--steps", str(steps), *extra, *(per_rank(r) if per_rank else [])]
            procs.append(spawn_python(args, env={"PCCL_HOST_TOKEN": f"simhost{r // per_host}"},
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        outs = communicate_all(procs, 300, DIAG_SIGNALS)
    res = []
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        res.append([json.loads(x) for x in o.splitlines() if x.startswith("{")])
    return res


def _expect(world, step, op):
    vals = [r + 1 + step for r in range(world)]
    return {"sum": sum(vals), "avg": sum(vals) / world, "max": max(vals)}[op]


def test_layout_and_extra_connections_keep_host_ring_working():
    res = _run(2, 2, "cpu")
    for lines in res:
        assert len(lines) == 3
        for ln in lines:
            assert ln["lo"] == ln["hi"] == _expect(4, ln["step"], "sum")
            assert ln["path"] == pccl.ReducePath.HOST_RING.value


@pytest.mark.gpu
@pytest.mark.parametrize("hosts,per_host", [(2, 2), (3, 2), (2, 3)])
@pytest.mark.parametrize("op", ["sum", "avg", "max"])
def test_hierarchical_device(hip, hosts, per_host, op):
    world = hosts * per_host
    res = _run(hosts, per_host, "cuda:0", extra=["--op", op])
    for lines in res:
        assert len(lines) == 3
        for ln in lines:
            e = _expect(world, ln["step"], op)
            assert abs(ln["lo"] - e) <= 1e-6 * e and abs(ln["hi"] - e) <= 1e-6 * e, (ln, e)
            assert ln["path"] == pccl.ReducePath.HIERARCHICAL.value


@pytest.mark.gpu
def test_hierarchical_inplace_mixed_bf16(hip):
    res = _run(2, 2, "cuda:0", dtype="bf16", per_rank=lambda r: ["--inplace"] if r % 2 else [])
    for lines in res:
        for ln in lines:
            assert ln["lo"] == ln["hi"] == _expect(4, ln["step"], "sum")
            assert ln["path"] == pccl.ReducePath.HIERARCHICAL.value


@pytest.mark.gpu
def test_hierarchical_quantized_inter_host(hip):
    """uint8 min-max on the inter-host ring: constant inputs quantize exactly, wire bytes shrink."""
    res = _run(2, 2, "cuda:0", extra=["--quant", "u8"])
    for lines in res:
        for ln in lines:
            e = _expect(4, ln["step"], "sum")
            assert abs(ln["lo"] - e) < 0.05 and abs(ln["hi"] - e) < 0.05
            assert ln["path"] == pccl.ReducePath.HIERARCHICAL.value


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_peer_crash_with_host_layout(device, request):
    """A peer of a 2 x 2 layout crashes between ops: the hosts become unequal, the master drops the layout (flat ring
    from then on) and the survivors keep reducing with exact results."""
    if device != "cpu":
        request.getfixturevalue("hip")
    world = 4
    with local_master() as addr:
        procs = []
        for r in range(world):
            args = [WORKER, addr, str(world), str(r), "--n", str(1 << 16), "--dtype", "f32", "--device", device,
                    "--steps", "12", "--const", *(["--die-at", "4"] if r == 3 else [])]
            procs.append(spawn_python(args, env={"PCCL_HOST_TOKEN": f"simhost{r // 2}"},
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        outs = communicate_all(procs, 300, DIAG_SIGNALS)
    assert procs[3].returncode == 17
    for r in range(3):
        assert procs[r].returncode == 0, outs[r][1][-3000:]
        lines = [json.loads(x) for x in outs[r][0].splitlines() if x.startswith("{")]
        oks = [ln for ln in lines if "error" not in ln]
        assert len(oks) == 12 and not any(ln.get("bad") for ln in oks)
        assert oks[-1]["world"] == 3
        if device != "cpu":
            assert oks[0]["path"] == pccl.ReducePath.HIERARCHICAL.value
