"""Data-plane framing interoperability (CCoIP/TCP stays wire-compatible with the reference).

Every op agrees on its framing through the master (csrc/proto/packets.hpp kCollFlagExtWire + WireShape): if every
participant speaks the pccl-amd extensions, the commence packet carries one agreed shape (stripes, stripe minimum,
quantized lanes) that every peer runs, whatever its own environment says; if any participant does not (a reference
peer, emulated here by PCCL_WIRE=reference, which registers and initiates exactly like one), the whole ring runs the
reference framing: one connection seq % pool per op, the dequantization packet on the data tag before each step's
data, one lane (reference ccoip/src/cpp/reduce.cpp:149-192). Golden bytes of a reference-framed quantized ring are
pinned natively (tests/native/wire_reference_tests.cpp).

Each peer is its own process (tests/workers/wire_peer.py): random inputs, SUM; the results must be bit-identical on
every peer and within the format's error of the fp64 sum.
"""
import json
import os
import subprocess

import pytest

from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, spawn_python

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "workers", "wire_peer.py")
REF = {"PCCL_WIRE": "reference"}


def _ring(envs, *args, device="cpu", timeout=300):
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, str(len(envs)), str(r), "--device", device, *args],
                           env=dict(e, **({"PCCL_DISABLE_IPC": "1"} if device != "cpu" else {})),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r, e in enumerate(envs)]
        outs = communicate_all(ps, timeout, DIAG_SIGNALS)
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, e[-3000:]
    return [[json.loads(ln) for ln in o.splitlines() if ln.startswith("{")] for o, _ in outs]


def _check(lines, framing, err, path):
    steps = len(lines[0])
    assert steps > 0 and all(len(x) == steps for x in lines)
    for s in range(steps):
        rows = [x[s] for x in lines]
        assert len({r["digest"] for r in rows}) == 1, rows  # bit-identical on every peer
        assert all(r["framing"] == framing and r["path"] == path for r in rows), rows
        assert max(r["max_err"] for r in rows) <= err, rows


@pytest.mark.parametrize("pool", [1, 4])
@pytest.mark.parametrize("quant", ["none", "u8"])
def test_mixed_reference_and_default_peers_host(pool, quant):
    """A reference peer in a ring of default peers: every op of the ring runs the reference framing, on host memory."""
    lines = _ring([{}, REF, {}], "--pool", str(pool), "--quant", quant)
    _check(lines, framing=2, err=1e-4 if quant == "none" else 0.25, path=1)


@pytest.mark.parametrize("envs,framing", [([{}, {}, {}], 1), ([REF, REF, REF], 2)])
def test_uniform_rings_pick_their_framing(envs, framing):
    lines = _ring(envs, "--pool", "4", "--quant", "u8", "--steps", "2")
    _check(lines, framing=framing, err=0.25, path=1)


@pytest.mark.parametrize("quant", ["none", "u8"])
def test_peers_with_different_shape_settings_agree(quant):
    """Peers whose PCCL_RING_STRIPES / PCCL_STRIPE_MIN_BYTES / PCCL_QUANT_LANES / PCCL_SEGMENT_CHUNK_MIB differ used
    to post their sinks on different connections and lane tags and hang; the master's agreed shape makes them derive
    one plan. 48 Mi f32 elements: 64 MiB chunks, so stripes, (quantized) two lanes and 16 MiB segments are in play."""
    envs = [{"PCCL_RING_STRIPES": "8", "PCCL_STRIPE_MIN_BYTES": str(1 << 20), "PCCL_QUANT_LANES": "4",
             "PCCL_SEGMENT_CHUNK_MIB": "16"},
            {"PCCL_RING_STRIPES": "2", "PCCL_STRIPE_MIN_BYTES": str(4 << 20), "PCCL_QUANT_LANES": "1",
             "PCCL_SEGMENT_CHUNK_MIB": "0"},
            {"PCCL_RING_STRIPES": "4", "PCCL_QUANT_LANES": "2", "PCCL_SEGMENT_CHUNK_MIB": "24"}]
    lines = _ring(envs, "--pool", "8", "--quant", quant, "--n", str(48 << 20), "--steps", "1", timeout=400)
    _check(lines, framing=1, err=1e-4 if quant == "none" else 0.3, path=1)


@pytest.mark.gpu
@pytest.mark.parametrize("pool", [1, 4])
@pytest.mark.parametrize("quant", ["none", "u8"])
def test_mixed_reference_and_default_peers_hbm(hip, pool, quant):
    """The same mixed ring with HBM buffers (TCP device ring; the quantized reference framing bounces through pinned
    memory): bit-identical on every peer."""
    lines = _ring([{}, REF, {}], "--pool", str(pool), "--quant", quant, "--dtype", "bf16", device="cuda:0")
    _check(lines, framing=2, err=0.1 if quant == "none" else 0.35, path=2)


@pytest.mark.gpu
def test_mixed_host_and_hbm_reference_peer(hip):
    """A reference-framed CPU peer among HBM peers (mixed memory and mixed framing, quantized)."""
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "3", str(r), "--device", dev, "--quant", "u8", "--dtype", "f32",
                            "--pool", "2"], env=dict(env, PCCL_DISABLE_IPC="1"), stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
              for r, (dev, env) in enumerate([("cuda:0", {}), ("cpu", REF), ("cuda:0", {})])]
        outs = communicate_all(ps, 300, DIAG_SIGNALS)
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [[json.loads(ln) for ln in o.splitlines() if ln.startswith("{")] for o, _ in outs]
    for s in range(len(lines[0])):
        rows = [x[s] for x in lines]
        assert len({r["digest"] for r in rows}) == 1 and all(r["framing"] == 2 for r in rows), rows
        assert max(r["max_err"] for r in rows) <= 0.25, rows


@pytest.mark.gpu
def test_peers_with_different_shape_settings_agree_hbm(hip):
    envs = [{"PCCL_RING_STRIPES": "8", "PCCL_QUANT_LANES": "4", "PCCL_SEGMENT_CHUNK_MIB": "8"},
            {"PCCL_RING_STRIPES": "1", "PCCL_QUANT_LANES": "1"},
            {"PCCL_RING_STRIPES": "4", "PCCL_QUANT_LANES": "2", "PCCL_SEGMENT_CHUNK_MIB": "32"}]
    for quant in ("none", "u8"):
        lines = _ring(envs, "--pool", "8", "--quant", quant, "--dtype", "bf16", "--n", str(64 << 20), "--steps", "2",
                      device="cuda:0")
        _check(lines, framing=1, err=0.15 if quant == "none" else 0.35, path=2)
