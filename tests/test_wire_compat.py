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


def _ltv(pid, payload):
    return len(payload).__add__(2).to_bytes(8, "big") + pid.to_bytes(2, "big") + payload


def _ref_str(s):
    b = s.encode()
    return len(b).to_bytes(8, "big") + b


class _ReferenceDistributor:
    """A shared-state distributor at the socket level that speaks only the reference's S2C protocol, written from the
    reference sources, not from this library's code: C2SPacketRequestSharedState (id 1) = u64 key count + (u64 length
    + bytes) per key; S2CPacketSharedStateResponse (id 1) = u8 status (1 = SUCCESS) + u64 revision + u64 entry count +
    (string key, u64 size) per entry, then every entry's raw bytes in order (ccoip_packets.cpp:551-596,
    ccoip_client_handler.cpp:1022-1164). Any other packet id (the same-host IPC extension) closes the connection."""

    def __init__(self, tensors, revision):
        import socket
        import threading
        self.tensors, self.revision = tensors, revision
        self.requests, self.refused = [], 0
        self.lock = threading.Lock()
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(16)
        self.port = self.srv.getsockname()[1]
        threading.Thread(target=self._accept, daemon=True).start()

    @staticmethod
    def _read(c, n):
        out = b""
        while len(out) < n:
            k = c.recv(n - len(out))
            if not k:
                raise ConnectionError
            out += k
        return out

    def _accept(self):
        import threading
        while True:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        try:
            hdr = self._read(c, 10)
            n, pid = int.from_bytes(hdr[:8], "big"), int.from_bytes(hdr[8:], "big")
            payload = self._read(c, n - 2)
            if pid != 1:
                with self.lock:
                    self.refused += 1
                return
            keys, off = [], 8
            for _ in range(int.from_bytes(payload[:8], "big")):
                ln = int.from_bytes(payload[off:off + 8], "big")
                keys.append(payload[off + 8:off + 8 + ln].decode())
                off += 8 + ln
            with self.lock:
                self.requests.append((keys, payload))
            body = bytes([1]) + self.revision.to_bytes(8, "big") + len(keys).to_bytes(8, "big")
            for k in keys:
                body += _ref_str(k) + self.tensors[k].nbytes.to_bytes(8, "big")
            c.sendall(_ltv(1, body))
            for k in keys:
                c.sendall(self.tensors[k].tobytes())
        except (ConnectionError, OSError):
            pass
        finally:
            c.close()

    def close(self):
        self.srv.close()


def test_shared_state_fetch_from_reference_distributor(monkeypatch):
    """A late joiner (revision 0) fetches 6 outdated tensors from a distributor that speaks only the reference's S2C
    bytes (_ReferenceDistributor, advertised as the shared-state address of the peer that holds revision 3). The
    joiner first tries the same-host IPC request (forced: PCCL_SS_IPC_PROTOCOL=1), which the reference distributor
    refuses by closing the connection, then requests the keys over PCCL_SS_STREAMS = 4 parallel connections: every
    request is reference bytes (checked against the reference serialization), every key is requested exactly once,
    and the joiner ends with the exact tensors, hash-verified, at revision 3."""
    import numpy as np
    import torch

    import pccl_amd as pccl
    from pccl_amd.utils import run_threaded_peers
    monkeypatch.setenv("PCCL_SS_IPC_PROTOCOL", "1")
    monkeypatch.setenv("PCCL_SS_STREAMS", "4")
    sizes = [1 << 20, 3, 70_001, 1 << 16, 12_345, 5]
    truth = {f"layer{k}.w": (np.arange(n, dtype=np.float32) * (k + 1) % 97) for k, n in enumerate(sizes)}
    dist = _ReferenceDistributor(truth, revision=3)

    def kwargs(rank):  # the holder of revision 3: its shared-state address is the reference distributor
        return {"advertised_shared_state_port": dist.port} if rank == 0 else {}

    def fn(rank, comm):
        ts = {k: torch.from_numpy(v.copy()) if rank == 0 else torch.zeros(len(v)) for k, v in truth.items()}
        st = pccl.SharedState([pccl.TensorInfo.from_torch(t, k) for k, t in ts.items()])
        st.revision = 3 if rank == 0 else 0
        # the holder only sends, the joiner only receives: the election does not depend on the order of the votes
        info = comm.sync_shared_state(st, strategy=pccl.SharedStateSyncStrategy.SEND_ONLY if rank == 0 else
                                      pccl.SharedStateSyncStrategy.RECEIVE_ONLY)
        return {k: t.numpy().copy() for k, t in ts.items()}, info.rx_bytes, st.revision

    try:
        with local_master() as addr:
            res = run_threaded_peers(2, fn, address=addr, comm_kwargs=kwargs)
    finally:
        dist.close()
    got, rx, rev = res[1]
    assert rev == 3 and rx == sum(v.nbytes for v in truth.values())
    for k, v in truth.items():
        assert np.array_equal(got[k], v), k
    assert dist.refused == 1  # the IPC extension request, closed like a reference distributor does
    requested = sorted(k for keys, _ in dist.requests for k in keys)
    assert requested == sorted(truth) and len(dist.requests) == 4
    for keys, payload in dist.requests:  # reference C2SPacketRequestSharedState bytes
        assert payload == len(keys).to_bytes(8, "big") + b"".join(_ref_str(k) for k in keys)
