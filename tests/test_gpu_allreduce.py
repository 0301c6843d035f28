"""All-reduce of HIP device tensors on an MI355X: xGMI IPC path, device ring path, quantized, shared state.

Multi-peer cases share cuda:0 (the GPU box has one GPU); the IPC path is exercised both between threads of one
process and between two processes (real hipIpc export/open).
"""
import json
import os
import subprocess
import time

import pytest
import torch

import pccl_amd as pccl
from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, run_threaded_peers, spawn_python

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(world, fn):
    with local_master() as addr:
        return run_threaded_peers(world, fn, address=addr, timeout=180)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.float16])
@pytest.mark.parametrize("disable_ipc", [False, True])
def test_device_all_reduce_two_peers(hip, dtype, disable_ipc, monkeypatch):
    if disable_ipc:
        monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    n = (1 << 22) + 5
    gen = [torch.Generator().manual_seed(k) for k in range(2)]
    inputs = [torch.randn(n, generator=g).to(dtype) for g in gen]
    expect = (inputs[0].float() + inputs[1].float()).to(dtype)

    def fn(rank, comm):
        x = inputs[rank].to(hip)
        y = torch.empty_like(x)
        info = comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
        torch.cuda.synchronize()
        return y.cpu(), info, comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    res = _run(2, fn)
    want_path = pccl.ReducePath.DEVICE_RING if disable_ipc else pccl.ReducePath.DEVICE_IPC
    for y, info, path in res:
        assert path == want_path.value
        assert torch.equal(y, expect)


def test_device_avg_three_peers_in_place(hip):
    n = 1_000_003

    def fn(rank, comm):
        x = torch.full((n,), float(3 * rank), device=hip)
        comm.all_reduce(x, x, op=pccl.ReduceOp.AVG, tag=0)
        torch.cuda.synchronize()
        return x.cpu()

    for y in _run(3, fn):
        assert torch.all(y == 3.0)


@pytest.mark.parametrize("disable_ipc", [False, True])
def test_device_concurrent_tags(hip, disable_ipc, monkeypatch):
    if disable_ipc:
        monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    n, k = 1 << 20, 6

    def fn(rank, comm):
        xs = [torch.full((n,), float(rank + j), device=hip, dtype=torch.bfloat16) for j in range(k)]
        ys = [torch.empty_like(x) for x in xs]
        hs = [comm.all_reduce_async(xs[j], ys[j], op=pccl.ReduceOp.SUM, tag=j) for j in range(k)]
        for h in hs:
            ok, _, _ = h.wait()
            assert ok
        torch.cuda.synchronize()
        return [y.float().cpu() for y in ys]

    for ys in _run(2, fn):
        for j, y in enumerate(ys):
            assert torch.all(y == float(1 + 2 * j))


@pytest.mark.parametrize("disable_ipc", [False, True])
def test_device_zero_length(hip, disable_ipc, monkeypatch):
    """Empty ops on HBM tensors: a null pointer (torch.empty(0)) on one peer, a non-null zero-length slice on the
    others; every peer runs the protocol, no buffer is touched, and a real op follows on the same ring."""
    if disable_ipc:
        monkeypatch.setenv("PCCL_DISABLE_IPC", "1")

    def fn(rank, comm):
        base = torch.ones(16, device=hip)
        x = torch.empty(0, device=hip) if rank == 0 else base[:0]
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)
        y = torch.empty_like(base)
        comm.all_reduce(base, y, op=pccl.ReduceOp.SUM, tag=1)
        torch.cuda.synchronize()
        return base.cpu(), y.cpu()

    for base, y in _run(3, fn):
        assert base.tolist() == [1.0] * 16 and y.tolist() == [3.0] * 16


@pytest.mark.parametrize("world,inplace,op", [(3, True, "sum"), (4, False, "avg"), (2, True, "max")])
def test_device_ring_pipelined_large(hip, world, inplace, op, monkeypatch):
    """Device TCP ring with many pieces per stripe and several stripes per step (1 MiB copies, 4 stripes, uneven
    chunks): copy-engine staging, cross-stream waits and next-step payload staging must give exact results; the second
    op reuses pooled staging buffers and events."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    monkeypatch.setenv("PCCL_DEVICE_PIECE_BYTES", str(1 << 20))
    monkeypatch.setenv("PCCL_STRIPE_MIN_BYTES", str(1 << 20))
    n = 9_000_011
    base = (torch.arange(n, dtype=torch.int64) % 31).float()  # every partial sum < 256: exact in bf16
    inputs = [(base + 7 * r).to(torch.bfloat16) for r in range(world)]
    stack = torch.stack([x.float() for x in inputs])
    if op == "sum":
        expect = stack.sum(0)
    elif op == "avg":
        expect = stack.sum(0) / world
    else:
        expect = stack.max(0).values
    expect = expect.to(torch.bfloat16)
    rop = {"sum": pccl.ReduceOp.SUM, "avg": pccl.ReduceOp.AVG, "max": pccl.ReduceOp.MAX}[op]

    def fn(rank, comm):
        x = inputs[rank].to(hip)
        y = x if inplace else torch.empty_like(x)
        for tag in range(2):  # second op reuses pooled staging buffers and events
            if tag:
                x.copy_(inputs[rank].to(hip))
            comm.all_reduce(x, y, op=rop, tag=tag)
        torch.cuda.synchronize()
        return y.cpu(), comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, timeout=180, comm_kwargs={"p2p_connection_pool_size": 4})
    for y, path in res:
        assert path == pccl.ReducePath.DEVICE_RING.value
        assert torch.equal(y, expect)


def test_device_ring_mixed_pool_sizes(hip, monkeypatch):
    """Neighbours with different P2P connection pool sizes (1 / 3 / 2 stripes) and chunks that are no multiple of the
    staging piece: a TX stripe of the next step then spans several RX stripes of this one, and the send-ahead
    pipeline must send no byte before it has been received and reduced (advisor round 2, high)."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    monkeypatch.setenv("PCCL_DEVICE_PIECE_BYTES", str(1 << 20))
    monkeypatch.setenv("PCCL_STRIPE_MIN_BYTES", str(1 << 20))
    world, n = 3, 9_000_011
    pools = [1, 3, 2]
    base = (torch.arange(n, dtype=torch.int64) % 29).float()
    inputs = [(base * (r + 1) + r).to(torch.bfloat16) for r in range(world)]
    expect = torch.stack([x.float() for x in inputs]).sum(0).to(torch.bfloat16)

    def fn(rank, comm):
        x = inputs[rank].to(hip)
        y = torch.empty_like(x)
        for tag in range(3):  # later ops reuse pooled staging buffers, events and the connections' sink queues
            comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag)
        torch.cuda.synchronize()
        return y.cpu(), comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, timeout=180,
                                 comm_kwargs=lambda r: {"p2p_connection_pool_size": pools[r]})
    for y, path in res:
        assert path == pccl.ReducePath.DEVICE_RING.value
        assert torch.equal(y, expect)


def _mixed_session(world, inputs, qopt, op=pccl.ReduceOp.SUM, pool=2):
    """One session, three ops in one ring order: every peer on host memory (tag 0), peer 0 on host memory and the
    others on HBM (tag 1), every peer on HBM (tag 2). Returns per rank [(result, tx, rx, path)] of the three ops."""
    def fn(rank, comm):
        out = []
        for tag in range(3):
            on_gpu = tag == 2 or (tag == 1 and rank != 0)
            x = inputs[rank].to(hip_dev() if on_gpu else "cpu")
            y = torch.empty_like(x)
            info = comm.all_reduce(x, y, op=op, tag=tag, quantization_options=qopt)
            if on_gpu:
                torch.cuda.synchronize()
            out.append((y.cpu(), info.tx_bytes, info.rx_bytes, comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)))
        return out

    with local_master() as addr:
        return run_threaded_peers(world, fn, address=addr, timeout=240, comm_kwargs={"p2p_connection_pool_size": pool})


def hip_dev():
    return torch.device("cuda:0")


@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_device_ring_random_bit_identical(hip, world, dtype, monkeypatch):
    """Random data (rounding order matters) on the pipelined device ring at 4 and 8 peers: every peer ends with the
    same bits, and those bits equal the host ring's (CPU tensors, same session and ring order) and a mixed ring's
    where one peer holds CPU tensors and the others HBM tensors on the same wire protocol."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    monkeypatch.setenv("PCCL_DEVICE_PIECE_BYTES", str(1 << 20))
    monkeypatch.setenv("PCCL_STRIPE_MIN_BYTES", str(1 << 20))
    n = 3_000_017
    inputs = [torch.randn(n, generator=torch.Generator().manual_seed(90 + r)).to(dtype) for r in range(world)]
    res = _mixed_session(world, inputs, None, op=pccl.ReduceOp.AVG if dtype == torch.float32 else pccl.ReduceOp.SUM)
    ref = res[0][0][0]
    exact = torch.stack([x.double() for x in inputs]).sum(0)
    if dtype == torch.float32:
        exact = exact / world
    tol = {torch.bfloat16: 0.05, torch.float16: 0.01, torch.float32: 1e-5}[dtype]
    assert (ref.double() - exact).abs().max().item() <= tol * (1 + exact.abs().max().item())
    host, dev = pccl.ReducePath.HOST_RING.value, pccl.ReducePath.DEVICE_RING.value
    for rank, ops in enumerate(res):
        assert [o[3] for o in ops] == [host, host if rank == 0 else dev, dev]
        for y, *_ in ops:
            assert torch.equal(y, ref)


@pytest.mark.parametrize("qdtype,algo", [(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX),
                                         (pccl.DataType.INT8, pccl.QuantizationAlgorithm.ZERO_POINT_SCALE),
                                         (pccl.DataType.FLOAT8_E5M2, pccl.QuantizationAlgorithm.MIN_MAX)])
def test_device_quantized_matches_host_ring(hip, qdtype, algo, monkeypatch):
    """Quantized ring, host memory vs mixed vs HBM in one session (one ring order: a quantized result depends on the
    partial sums that get quantized): identical results and wire bytes on every peer and every op, over several
    pieces per step and uneven chunks. The device ring folds every payload's min / max from the de-quantize kernels'
    partials except the first reduce-scatter step's."""
    from pccl_amd.ops import kernels as K
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    monkeypatch.setenv("PCCL_QUANT_PIECE_BYTES", str(1 << 20))
    world, n = 4, 3_000_017
    inputs = [torch.randn(n, generator=torch.Generator().manual_seed(60 + r)).bfloat16() for r in range(world)]
    s0 = K.quant_minmax_stats()
    res = _mixed_session(world, inputs, pccl.QuantizationOptions(qdtype, algo))
    s1 = K.quant_minmax_stats()
    ref = res[0][0]
    for ops in res:
        for y, tx, rx, _ in ops:
            assert torch.equal(y, ref[0])
        assert len({(o[1], o[2]) for o in ops}) == 1, ops
    # device peers: 3 in the mixed op, 4 in the all-HBM op; per peer and lane: world - 1 folded payloads + 1 pass
    peers = (world - 1) + world
    assert {k: s1[k] - s0[k] for k in s0} == {"folds": peers * (world - 1), "passes": peers}


@pytest.mark.parametrize("lanes", ["1", "2", "3"])
@pytest.mark.parametrize("qdtype", [pccl.DataType.UINT8, pccl.DataType.FLOAT8_E4M3])
def test_device_quantized_all_reduce(hip, qdtype, lanes, monkeypatch):
    """Quantized device ring, 1-3 lanes (PCCL_QUANT_LANES; a lane needs >= 8 MiB of wire bytes per chunk): result
    within the quantization bound, identical on every peer, fewer wire bytes than fp32."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")  # quantization applies to the ring (wire) path
    monkeypatch.setenv("PCCL_QUANT_LANES", lanes)
    monkeypatch.setenv("PCCL_QUANT_PIECE_BYTES", str(4 << 20))
    n = (3 << 24) + 3
    inputs = [torch.randn(n, generator=torch.Generator().manual_seed(40 + r)) for r in range(3)]

    def fn(rank, comm):
        x = inputs[rank].to(hip)
        y = torch.empty_like(x)
        info = comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0, quantization_options=pccl.QuantizationOptions(
            qdtype, pccl.QuantizationAlgorithm.MIN_MAX))
        torch.cuda.synchronize()
        return y.cpu(), info

    res = _run(3, fn)
    expect = inputs[0] + inputs[1] + inputs[2]
    for y, info in res:
        assert torch.equal(y, res[0][0])
        assert info.tx_bytes < n * 4
        err = (y - expect).abs()
        bound = 3 * (max(float(t.max() - t.min()) for t in inputs) / 255) if qdtype == pccl.DataType.UINT8 else None
        if bound is not None:
            assert err.max().item() <= bound
        else:
            # partial sums are re-quantized at every ring hop: error scales with sum(|x_r|), not |sum(x_r)|
            mag = inputs[0].abs() + inputs[1].abs() + inputs[2].abs()
            assert (err <= mag * 0.15 + 0.05).all()


def test_device_shared_state(hip):
    n = (1 << 22) + 1

    def fn(rank, comm):
        w = torch.full((n,), 1.0 if rank == 1 else 2.0, device=hip)
        m = torch.arange(1000, device=hip, dtype=torch.bfloat16)
        st = pccl.SharedState([pccl.TensorInfo.from_torch(w, "w"), pccl.TensorInfo.from_torch(m, "m")])
        info = comm.sync_shared_state(st)
        torch.cuda.synchronize()
        return w.cpu(), info.rx_bytes

    res = _run(3, fn)
    for w, _ in res:
        assert torch.all(w == 2.0)
    assert [r[1] for r in res] == [0, n * 4, 0]


@pytest.mark.parametrize("ipc_mode", ["safe", "fast"])
@pytest.mark.parametrize("mode", ["zero_copy", "inplace", "mixed", "shareable", "shareable_inplace"])
def test_two_process_ipc(hip, mode, ipc_mode):
    """Two processes on cuda:0 exchange device buffers (the intra-node xGMI path). safe (default): staged VMM
    buffers shared as fds; fast: hipIpc handles, out-of-place ops export the caller's buffers (zero-copy, interior
    offsets), in-place ops a staged comm buffer. shareable*: the tensors live in fd-shareable memory
    (pccl_amd.memory) and are handed to the peer directly in either mode."""
    def extra(r):
        e = ["--inplace"] if mode in ("inplace", "shareable_inplace") or (mode == "mixed" and r == 1) else []
        return e + (["--shareable"] if mode.startswith("shareable") else [])
    with local_master() as addr:
        procs = [spawn_python([os.path.join(HERE, "workers", "allreduce_peer.py"), addr, "2", str(r), "--n",
                               str((1 << 24) + 1), "--dtype", "bf16", "--device", "cuda:0", "--steps", "3",
                               *extra(r)], env={"PCCL_IPC_MODE": ipc_mode},
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = communicate_all(procs, 240, DIAG_SIGNALS)
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
        assert len(lines) == 3
        for ln in lines:
            expect = float(1 + 2 + 2 * ln["step"])
            assert ln["lo"] == ln["hi"] == expect
            assert ln["path"] == pccl.ReducePath.DEVICE_IPC.value
        b = lines[-1]["ipc_bufs"]
        if mode.startswith("shareable") or (mode == "zero_copy" and ipc_mode == "fast"):
            assert b["direct_out"] == 3 and b["staged_out"] == 0, b
        if mode == "shareable" or (mode == "zero_copy" and ipc_mode == "fast"):
            assert b["direct_in"] == 3 and b["staged_in"] == 0, b
        if ipc_mode == "safe" and mode in ("zero_copy", "inplace", "mixed"):  # plain torch memory: staged
            assert b["direct_in"] == 0 and b["direct_out"] == 0, b


@pytest.mark.parametrize("world", [2, 3])
def test_ipc_preflight_rehearsal(hip, world):
    """The cross-GPU pre-flight (first op of an arena whose peers span several GPUs: a 256-byte probe written into
    every peer's output through the push kernels' mappings, read back after a barrier) forced on one GPU with
    PCCL_IPC_PREFLIGHT=2: it passes once per process, and that first op and every later one stay exact on the IPC
    path. This is the 1-GPU rehearsal of what an 8-GPU node runs first."""
    with local_master() as addr:
        procs = [spawn_python([os.path.join(HERE, "workers", "allreduce_peer.py"), addr, str(world), str(r), "--n",
                               str((1 << 20) + 3), "--dtype", "bf16", "--device", "cuda:0", "--steps", "4"],
                              env={"PCCL_IPC_PREFLIGHT": "2"}, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(world)]
        outs = communicate_all(procs, 240, DIAG_SIGNALS)
    tri = world * (world + 1) // 2
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
        assert len(lines) == 4 and not any("error" in ln for ln in lines), lines
        for ln in lines:
            assert ln["lo"] == ln["hi"] == float(tri + world * ln["step"])
            assert ln["path"] == pccl.ReducePath.DEVICE_IPC.value
        b = lines[-1]["ipc_bufs"]
        assert b["preflight_passed"] == 1 and b["preflight_failed"] == 0, b


@pytest.mark.parametrize("gib", [1.25, 2.5])
def test_two_process_ipc_large(hip, gib):
    """Ops whose staged comm buffers / user allocations exceed 1-2 GiB: staged buffers are built from 1 GiB segments
    and kernels run per segment piece; user allocations above kIpcMaxExport are staged (PyTorch's ROCm 7.0 runtime
    never returns from hipIpcOpenMemHandle for >= 2 GiB allocations). Rank 1 runs in place (staged input)."""
    n = int(gib * (1 << 30)) // 2 + 3
    with local_master() as addr:
        procs = [spawn_python([os.path.join(HERE, "workers", "allreduce_peer.py"), addr, "2", str(r), "--n", str(n),
                               "--dtype", "bf16", "--device", "cuda:0", "--steps", "2",
                               *(["--inplace"] if r == 1 else [])],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = communicate_all(procs, 200, DIAG_SIGNALS)
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
        assert len(lines) == 2
        for ln in lines:
            assert ln["lo"] == ln["hi"] == float(1 + 2 + 2 * ln["step"])
            assert ln["path"] == pccl.ReducePath.DEVICE_IPC.value


@pytest.mark.parametrize("inplace", [(False, True), (True, False), (True, True)])
@pytest.mark.parametrize("no_zc", [False, True])
def test_device_ipc_modes(hip, inplace, no_zc, monkeypatch):
    """Zero-copy and staged peers mixed in one op; interior (offset) views of larger allocations."""
    if no_zc:
        monkeypatch.setenv("PCCL_IPC_NO_ZERO_COPY", "1")
    n = 3_000_001
    big = [torch.randn(n + 1000, device=hip) for _ in range(2)]
    orig = [b[777:777 + n].cpu() for b in big]
    expect_all = (big[0][777:777 + n] + big[1][777:777 + n]).clone()  # before any peer reduces in place
    torch.cuda.synchronize()

    def fn(rank, comm):
        x = big[rank][777:777 + n]  # interior view: the IPC handle maps the allocation base
        expect = expect_all
        y = x if inplace[rank] else torch.empty_like(x)
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
        torch.cuda.synchronize()
        return y.cpu(), expect.cpu(), comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    for rank, (y, expect, path) in enumerate(_run(2, fn)):
        assert path == pccl.ReducePath.DEVICE_IPC.value
        bad = (y != expect).nonzero().flatten()
        assert bad.numel() == 0, dict(rank=rank, wrong=bad.numel(), first=bad[:4].tolist(), last=bad[-4:].tolist(),
                                      zeros=int((y[bad] == 0).sum()), own_input=int((y[bad] == orig[rank][bad]).sum()),
                                      peer_input=int((y[bad] == orig[1 - rank][bad]).sum()))


def test_shareable_memory_module(hip):
    """pccl_amd.memory: tensors allocated in the shareable pool resolve to a live VMM allocation (interior views
    included); ordinary tensors do not; the pool serves repeated allocations."""
    before = pccl.memory.live_bytes()
    with pccl.shareable_memory(hip):
        a = torch.arange(1 << 22, device=hip, dtype=torch.float32)
        b = torch.empty(3_000_001, device=hip, dtype=torch.bfloat16)
    c = torch.empty(1 << 20, device=hip)
    assert pccl.memory.is_shareable(a) and pccl.memory.is_shareable(b) and pccl.memory.is_shareable(a[12345:])
    assert not pccl.memory.is_shareable(c) and not pccl.memory.is_shareable(torch.empty(4))
    assert pccl.memory.live_bytes() > before
    assert torch.equal(a.cpu(), torch.arange(1 << 22, dtype=torch.float32))
    d = pccl.memory.empty(1000, dtype=torch.float16, device=hip)
    assert pccl.memory.is_shareable(d) and d.dtype == torch.float16


def test_threaded_peers_skip_staging(hip):
    """Peers that are threads of one process cannot die independently: safe mode hands them the caller's buffers
    directly (no copy-in / copy-out), in-place ops still stage the input (abort backup)."""
    n = 1 << 20
    s0 = pccl.memory.ipc_buffer_stats()

    def fn(rank, comm):
        x = torch.full((n,), float(rank + 1), device=hip)
        y = torch.empty_like(x)
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=1)
        torch.cuda.synchronize()
        return float(y.min()), float(y.max()), float(x.min()), float(x.max())

    for lo, hi, xlo, xhi in _run(2, fn):
        assert lo == hi == 3.0 and xlo == xhi == 3.0
    s1 = pccl.memory.ipc_buffer_stats()
    d = {k: s1[k] - s0[k] for k in ("direct_in", "direct_out", "staged_in", "staged_out")}
    assert d == {"direct_in": 2, "direct_out": 4, "staged_in": 2, "staged_out": 0}, d


def test_shareable_memory_concurrent_threads(hip):
    """Peer threads of one process allocate in the shareable pool at the same time (PyTorch allows one thread per
    MemPool context: the context serialises them) and reduce over the xGMI path with direct buffers."""
    n = 1 << 20

    def fn(rank, comm):
        with pccl.shareable_memory(hip):
            with pccl.shareable_memory(hip):  # nested: no-op
                x = torch.full((n,), float(rank + 1), device=hip)
            y = torch.empty_like(x)
        assert pccl.memory.is_shareable(x) and pccl.memory.is_shareable(y)
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
        torch.cuda.synchronize()
        return float(y.min()), float(y.max())

    for lo, hi in _run(4, fn):
        assert lo == hi == 10.0


@pytest.mark.parametrize("n", [1, 1000, 65536, 300_000])
def test_device_ring_small_messages(hip, n, monkeypatch):
    """Device tensors over the TCP ring below PCCL_SMALL_ALLREDUCE_BYTES (1 MiB): one D2H, host all-gather +
    ring-order reduce, one H2D; 300k fp32 (1.2 MB) takes the pipelined ring. Exact, identical on every peer."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")

    def fn(rank, comm):
        x = torch.arange(n, device=hip, dtype=torch.float32) % 7 + rank
        y = torch.empty_like(x)
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
        comm.all_reduce(x, x, op=pccl.ReduceOp.MAX, tag=1)
        torch.cuda.synchronize()
        return y.cpu(), x.cpu(), comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    res = _run(3, fn)
    base = torch.arange(n, dtype=torch.float32) % 7
    for y, x, path in res:
        assert path == pccl.ReducePath.DEVICE_RING.value
        assert torch.equal(y, 3 * base + 3) and torch.equal(x, base + 2)


@pytest.mark.parametrize("n", [1, 3, 5, 4097])
@pytest.mark.parametrize("quant", [False, True])
def test_device_ring_fewer_elements_than_peers(hip, n, quant, monkeypatch):
    """The pipelined device ring (small-message path off) with chunks of zero or one element: empty reduce-scatter /
    all-gather steps must neither hang nor touch memory outside the buffer; quantized and plain."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    monkeypatch.setenv("PCCL_SMALL_ALLREDUCE_BYTES", "0")
    world = 4
    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if quant else None

    def fn(rank, comm):
        x = (torch.arange(n, device=hip, dtype=torch.float32) % 5 + rank).bfloat16()
        y = torch.full((n + 64,), -7.0, device=hip, dtype=torch.bfloat16)  # guard elements after the output
        for tag in range(2):
            comm.all_reduce(x, y[:n], op=pccl.ReduceOp.SUM, tag=tag, quantization_options=qopt)
        torch.cuda.synchronize()
        return y.cpu()

    res = _run(world, fn)
    base = (torch.arange(n, dtype=torch.float32) % 5)
    expect = (world * base + sum(range(world))).bfloat16()
    for y in res:
        assert torch.all(y[n:] == -7.0)
        assert torch.equal(y[:n], res[0][:n])
        if not quant:
            assert torch.equal(y[:n], expect)
        else:
            assert (y[:n].float() - expect.float()).abs().max() <= 0.5


@pytest.mark.parametrize("disable_ipc", [False, True])
@pytest.mark.parametrize("blocking", [False, True])
def test_stream_ordered_all_reduce_with_queued_producer(hip, disable_ipc, blocking, monkeypatch):
    """pcclxAllReduce[Async]OnStream: the input's producer is still queued (a ~150 ms spin kernel, then the fill)
    when all_reduce(_async) is called on its stream; the async call returns at once (no host synchronisation of the
    stream), the op waits for the producer itself, and the result is exact."""
    if disable_ipc:
        monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    n = (1 << 20) + 3
    cycles = int(3e8)  # ~150 ms at MI355X clocks

    def fn(rank, comm):
        s = torch.cuda.Stream(hip)
        x = torch.zeros(n, device=hip, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        outs = []
        for it in range(3):
            with torch.cuda.stream(s):
                torch.cuda._sleep(cycles)
                x.fill_(float(rank + 1 + it))
            t0 = time.perf_counter()
            if blocking:
                comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=it, stream=s)
                call = time.perf_counter() - t0
            else:
                h = comm.all_reduce_async(x, y, op=pccl.ReduceOp.SUM, tag=it, stream=s)
                call = time.perf_counter() - t0
                ok, _, _ = h.wait()
                assert ok
            outs.append((call, time.perf_counter() - t0, float(y.float().min()), float(y.float().max())))
        return outs, comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    res = _run(2, fn)
    for outs, path in res:
        assert path == (pccl.ReducePath.DEVICE_RING if disable_ipc else pccl.ReducePath.DEVICE_IPC).value
        for it, (call, total, lo, hi) in enumerate(outs):
            assert lo == hi == 3 + 2 * it, outs  # (1 + it) + (2 + it)
            assert total > 0.05, outs  # the op did wait for the queued producer
            if not blocking:
                assert call < 0.05, outs  # ... without the caller waiting for it


def test_ddp_overlap_launches_without_stream_sync(hip):
    """DataParallel(overlap=True) starts bucket all-reduces from the backward hooks as stream-ordered ops (no thread
    synchronises the backward stream) and the averaged gradients are exact."""
    import copy

    from pccl_amd.parallel import DataParallel
    torch.manual_seed(0)
    base = torch.nn.Sequential(*[torch.nn.Linear(256, 256) for _ in range(6)])

    def fn(rank, comm):
        model = copy.deepcopy(base).to(hip)
        dp = DataParallel(model, comm, bucket_bytes=256 * 1024, overlap=True)
        x = torch.full((32, 256), float(rank + 1), device=hip)
        model(x).sum().backward()
        res = dp.sync_gradients()
        torch.cuda.synchronize()
        grads = [p.grad.detach().clone() for p in model.parameters()]
        dp.close()
        return res.ok, grads

    outs = _run(2, fn)
    # reference: the mean of both peers' gradients, computed locally
    ref = []
    for r in range(2):
        model = copy.deepcopy(base).to(hip)
        model(torch.full((32, 256), float(r + 1), device=hip)).sum().backward()
        ref.append([p.grad.detach().clone() for p in model.parameters()])
    for ok, grads in outs:
        assert ok
        for g, a, b in zip(grads, ref[0], ref[1]):
            torch.testing.assert_close(g, (a + b) / 2, rtol=1e-5, atol=1e-5)


def test_device_ring_staging_bounded_by_segment(hip):
    """2 peer processes x 8 GiB bf16, in place, TCP device ring: the op runs as 64 pipelined segments of 128 MiB ring
    chunks (PCCL_SEGMENT_CHUNK_MIB), so each peer's pinned staging peaks at 6 x 128 MiB, not 6 x 4 GiB; exact sums."""
    worker = os.path.join(HERE, "workers", "allreduce_peer.py")
    n = 4 << 30  # bf16 elements: 8 GiB per peer
    with local_master() as addr:
        ps = [spawn_python([worker, addr, "2", str(r), "--device", "cuda:0", "--dtype", "bf16", "--n", str(n),
                            "--const", "--inplace", "--steps", "2", "--pool", "4"],
                           env={"PCCL_DISABLE_IPC": "1"}, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
              for r in range(2)]
        outs = communicate_all(ps, 280, DIAG_SIGNALS)
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(ln) for ln in o.splitlines() if ln.startswith("{")]
        assert len(lines) == 2 and not any(ln.get("bad") for ln in lines), lines
        assert all(ln["path"] == pccl.ReducePath.DEVICE_RING.value for ln in lines), lines
        pinned_peak = max(ln["staging"]["pinned"]["peak"] for ln in lines)
        assert pinned_peak <= (1 << 30), lines[-1]["staging"]


def test_ipc_op_above_arena_size_runs_as_sub_ops(hip):
    """2 threaded peers x 20 GiB bf16 (above one arena op's 16 GiB of staged segments): the op runs on the xGMI path
    as consecutive sub-ops (Client::ipc_reduce_segmented) instead of dropping to the TCP ring; exact sums, path IPC.
    Then a second op in place with a non-uniform input: every element is restored or reduced correctly across the
    sub-op boundary."""
    n = 10 << 30  # bf16 elements: 20 GiB per buffer

    def fn(rank, comm):
        x = torch.full((n,), float(rank + 1), device=hip, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
        torch.cuda.synchronize()
        p1 = comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)
        ok1 = bool((y == 3.0).all())
        del y
        # in place, values that differ per 1 Mi block (the sub-op boundary at 8 Gi elements is not block aligned)
        rows = x.view(-1, 1 << 20)
        pat = (torch.arange(rows.shape[0], device=hip) % 7).to(torch.bfloat16)
        rows.copy_(pat.unsqueeze(1).expand_as(rows))
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=1)
        torch.cuda.synchronize()
        want = (pat.float() * 2).to(torch.bfloat16).unsqueeze(1)
        ok2 = all(bool((rows[k:k + 1024] == want[k:k + 1024]).all()) for k in range(0, rows.shape[0], 1024))
        return p1, ok1, comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH), ok2

    res = _run(2, fn)
    for p1, ok1, p2, ok2 in res:
        assert ok1 and ok2, res
        assert p1 == p2 == pccl.ReducePath.DEVICE_IPC.value, res


@pytest.mark.gpu
def test_device_ring_reference_framing_staging_bounded(hip):
    """The same 2 x 8 GiB bf16 in-place op with one peer speaking the reference protocol (PCCL_WIRE=reference): the
    op runs in the reference framing, which cannot be segmented (every ring step carries its whole 4 GiB chunk on one
    connection), so the device ring moves each step in 64 MiB pieces through fixed staging rings
    (device_ring_reference_pieces): exact sums, framing 2 (reference) reported, pinned staging <= 1 GiB per peer
    (was 6 x 4 GiB)."""
    worker = os.path.join(HERE, "workers", "allreduce_peer.py")
    n = 4 << 30  # bf16 elements: 8 GiB per peer
    with local_master() as addr:
        ps = [spawn_python([worker, addr, "2", str(r), "--device", "cuda:0", "--dtype", "bf16", "--n", str(n),
                            "--const", "--inplace", "--steps", "2", "--pool", "2", "--report-framing"],
                           env=dict({"PCCL_DISABLE_IPC": "1"}, **({"PCCL_WIRE": "reference"} if r == 0 else {})),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
              for r in range(2)]
        outs = communicate_all(ps, 280, DIAG_SIGNALS)
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(ln) for ln in o.splitlines() if ln.startswith("{")]
        assert len(lines) == 2 and not any(ln.get("bad") for ln in lines), lines
        assert all(ln["path"] == pccl.ReducePath.DEVICE_RING.value and ln["framing"] == 2 for ln in lines), lines
        pinned_peak = max(ln["staging"]["pinned"]["peak"] for ln in lines)
        assert pinned_peak <= (1 << 30), lines[-1]["staging"]


def test_device_ring_pcie_bytes_match_model(hip, monkeypatch):
    """pcclxPcieStats (bench.py extra.per_rank): a device-ring op queues exactly the ring's staging traffic - per peer
    S device->host (the step-0 payload and every reduced next payload) and 2(W-1)/W S host->device (every received
    piece) - for W = 3 threaded peers of this process, 8 MiB + 3 elements each (chunks of unequal size)."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    n = (4 << 20) + 3
    es = 2
    state = {}

    def fn(rank, comm):
        x = torch.full((n,), float(rank + 1), device=hip, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)  # warm-up (pools, connections)
        torch.cuda.synchronize()
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=1)  # barrier: every peer finished the warm-up op
        torch.cuda.synchronize()
        if rank == 0:
            state["before"] = pccl.memory.pcie_stats()
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=2)
        torch.cuda.synchronize()
        comm.all_reduce(x[:1], y[:1], op=pccl.ReduceOp.SUM, tag=3)  # (small path: host all-gather, 2 + 2 bytes)
        torch.cuda.synchronize()
        return float(y[:1].float().item()), comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    res = _run(3, fn)
    after = pccl.memory.pcie_stats()
    assert all(v == 6.0 for v, _ in res)
    S = n * es
    d2h = after["d2h"] - state["before"]["d2h"]
    h2d = after["h2d"] - state["before"]["h2d"]
    # three peers' op 2 (+ the 1-element small-path op 3: one element each way per peer), plus whatever of op 1 was
    # still being counted when peer 0 sampled (at most its last steps: bounded by the op itself)
    assert 3 * S + 3 * es <= d2h <= 2 * (3 * S) + 3 * es, (d2h, S)
    assert 3 * (4 * S // 3) <= h2d <= 2 * 3 * (4 * S // 3) + 3 * es + 16, (h2d, S)


def test_reserved_staging_serves_the_first_device_ring_op(hip, monkeypatch):
    """pccl.memory.reserve_device_ring_staging (pcclxPoolReserve) fills the pools with what a device-ring op of that
    size leases, so the op itself allocates nothing (benchmarks/fault_tolerance.py runs it next to a replacement's
    connect()). Two threaded peers share the process's pools: reserved for both."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    C = (48 << 20) + 4096  # one ring chunk (bytes), a size no other test leases
    n = C  # bf16 elements per peer: 2 C bytes, W = 2 -> chunks of C bytes
    pccl.memory.reserve_device_ring_staging(2 * C, 2, device=hip, peers=2)
    st = pccl.memory.staging_pool_stats()
    assert st["pinned"]["cached"] >= 12 * C and st["device"]["cached"] >= 6 * C, st
    state = {}

    def fn(rank, comm):
        x = torch.full((n,), float(rank + 1), device=hip, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        comm.all_reduce(x[:1024], y[:1024], op=pccl.ReduceOp.SUM, tag=0)  # connections up, both peers here
        torch.cuda.synchronize()
        if rank == 0:
            state["before"] = pccl.memory.staging_pool_stats()
        comm.all_reduce(x[:1024], y[:1024], op=pccl.ReduceOp.SUM, tag=1)  # (rank 0 sampled before the big op)
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=2)
        torch.cuda.synchronize()
        return float(y.float().min().item()), float(y.float().max().item()), \
            comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    res = _run(2, fn)
    after = pccl.memory.staging_pool_stats()
    assert all(r[0] == r[1] == 3.0 for r in res), res
    assert all(r[2] == pccl.ReducePath.DEVICE_RING.value for r in res), res
    for pool in ("pinned", "device"):
        assert after[pool]["allocs"] == state["before"][pool]["allocs"], (pool, state["before"], after)


def test_device_ring_stripe_bound_with_uneven_chunks(hip, monkeypatch):
    """Chunks of 2 MiB + 4 bytes and 2 MiB with 256 KiB stripes over 4 connections: the larger chunk rounds to 3
    stripes, the smaller one to 4. The op's connection group and sender threads are sized by the stripe bound of its
    largest step, which covers every step (sizing them by the largest step's own stripe count left a stripe unsent)."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    monkeypatch.setenv("PCCL_STRIPE_MIN_BYTES", str(256 << 10))
    n = 2 * 524288 + 1  # fp32: chunks of 524289 and 524288 elements

    def fn(rank, comm):
        x = torch.full((n,), float(rank + 1), device=hip)
        y = torch.empty_like(x)
        for tag in range(2):
            comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag)
        torch.cuda.synchronize()
        return float(y.min()), float(y.max()), comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    with local_master() as addr:
        res = run_threaded_peers(2, fn, address=addr, timeout=120, comm_kwargs={"p2p_connection_pool_size": 4})
    for lo, hi, path in res:
        assert path == pccl.ReducePath.DEVICE_RING.value
        assert lo == hi == 3.0
