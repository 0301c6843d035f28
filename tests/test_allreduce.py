"""End-to-end all-reduce over the CCoIP ring on the host path: in-process master + threaded peers.

Covers the reference's python/tests/{numpy_only_tests,pytorch_only_tests}/*all_reduce* and
tests/basic_reduce_test scenarios: every op, float/int dtypes, uneven chunking, concurrent tags,
multi-op retry API, numpy buffers and quantized reductions.
"""
import numpy as np
import pytest
import torch

import pccl_amd as pccl
from pccl_amd.utils import local_master, run_threaded_peers


def _peer_tensor(rank, n, dtype):
    g = torch.Generator().manual_seed(100 + rank)
    if dtype.is_floating_point:
        return torch.randn(n, generator=g).to(dtype)
    return torch.randint(-50, 50, (n,), generator=g, dtype=torch.int64).to(dtype)


def _expected(tensors, op):
    acc_dtype = torch.float64 if tensors[0].dtype.is_floating_point else torch.int64
    xs = [t.to(acc_dtype) for t in tensors]
    if op in (pccl.ReduceOp.SUM, pccl.ReduceOp.AVG):
        r = sum(xs[1:], xs[0].clone())
        if op == pccl.ReduceOp.AVG:
            r = r / len(xs) if tensors[0].dtype.is_floating_point else torch.div(r, len(xs), rounding_mode="trunc")
    elif op == pccl.ReduceOp.PROD:
        r = xs[0].clone()
        for x in xs[1:]:
            r = r * x
    elif op == pccl.ReduceOp.MAX:
        r = torch.stack(xs).max(0).values
    else:
        r = torch.stack(xs).min(0).values
    return r


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("op", list(pccl.ReduceOp))
def test_ops_fp32(world, op):
    n = 1025
    inputs = [_peer_tensor(r, n, torch.float32) for r in range(world)]

    def fn(rank, comm):
        out = torch.empty(n)
        info = comm.all_reduce(inputs[rank], out, op=op, tag=0)
        return out, info

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    expect = _expected(inputs, op).float()
    for out, info in res:
        assert info.local_world_size == world
        torch.testing.assert_close(out, expect, rtol=1e-5, atol=1e-5)
    for out, _ in res[1:]:
        assert torch.equal(out, res[0][0]), "peers must agree bit-for-bit"


@pytest.mark.parametrize("dtype", [torch.float64, torch.bfloat16, torch.float16, torch.int32, torch.int64, torch.int8,
                                   torch.uint8])
def test_dtypes_sum(dtype):
    world, n = 3, 4099
    inputs = [_peer_tensor(r, n, dtype) for r in range(world)]
    if dtype == torch.uint8:
        inputs = [t.abs() for t in inputs]

    def fn(rank, comm):
        out = torch.empty(n, dtype=dtype)
        comm.all_reduce(inputs[rank], out, op=pccl.ReduceOp.SUM, tag=0)
        return out

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for out in res[1:]:
        assert torch.equal(out, res[0])
    if dtype.is_floating_point:
        tol = {torch.bfloat16: 5e-2, torch.float16: 5e-3}.get(dtype, 1e-9)
        torch.testing.assert_close(res[0].double(), _expected(inputs, pccl.ReduceOp.SUM), rtol=tol, atol=tol)
    else:
        assert torch.equal(res[0], _expected(inputs, pccl.ReduceOp.SUM).to(dtype))


@pytest.mark.parametrize("n", [1, 2, 3, 7, 1000003])
def test_uneven_sizes(n):
    world = 3

    def fn(rank, comm):
        x = torch.full((n,), float(rank + 1))
        out = torch.empty(n)
        comm.all_reduce(x, out, op=pccl.ReduceOp.SUM, tag=0)
        return out

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for out in res:
        assert torch.all(out == 6.0)


def test_in_place_and_numpy():
    world, n = 2, 333

    def fn(rank, comm):
        x = np.full(n, rank + 1, dtype=np.float32)
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)
        return x

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for x in res:
        assert np.all(x == 3.0)


def test_concurrent_async_tags():
    world, n, n_ops = 3, 10007, 8

    def fn(rank, comm):
        xs = [torch.full((n,), float(rank + 1 + k)) for k in range(n_ops)]
        outs = [torch.empty(n) for _ in range(n_ops)]
        handles = [comm.all_reduce_async(xs[k], outs[k], op=pccl.ReduceOp.SUM, tag=k) for k in range(n_ops)]
        for h in handles:
            ok, status, info = h.wait()
            assert ok, status
        return outs

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for outs in res:
        for k, o in enumerate(outs):
            assert torch.all(o == float(6 + 3 * k)), k


def test_all_reduce_multiple_with_retry():
    world, n, n_ops = 2, 4096, 6

    def fn(rank, comm):
        xs = [torch.full((n,), float(rank + k)) for k in range(n_ops)]
        outs = [torch.empty(n) for _ in range(n_ops)]
        descs = []
        for k in range(n_ops):
            rd = pccl.ReduceDescriptor(n, pccl.ReduceOp.SUM, k,
                                       pccl.ReduceOperandDescriptor(pccl.DataType.FLOAT, pccl.DistributionHint.NONE),
                                       pccl.QuantizationOptions(pccl.DataType.FLOAT, pccl.QuantizationAlgorithm.NONE))
            descs.append(pccl.ReduceOpDescriptor.from_torch(xs[k], outs[k], rd))
        info = comm.all_reduce_multiple_with_retry(descs, max_in_flight=3)
        return outs, info

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for outs, info in res:
        assert info.local_world_size == 2
        for k, o in enumerate(outs):
            assert torch.all(o == float(1 + 2 * k))


def test_bounded_collective_worker_pool():
    """64 concurrent async ops per peer run on at most PCCL_MAX_CONCURRENT_COLLECTIVE_OPS (16) worker threads
    (reference ccoip_client_state.hpp:17-25); the queued ones start as workers free up, in submission order."""
    world, n, n_ops = 2, 2048, 64

    def fn(rank, comm):
        xs = [torch.full((n,), float(rank + k)) for k in range(n_ops)]
        outs = [torch.empty(n) for _ in range(n_ops)]
        hs = [comm.all_reduce_async(xs[k], outs[k], op=pccl.ReduceOp.SUM, tag=k) for k in range(n_ops)]
        for h in hs:
            ok, status, _ = h.wait()
            assert ok, status
        return outs, comm.get_attribute(pccl.Attribute.COLLECTIVE_WORKER_THREADS)

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for outs, workers in res:
        assert 1 <= workers <= 16, workers
        for k, o in enumerate(outs):
            assert torch.all(o == float(1 + 2 * k)), k


_SLIDING = r"""
import json, sys, time, torch
sys.path.insert(0, sys.argv[1])
import pccl_amd as pccl
from pccl_amd.utils import local_master, run_threaded_peers
n_ops, n = 256, 1024
def fn(rank, comm):
    xs = [torch.full((n,), float(rank + k)) for k in range(n_ops)]
    outs = [torch.empty(n) for _ in range(n_ops)]
    descs = []
    for k in range(n_ops):
        rd = pccl.ReduceDescriptor(n, pccl.ReduceOp.SUM, k,
                                   pccl.ReduceOperandDescriptor(pccl.DataType.FLOAT, pccl.DistributionHint.NONE),
                                   pccl.QuantizationOptions(pccl.DataType.FLOAT, pccl.QuantizationAlgorithm.NONE))
        descs.append(pccl.ReduceOpDescriptor.from_torch(xs[k], outs[k], rd))
    t0 = time.perf_counter()
    comm.all_reduce_multiple_with_retry(descs, max_in_flight=8)
    dt = time.perf_counter() - t0
    ok = all(bool(torch.all(outs[k] == float(1 + 2 * k))) for k in range(n_ops))
    return dt, ok
with local_master() as addr:
    res = run_threaded_peers(2, fn, address=addr, timeout=120)
print(json.dumps({"t": max(r[0] for r in res), "ok": all(r[1] for r in res)}))
"""


def test_all_reduce_multiple_sliding_window():
    """256 ops, max_in_flight 8, op 0 is slow (800 ms before it starts), every other op takes >= 20 ms: a batch
    window (or awaiting the oldest op first, as the reference does) stalls all launches behind op 0 (>= 0.8 s +
    31 x 20 ms); the sliding window keeps 7 slots busy meanwhile (~0.8 s + ~0.1 s)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PCCL_FAULT_DELAY="0:800,*:20")
    r = subprocess.run([sys.executable, "-c", _SLIDING, root], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"]
    assert out["t"] < 1.25, out  # stalled scheduling: >= 1.42 s


@pytest.mark.parametrize("qdtype,algo", [(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX),
                                         (pccl.DataType.INT8, pccl.QuantizationAlgorithm.MIN_MAX),
                                         (pccl.DataType.UINT16, pccl.QuantizationAlgorithm.MIN_MAX),
                                         (pccl.DataType.UINT8, pccl.QuantizationAlgorithm.ZERO_POINT_SCALE),
                                         (pccl.DataType.INT32, pccl.QuantizationAlgorithm.ZERO_POINT_SCALE),
                                         (pccl.DataType.UINT64, pccl.QuantizationAlgorithm.ZERO_POINT_SCALE),
                                         (pccl.DataType.INT64, pccl.QuantizationAlgorithm.ZERO_POINT_SCALE)])
def test_quantized_all_reduce(qdtype, algo):
    world, n = 3, 20011
    inputs = [_peer_tensor(r, n, torch.float32) for r in range(world)]

    def fn(rank, comm):
        out = torch.empty(n)
        info = comm.all_reduce(inputs[rank], out, op=pccl.ReduceOp.SUM, tag=0,
                               quantization_options=pccl.QuantizationOptions(qdtype, algo))
        return out, info

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    expect = _expected(inputs, pccl.ReduceOp.SUM).float()
    for out, info in res:
        assert torch.equal(out, res[0][0]), "quantized results must still be identical on every peer"
        span = max(float(t.max() - t.min()) for t in inputs)
        levels = 65535 if qdtype == pccl.DataType.UINT16 else 255
        assert (out - expect).abs().max().item() <= world * span / levels + 1e-4
    # the wire carries the quantized type: ~4x fewer bytes than fp32 for 8-bit
    tx = res[0][1].tx_bytes
    full = n * 4 * 2 * (world - 1) / world
    if qdtype in (pccl.DataType.UINT8, pccl.DataType.INT8):
        assert tx < full / 2


def test_single_peer_too_few_peers():
    """A lone peer gets pcclTooFewPeers (reference src/pccl.cpp:282-285)."""
    def fn(rank, comm):
        x = torch.arange(10, dtype=torch.float32)
        with pytest.raises(pccl.PCCLError) as e:
            comm.all_reduce(x, torch.empty(10), op=pccl.ReduceOp.AVG, tag=0)
        return e.value.result

    with local_master() as addr:
        res = run_threaded_peers(1, fn, address=addr)
    assert res[0] == pccl.Result.TOO_FEW_PEERS


@pytest.mark.parametrize("world,pool", [(2, 4), (3, 3), (3, 8)])
@pytest.mark.parametrize("quant", [False, True])
def test_striped_large_all_reduce(world, pool, quant, monkeypatch):
    """Large chunks are striped over the connection pool (PCCL_STRIPE_MIN_BYTES lowered to exercise uneven plans)."""
    monkeypatch.setenv("PCCL_STRIPE_MIN_BYTES", str(1 << 20))
    n = 3_000_017
    inputs = [_peer_tensor(r, n, torch.float32) for r in range(world)]
    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if quant else None

    def fn(rank, comm):
        out = torch.empty(n)
        comm.all_reduce(inputs[rank], out, op=pccl.ReduceOp.SUM, tag=0, quantization_options=qopt)
        return out

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, comm_kwargs={"p2p_connection_pool_size": pool})
    for out in res[1:]:
        assert torch.equal(out, res[0])
    expect = _expected(inputs, pccl.ReduceOp.SUM).float()
    tol = 3 * world * max(float(t.max() - t.min()) for t in inputs) / 255 if quant else 1e-4
    assert (res[0] - expect).abs().max().item() <= tol


@pytest.mark.parametrize("quant", [False, True])
def test_mixed_pool_sizes_host(quant, monkeypatch):
    """Neighbours with different P2P connection pool sizes (1 / 3 / 2): the two ends of every pool derive the same
    stripe count and connection group for each op from the pool they share, also with several ops in flight."""
    monkeypatch.setenv("PCCL_STRIPE_MIN_BYTES", str(256 << 10))
    world, n, ops = 3, 1_500_007, 4
    pools = [1, 3, 2]
    inputs = [_peer_tensor(r, n, torch.float32) for r in range(world)]
    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if quant else None

    def fn(rank, comm):
        outs = [torch.empty(n) for _ in range(ops)]
        handles = [comm.all_reduce_async(inputs[rank], outs[k], op=pccl.ReduceOp.SUM, tag=k,
                                         quantization_options=qopt) for k in range(ops)]
        assert all(h.wait()[0] for h in handles)
        return outs

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, timeout=120,
                                 comm_kwargs=lambda r: {"p2p_connection_pool_size": pools[r]})
    expect = _expected(inputs, pccl.ReduceOp.SUM).float()
    tol = 3 * world * max(float(t.max() - t.min()) for t in inputs) / 255 if quant else 1e-4
    for k in range(ops):
        for outs in res[1:]:
            assert torch.equal(outs[k], res[0][k])
        assert (res[0][k] - expect).abs().max().item() <= tol


@pytest.mark.parametrize("lanes,inplace", [("1", False), ("2", True), ("3", False)])
def test_quantized_lanes(lanes, inplace, monkeypatch):
    """Quantized all-reduce split into lanes (PCCL_QUANT_LANES, each >= 8 MiB of wire bytes per ring chunk): every
    lane is its own ring on its own data / metadata tags; the result is within the quantization bound, identical on
    every peer, and the wire bytes are the same for any lane count up to the per-step metadata packets."""
    monkeypatch.setenv("PCCL_QUANT_LANES", lanes)
    world, n = 2, (1 << 25) + 7
    inputs = [_peer_tensor(r, n, torch.float32) for r in range(world)]
    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX)

    def fn(rank, comm):
        x = inputs[rank].clone()
        out = x if inplace else torch.empty(n)
        info = comm.all_reduce(x, out, op=pccl.ReduceOp.SUM, tag=5, quantization_options=qopt)
        return out, info.tx_bytes

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, comm_kwargs={"p2p_connection_pool_size": 2})
    nl = int(lanes)
    for out, tx in res:
        assert torch.equal(out, res[0][0])
        payload = n * 2 * (world - 1) // world  # uint8 bytes of the 2(W-1) steps
        assert payload <= tx <= payload + 200 * 2 * (world - 1) * nl, tx  # + one metadata packet per step and lane
    expect = _expected(inputs, pccl.ReduceOp.SUM).float()
    assert (res[0][0] - expect).abs().max().item() <= 3 * world * max(float(t.max() - t.min()) for t in inputs) / 255


@pytest.mark.parametrize("small_limit", [0, 1 << 18])
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int32])
@pytest.mark.parametrize("inplace", [False, True])
def test_small_message_allgather_path(small_limit, world, dtype, inplace, monkeypatch):
    """Ops up to PCCL_SMALL_ALLREDUCE_BYTES take the all-gather + local-reduce path (W-1 hops instead of 2(W-1));
    0 forces the ring. Both must give the same (exact for integer-valued data) sums, bit-identical on every peer,
    for every op incl. AVG, in place or not, and sizes that do not divide by the world."""
    monkeypatch.setenv("PCCL_SMALL_ALLREDUCE_BYTES", str(small_limit))
    n = 1003
    lim = 4 if dtype == torch.bfloat16 else 8  # products of 4 values stay exactly representable in bf16
    inputs = [torch.randint(-lim, lim, (n,), generator=torch.Generator().manual_seed(7 + r)).to(dtype)
              for r in range(world)]
    ops = [pccl.ReduceOp.SUM, pccl.ReduceOp.MAX, pccl.ReduceOp.MIN, pccl.ReduceOp.PROD]
    if dtype.is_floating_point:
        ops.append(pccl.ReduceOp.AVG)

    def fn(rank, comm):
        outs = []
        for k, op in enumerate(ops):
            x = inputs[rank].clone()
            y = x if inplace else torch.empty_like(x)
            info = comm.all_reduce(x, y, op=op, tag=k)
            outs.append((y, info.tx_bytes))
        return outs

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for k, op in enumerate(ops):
        expect = _expected(inputs, op)
        for r in range(world):
            y, tx = res[r][k]
            assert torch.equal(y, res[0][k][0]), "peers must agree bit-for-bit"
            if dtype == torch.bfloat16 and op == pccl.ReduceOp.AVG:
                torch.testing.assert_close(y.double(), expect, rtol=1e-2, atol=1e-2)
            else:
                assert torch.equal(y.double(), expect.double()), (op, y[:8], expect[:8])
            nbytes = n * inputs[0].element_size()
            assert tx == (nbytes * (world - 1) if small_limit else tx), tx  # all-gather sends W-1 whole vectors


def test_small_message_threshold_mismatch_is_agreed():
    """Peers whose PCCL_SMALL_ALLREDUCE_BYTES differ (one would take the all-gather small-message algorithm, the other
    the reduce-scatter ring) must not split the ring between the two: the choice travels as a capability bit of the
    collective initiate that the master ANDs, so both run the same algorithm and the results stay exact."""
    import json
    import os
    import subprocess

    from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, spawn_python
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "workers", "allreduce_peer.py")
    with local_master() as addr:
        ps = [spawn_python([worker, addr, "2", str(r), "--n", "1000", "--steps", "3"],
                           env={"PCCL_SMALL_ALLREDUCE_BYTES": "0" if r == 0 else str(1 << 20)},
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = communicate_all(ps, 120, DIAG_SIGNALS)
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, e[-2000:]
        lines = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
        assert len(lines) == 3 and all("error" not in ln for ln in lines), lines
        for ln in lines:
            assert ln["lo"] == ln["hi"] == float(3 + 2 * ln["step"])


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("quant", [False, True])
def test_zero_length(world, quant):
    """An empty all-reduce is a legal no-op that still runs the protocol on every peer (the reference's ring tests
    include zero-length inputs); the next op on the same communicators works."""
    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if quant else None

    def fn(rank, comm):
        # null data pointers (torch.empty(0)) on rank 0, a non-null zero-length slice elsewhere
        e = torch.empty(0) if rank == 0 else torch.ones(4)[:0]
        info = comm.all_reduce(e, e, op=pccl.ReduceOp.SUM, tag=0, quantization_options=qopt)
        x, out = torch.full((5,), float(rank + 1)), torch.empty(5)
        comm.all_reduce(x, out, op=pccl.ReduceOp.SUM, tag=1)
        return info, out

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for info, out in res:
        assert info.local_world_size == world
        assert quant or info.tx_bytes == 0  # the quantized ring still exchanges its per-step metadata
        assert out.tolist() == [world * (world + 1) / 2] * 5
