"""All-reduce scenarios ported from the reference's end-to-end suite
(/root/reference/ccoip/tests/end_to_end/test_all_reduce.cpp): the typed matrix (10 integer / float types x
Sum/Avg/Min/Max, world sizes 2-4, 2 / 3 / 1025 / 203530 elements, src == dst variants; bf16 / fp16 added here),
and the concurrency rules (no peer admission or shared-state sync while a reduce is in flight, a tag cannot be reused
while its op runs)."""
import threading

import numpy as np
import pytest
import torch

import pccl_amd as pccl
from pccl_amd.utils import local_master, run_threaded_peers

R = pccl.ReduceOp
NP_TYPES = [np.uint8, np.int8, np.int16, np.uint16, np.int32, np.uint32, np.int64, np.uint64, np.float32,
            np.float64]
TORCH_TYPES = [torch.bfloat16, torch.float16]
OPS = [R.SUM, R.AVG, R.MIN, R.MAX]


def _input(rank, n, dtype):
    i = np.arange(n, dtype=np.int64)
    return ((i * (rank + 3)) % 11 + rank).astype(dtype)  # small values: exact in every type, min/max differ


def _expect(world, n, op):
    xs = np.stack([_input(r, n, np.int64) for r in range(world)])
    if op == R.SUM:
        return xs.sum(0).astype(np.float64)
    if op == R.AVG:
        return xs.sum(0) / world
    if op == R.MIN:
        return xs.min(0).astype(np.float64)
    return xs.max(0).astype(np.float64)


@pytest.mark.parametrize("world,n", [(2, 203530), (3, 2), (3, 3), (3, 1025), (4, 2)])
@pytest.mark.parametrize("inplace", [False, True])
def test_typed_matrix(world, n, inplace):
    def fn(rank, comm):
        failures = []
        tag = 0
        for op in OPS:
            exp = _expect(world, n, op)
            for dt in NP_TYPES + TORCH_TYPES:
                if isinstance(dt, torch.dtype):
                    x = torch.from_numpy(_input(rank, n, np.float32)).to(dt)
                    y = x if inplace else torch.empty_like(x)
                    comm.all_reduce(x, y, op=op, tag=tag)
                    got = y.double().numpy()
                    e = exp if op != R.AVG else torch.tensor(exp).to(dt).double().numpy()
                else:
                    x = _input(rank, n, dt)
                    y = x if inplace else np.empty_like(x)
                    comm.all_reduce(x, y, op=op, tag=tag)
                    got = y.astype(np.float64)
                    if op == R.AVG:
                        # integer AVG divides with truncation (reference performAvgFinalization); floats divide
                        e = np.trunc(exp) if np.issubdtype(dt, np.integer) else exp.astype(dt).astype(np.float64)
                    else:
                        e = exp
                tag += 1
                if not np.array_equal(got, e):
                    failures.append((op.name, str(dt)))
        return failures

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, timeout=240)
    assert res == [[]] * world, res


def _two_peers(fn):
    with local_master() as addr:
        return run_threaded_peers(2, fn, address=addr)


def test_no_accept_new_peers_during_concurrent_reduce():
    """TestNoAcceptNewPeersDuringConcurrentReduce: update_topology is refused while an async reduce is in flight."""
    def fn(rank, comm):
        x = np.full(1024, 42 + rank, dtype=np.uint8)
        y = np.zeros_like(x)
        h = comm.all_reduce_async(x, y, op=R.SUM, tag=1)
        with pytest.raises(pccl.PCCLError):
            comm.update_topology()
        ok, _, _ = h.wait()
        return ok, int(y[0])

    assert _two_peers(fn) == [(True, 85), (True, 85)]


def test_no_shared_state_sync_during_concurrent_reduce():
    def fn(rank, comm):
        x = np.full(1024, 42 + rank, dtype=np.uint8)
        y = np.zeros_like(x)
        w = torch.zeros(16)
        h = comm.all_reduce_async(x, y, op=R.SUM, tag=1)
        with pytest.raises(pccl.PCCLError):
            comm.sync_shared_state(pccl.SharedState([pccl.TensorInfo.from_torch(w, "w")]))
        ok, _, _ = h.wait()
        return ok, int(y[0])

    assert _two_peers(fn) == [(True, 85), (True, 85)]


def test_multiple_concurrent_all_reduces():
    """TestMultipleConcurrentAllReduces: distinct tags run concurrently and each lands in its own buffer."""
    def fn(rank, comm):
        xs = [np.full(4096, (rank + 1) * (k + 1), dtype=np.int32) for k in range(6)]
        ys = [np.zeros_like(x) for x in xs]
        hs = [comm.all_reduce_async(x, y, op=R.SUM, tag=100 + k) for k, (x, y) in enumerate(zip(xs, ys))]
        oks = [h.wait()[0] for h in hs]
        return oks, [int(y[0]) for y in ys], all(np.all(y == y[0]) for y in ys)

    for oks, vals, uniform in _two_peers(fn):
        assert all(oks) and uniform
        assert vals == [3 * (k + 1) for k in range(6)]


def test_multiple_concurrent_all_reduces_same_tag_fail():
    """TestMultipleConcurrentAllReducesSameTagFail: a second op with a tag that is still running is rejected."""
    barrier = threading.Barrier(2)

    def fn(rank, comm):
        x1 = np.full(256, 10 * (rank + 1), dtype=np.int32)
        x2 = np.arange(256, dtype=np.int32) * (rank + 1)
        y1, y2 = np.zeros_like(x1), np.zeros_like(x2)
        barrier.wait()
        h = comm.all_reduce_async(x1, y1, op=R.SUM, tag=7)
        with pytest.raises(pccl.PCCLError):
            comm.all_reduce_async(x2, y2, op=R.SUM, tag=7)
        ok, _, _ = h.wait()
        return ok, int(y1[0]), int(y2.sum())

    assert _two_peers(fn) == [(True, 30, 0), (True, 30, 0)]
