"""Bandwidth-aware ring optimisation (pcclOptimizeTopology): peers benchmark each other, the master solves the ATSP
and rewires the ring; collectives keep working afterwards (reference ccoip_client_handler.cpp:640-736,
topology_optimizer.cpp)."""
import pytest
import torch

import pccl_amd as pccl
from pccl_amd.utils import local_master, run_threaded_peers


@pytest.mark.parametrize("world", [2, 3, 4])
def test_optimize_topology_then_reduce(world, monkeypatch):
    monkeypatch.setenv("PCCL_BENCHMARK_MILLIS", "150")
    monkeypatch.setenv("PCCL_NUM_BENCHMARK_CONNECTIONS", "2")
    monkeypatch.setenv("PCCL_SAME_HOST_MBPS", "0")  # benchmark same-host pairs too (every test peer is local)

    def fn(rank, comm):
        comm.optimize_topology()
        rev = comm.get_attribute(pccl.Attribute.CONNECTION_REVISION)
        x = torch.full((100_000,), float(rank + 1))
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)
        comm.optimize_topology()  # second round: bandwidths known, moonshot / no-op
        y = torch.full((10,), 1.0)
        comm.all_reduce(y, y, op=pccl.ReduceOp.SUM, tag=1)
        return float(x[0]), float(y[0]), rev, comm.get_attribute(pccl.Attribute.RING_RANK)

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, timeout=180)
    assert all(r[0] == world * (world + 1) / 2 and r[1] == world for r in res)
    assert sorted(r[3] for r in res) == list(range(world))  # a valid ring: every position taken once


def test_optimize_topology_same_host_pairs_not_benchmarked(monkeypatch):
    """Pairs on one host (same boot id + hostname) get a fixed xGMI-class cost instead of a 10 s loopback benchmark:
    with the reference defaults (16 connections x 10 s) a 3-peer optimisation would take >= 60 s of benchmarks."""
    import time
    monkeypatch.delenv("PCCL_BENCHMARK_MILLIS", raising=False)
    monkeypatch.delenv("PCCL_SAME_HOST_MBPS", raising=False)

    def fn(rank, comm):
        t0 = time.perf_counter()
        comm.optimize_topology()
        dt = time.perf_counter() - t0
        x = torch.full((1000,), float(rank + 1))
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)
        return dt, float(x[0])

    with local_master() as addr:
        res = run_threaded_peers(3, fn, address=addr, timeout=120)
    assert all(r[1] == 6.0 for r in res)
    assert max(r[0] for r in res) < 8.0, res
