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
    monkeypatch.setenv("PCCL_XGMI_CAPABLE", "1")  # peers that would take the xGMI path (this host may lack a GPU)
    from pccl_amd.utils import free_port
    port = free_port()
    master = pccl.MasterNode(f"127.0.0.1:{port}")
    master.run()

    tables = []

    def fn(rank, comm):
        t0 = time.perf_counter()
        comm.optimize_topology()
        dt = time.perf_counter() - t0
        if rank == 0:  # while every peer is still registered (leaving peers drop their edges)
            tables.append(master.bandwidth_table())
        x = torch.full((1000,), float(rank + 1))
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)
        return dt, float(x[0])

    try:
        res = run_threaded_peers(3, fn, address=f"127.0.0.1:{port}", timeout=120)
    finally:
        master.interrupt()
        master.await_termination()
    table = tables[0]
    assert all(r[1] == 6.0 for r in res)
    assert max(r[0] for r in res) < 8.0, res
    assert len(table) == 6 and all(t[3] == 1e6 for t in table), table


def test_optimize_topology_same_host_tcp_pairs_are_measured(monkeypatch):
    """Same-host peers that cannot use xGMI (PCCL_DISABLE_IPC=1: their ring runs over loopback TCP) are benchmarked
    like remote pairs, so the bandwidth store holds measured values rather than the fixed xGMI-class constant
    (reference ccoip_client_handler.cpp:640-736 measures every ordered pair)."""
    monkeypatch.setenv("PCCL_DISABLE_IPC", "1")
    monkeypatch.setenv("PCCL_BENCHMARK_MILLIS", "150")
    monkeypatch.setenv("PCCL_NUM_BENCHMARK_CONNECTIONS", "2")
    monkeypatch.delenv("PCCL_SAME_HOST_MBPS", raising=False)
    monkeypatch.delenv("PCCL_XGMI_CAPABLE", raising=False)
    from pccl_amd.utils import free_port
    port = free_port()
    master = pccl.MasterNode(f"127.0.0.1:{port}")
    master.run()

    tables = []

    def fn(rank, comm):
        comm.optimize_topology()
        if rank == 0:
            tables.append(master.bandwidth_table())
        x = torch.full((1000,), float(rank + 1))
        comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)
        return float(x[0])

    try:
        res = run_threaded_peers(3, fn, address=f"127.0.0.1:{port}", timeout=120)
    finally:
        master.interrupt()
        master.await_termination()
    table = tables[0]
    assert all(r == 6.0 for r in res)
    assert len(table) == 6, table  # every ordered pair
    assert all(0 < t[3] < 1e6 for t in table), table  # measured loopback throughput, not the constant
