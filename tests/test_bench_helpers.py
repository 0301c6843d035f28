"""bench.py's host-side helpers (no GPU): per-phase stripe sizing from the node's CPU share, the CPU-mask switch of
the latency phases and the per-peer CCD groups."""
import os
import types

import bench


def _job(world, a_pool=0):
    j = bench.Job.__new__(bench.Job)  # no torch / GPU setup
    j.a = types.SimpleNamespace(pool=a_pool)
    j.world = world
    j.auto_pool = a_pool <= 0
    return j


def test_pool_for_splits_the_node_cpu_share(monkeypatch):
    monkeypatch.setattr(bench, "_cpu_quota", lambda: 16.0)
    j1 = _job(1)
    # one GPU, 16 CPUs: 8 peers x 2, 4 x 4, 2 x 8 stripes (the measured optimum), never above 8
    assert [j1.pool_for(p) for p in (8, 4, 2, 1)] == [2, 4, 8, 8]
    # ranks share the node's quota: 8 ranks x 1 peer -> 2 stripes each, not 16 // 1
    assert _job(8).pool_for(1) == 2
    monkeypatch.setattr(bench, "_cpu_quota", lambda: 128.0)
    assert _job(8).pool_for(1) == 8 and _job(2).pool_for(4) == 8
    monkeypatch.setattr(bench, "_cpu_quota", lambda: 4.0)
    assert _job(8).pool_for(1) == 1  # at least one connection
    assert _job(1, a_pool=3).pool_for(8) == 3  # explicit --pool wins


def test_full_cpu_mask_restores_the_thread_mask(monkeypatch):
    own = os.sched_getaffinity(0)
    if len(own) < 2:
        return
    narrow = {min(own)}
    os.sched_setaffinity(0, narrow)
    try:
        monkeypatch.setenv("PCCL_BENCH_FULL_CPUS", ",".join(map(str, sorted(own))))
        with bench._full_cpu_mask():
            assert os.sched_getaffinity(0) == own
        assert os.sched_getaffinity(0) == narrow
        monkeypatch.delenv("PCCL_BENCH_FULL_CPUS")
        with bench._full_cpu_mask():  # nothing recorded: the mask stays as it is
            assert os.sched_getaffinity(0) == narrow
    finally:
        os.sched_setaffinity(0, own)


def test_peer_cpu_groups_off_by_default_and_disjoint(monkeypatch):
    monkeypatch.delenv("PCCL_BENCH_PEER_CCD", raising=False)
    assert bench._peer_cpu_groups(8) is None
    monkeypatch.setenv("PCCL_BENCH_PEER_CCD", "1")
    assert bench._peer_cpu_groups(1) is None
    groups = bench._peer_cpu_groups(2)
    if groups is None:  # fewer L3 domains than peers on this host
        return
    assert len(groups) == 2 and all(groups) and not (groups[0] & groups[1])
    assert groups[0] | groups[1] <= os.sched_getaffinity(0)


def test_full_cpu_mask_ccd_narrows_to_one_l3_domain(monkeypatch):
    own = os.sched_getaffinity(0)
    monkeypatch.delenv("PCCL_BENCH_FULL_CPUS", raising=False)
    with bench._full_cpu_mask(ccd=True):
        inside = os.sched_getaffinity(0)
    assert os.sched_getaffinity(0) == own
    assert inside <= own and min(own) in inside


def test_per_rank_diag_models_pcie_and_dram():
    """extra.per_rank: measured staging bytes next to the ring model (per peer D2H = S, H2D = 2(W-1)/W S) and the host
    DRAM estimate (2 x socket tx + PCIe bytes) per op."""
    S, P = 1 << 30, 8
    wire = 2 * (P - 1) / P * S
    ring = {"t": 0.25, "per_rank": [
        {"rank": r, "gpu": r, "peers": 2, "tx": 2 * wire, "rx": 2 * wire, "cpu_cores": 3.0, "cpu_by_thread": {},
         "pcie": {"h2d": 2 * wire, "d2h": 2 * S}} for r in range(4)]}
    rows = bench._per_rank_diag(ring, S, P)
    assert len(rows) == 4 and [r["rank"] for r in rows] == [0, 1, 2, 3]
    r0 = rows[0]
    assert r0["model_pcie_d2h_GB"] == round(2 * S / 1e9, 3) and r0["pcie_d2h_GB"] == r0["model_pcie_d2h_GB"]
    assert r0["model_pcie_h2d_GB"] == round(2 * wire / 1e9, 3) == r0["pcie_h2d_GB"]
    dram = 2 * 2 * wire + 2 * wire + 2 * S
    assert r0["host_dram_est_GB"] == round(dram / 1e9, 2)
    assert r0["host_dram_est_GBps"] == round(dram / 0.25 / 1e9, 1)
    # a rank without staging counters (e.g. an older library) still reports its socket bytes
    ring["per_rank"][1]["pcie"] = None
    assert "pcie_h2d_GB" not in bench._per_rank_diag(ring, S, P)[1]


def test_parse_cpulist():
    assert bench._parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert bench._parse_cpulist("5") == {5}


def test_numa_bind_to_the_gpus_node(monkeypatch):
    """Each process binds to its GPU's NUMA node (by PCI address), unless PCCL_BENCH_NUMA_BIND=0."""
    if not os.path.exists("/sys/devices/system/node/node0/cpulist"):
        return
    own = os.sched_getaffinity(0)
    monkeypatch.setattr(bench, "_gpu_numa_node_child", lambda local_rank=0: 0)
    monkeypatch.delenv("PCCL_BENCH_NUMA_BIND", raising=False)
    try:
        with open("/sys/devices/system/node/node0/cpulist") as f:
            node0 = bench._parse_cpulist(f.read())
        res = bench._numa_bind()
        if node0 & own:
            assert res == {"numa_node": 0, "cpus": len(node0 & own)}
            assert os.sched_getaffinity(0) == node0 & own
        monkeypatch.setenv("PCCL_BENCH_NUMA_BIND", "0")
        assert bench._numa_bind() is None
    finally:
        os.sched_setaffinity(0, own)


def test_config_tcp_mask_modes(monkeypatch):
    own = os.sched_getaffinity(0)
    monkeypatch.setenv("PCCL_BENCH_FULL_CPUS", ",".join(map(str, sorted(own))))
    monkeypatch.setenv("PCCL_BENCH_CONFIG_MASK", "full")
    assert bench._config_tcp_mask() is None
    monkeypatch.setenv("PCCL_BENCH_CONFIG_MASK", "spread")
    assert bench._config_tcp_mask() == own
    monkeypatch.setenv("PCCL_BENCH_CONFIG_MASK", "numa")
    monkeypatch.setattr(bench, "_gpu_numa_node_child", lambda: -1)
    assert bench._config_tcp_mask() == own  # node unknown: the spread
    monkeypatch.setattr(bench, "_gpu_numa_node_child", lambda: 0)
    m = bench._config_tcp_mask()
    assert m and m <= own
    monkeypatch.delenv("PCCL_BENCH_FULL_CPUS")
    assert bench._config_tcp_mask() is None  # no spread applied
    with bench._cpu_mask({min(own)}):
        assert os.sched_getaffinity(0) == {min(own)}
    assert os.sched_getaffinity(0) == own


def test_pool_reserve_nothing_is_a_no_op():
    import pccl_amd as pccl
    pccl.memory.reserve_staging()  # zero counts: nothing leased, success


def test_phase_ranks_path_preflight_and_sys_cores(monkeypatch):
    """extra.per_rank_phases: per rank and phase, the reduce paths its peers took, the pre-flight probes that ran in the
    phase (counter deltas) and the kernel CPU per socket throughput."""
    import pccl_amd as pccl
    monkeypatch.setattr(pccl.memory, "ipc_buffer_stats", lambda: {"preflight_passed": 3, "preflight_failed": 1})
    j = bench.Job.__new__(bench.Job)
    j.rank, j.gpu, j.dist = 0, 0, None
    ring = pccl.ReducePath.DEVICE_RING.value
    # two peers of this rank: 2 s window, 4 GB sent each, 3 s of kernel CPU in the process
    res = [{"main": (2.0, 4e9, 4e9, ring, 5.0, 3.0)}, {"main": (2.0, 4e9, 4e9, ring, 5.0, 3.0)}]
    rec = bench._phase_ranks(j, "device_ring", res, 0.25, {"preflight_passed": 2, "preflight_failed": 1})
    assert rec["phase"] == "device_ring" and rec["ms_per_op"] == 250.0
    (r,) = rec["per_rank"]
    assert r["paths"] == ["DEVICE_RING"] and r["peers"] == 2
    assert r["preflight_passed"] == 1 and r["preflight_failed"] == 0
    assert r["socket_tx_GBps"] == 4.0 and r["sys_cores"] == 1.5
    assert r["sys_cores_per_socket_GBps"] == round(1.5 / 4.0, 3)
    # no socket traffic (xGMI): no ratio
    res = [{"main": (2.0, 0, 0, pccl.ReducePath.DEVICE_IPC.value, 1.0, 0.1)}]
    r = bench._phase_ranks(j, "ipc", res, 0.01, {})["per_rank"][0]
    assert r["sys_cores_per_socket_GBps"] is None and r["socket_tx_GBps"] is None
