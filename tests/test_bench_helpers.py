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
