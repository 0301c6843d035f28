"""Shared-state synchronisation: hash-popularity election, partial transfers, strategies, late joiners.

Reference behaviour: src/pccl.cpp:545-621 (pcclSynchronizeSharedState), ccoip_master_handler.cpp:595-791 (election),
python/tests/end_to_end/mnist_ddp (late-joining peer catches up).
"""
import threading
import time

import numpy as np
import pytest
import torch

import pccl_amd as pccl
from pccl_amd.utils import local_master, peer_ports, run_threaded_peers

S = pccl.SharedStateSyncStrategy


def _state(tensors, allow=()):
    return pccl.SharedState([pccl.TensorInfo.from_torch(t, name, allow_content_inequality=name in allow)
                             for name, t in tensors.items()])


@pytest.mark.parametrize("ipc_protocol", [False, True])
def test_popular_state_wins(ipc_protocol, monkeypatch):
    """ipc_protocol: the same-host request extension (C2SRequestSharedStateIpc) is forced on; without a GPU the
    distributor answers every entry in stream mode, so the byte accounting is identical."""
    if ipc_protocol:
        monkeypatch.setenv("PCCL_SS_IPC_PROTOCOL", "1")
    world, n = 3, 100_000

    def fn(rank, comm):
        w = torch.full((n,), 0.0 if rank == 0 else 7.0)
        b = torch.arange(17, dtype=torch.float64)
        st = _state({"w": w, "b": b})
        st.revision = 0
        info = comm.sync_shared_state(st)
        first = (w.clone(), info.tx_bytes, info.rx_bytes)
        st.revision = 1
        info2 = comm.sync_shared_state(st)
        return first, (info2.tx_bytes, info2.rx_bytes), st.revision

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for (w, tx, rx), (tx2, rx2), _ in res:
        assert torch.all(w == 7.0)
        assert tx2 == 0 and rx2 == 0
    assert res[0][0][2] == n * 4  # only the outdated tensor moved, exactly once
    assert sum(r[0][1] for r in res) == n * 4


def test_only_mismatching_keys_are_transferred():
    world = 3

    def fn(rank, comm):
        ts = {f"t{k}": torch.full((1000 + k,), float(k)) for k in range(5)}
        if rank == 1:
            ts["t3"].fill_(-1.0)
        st = _state(ts)
        info = comm.sync_shared_state(st)
        return {k: v.clone() for k, v in ts.items()}, info.rx_bytes

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    assert [r[1] for r in res] == [0, 1003 * 4, 0]
    for s, _ in res[1:]:
        for k in s:
            assert torch.equal(s[k], res[0][0][k])


def test_mixed_strategies_kick_non_enforcing_peer():
    """ENFORCE_POPULAR is all-or-nothing (reference ccoip_master_handler.cpp:702-720)."""
    def fn(rank, comm):
        x = torch.full((10,), float(rank))
        st = _state({"x": x})
        try:
            comm.sync_shared_state(st, S.ENFORCE_POPULAR if rank == 0 else S.SEND_ONLY)
            return "ok"
        except pccl.PCCLError:
            return "kicked"

    with local_master() as addr:
        res = run_threaded_peers(2, fn, address=addr)
    assert res[1] == "kicked"


def test_allow_content_inequality_is_not_synced():
    def fn(rank, comm):
        a = torch.full((64,), float(rank))
        b = torch.full((64,), 5.0)
        st = _state({"a": a, "b": b}, allow=("a",))
        info = comm.sync_shared_state(st)
        return a.clone(), info.rx_bytes

    with local_master() as addr:
        res = run_threaded_peers(2, fn, address=addr)
    assert torch.all(res[0][0] == 0.0) and torch.all(res[1][0] == 1.0)
    assert res[0][1] == 0 and res[1][1] == 0


def test_receive_only_gets_state():
    def fn(rank, comm):
        x = np.full(1000, 3.0 if rank == 0 else 9.0, dtype=np.float32)
        st = pccl.SharedState([pccl.TensorInfo.from_numpy(x, "x")])
        comm.sync_shared_state(st, S.SEND_ONLY if rank == 0 else S.RECEIVE_ONLY)
        return x.copy()

    with local_master() as addr:
        res = run_threaded_peers(2, fn, address=addr)
    assert np.all(res[0] == 3.0) and np.all(res[1] == 3.0)


def test_late_joiner_catches_up():
    """Two peers train for a few steps (revision advances); a third joins and receives the current state."""
    n = 50_000
    ports = peer_ports(3)
    out = {}
    errors = []
    joined = threading.Event()
    done = threading.Event()

    def trainer(rank, addr):
        try:
            c = pccl.Communicator(addr, 0, **ports[rank])
            c.connect(n_attempts=10)
            w = torch.zeros(n)
            st = _state({"w": w})
            step, it = 0, 0
            while not done.is_set() and step < 2000:
                it += 1
                # a freshly accepted peer skips its first pending check: the peers that accepted it already
                # performed this iteration's vote (same loop shape as the reference's mnist_peer.py:263-273)
                if it > 1 and c.are_peers_pending():
                    c.update_topology()
                ws = c.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
                if ws < 2:
                    time.sleep(0.01)
                    continue
                st.revision = step
                c.sync_shared_state(st)
                w += 1.0  # "optimizer step"
                g = torch.ones(n)
                c.all_reduce(g, g, op=pccl.ReduceOp.SUM, tag=0)
                step += 1
                if ws == 3:
                    out[rank] = (step, w.clone())
                    break
                time.sleep(0.005)
            c.destroy()
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    def joiner(addr):
        try:
            c = pccl.Communicator(addr, 0, **ports[2])
            c.connect(n_attempts=30)
            joined.set()
            w = torch.zeros(n)
            st = _state({"w": w})
            st.revision = 0
            info = c.sync_shared_state(st)
            out["joiner"] = (w.clone(), info.rx_bytes, st.revision)
            w += 1.0
            g = torch.ones(n)
            c.all_reduce(g, g, op=pccl.ReduceOp.SUM, tag=0)
            out["joiner_g"] = g.clone()
            c.destroy()
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    with local_master() as addr:
        ts = [threading.Thread(target=trainer, args=(r, addr), daemon=True) for r in range(2)]
        for t in ts:
            t.start()
        time.sleep(1.0)
        j = threading.Thread(target=joiner, args=(addr,), daemon=True)
        j.start()
        for t in ts + [j]:
            t.join(timeout=120)
        done.set()
    assert not errors, errors
    w_join, rx, rev = out["joiner"]
    assert rx == n * 4
    assert torch.all(w_join == w_join[0]) and w_join[0].item() >= 1.0
    assert torch.all(out["joiner_g"] == 3.0)
    # the joiner adopted the revision of the run it joined
    assert rev == out[0][0] - 1
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][1], w_join + 1.0)


def test_concurrent_control_plane_call_is_refused():
    """A control-plane call (update_topology) while another thread of the same communicator is inside one
    (a shared-state sync waiting for its peer) fails with INVALID_USAGE instead of interleaving two master dialogues.
    The reference asserts such calls stay on one thread (THREAD_GUARD, ccoip_client_state.cpp:56,85,93)."""
    go = threading.Event()

    def fn(rank, comm):
        x = np.full(1000, float(rank), dtype=np.float32)
        st = pccl.SharedState([pccl.TensorInfo.from_numpy(x, "x")])
        if rank == 1:
            go.wait(30)
            comm.sync_shared_state(st)
            return None
        out = {}
        t = threading.Thread(target=lambda: out.setdefault("info", comm.sync_shared_state(st)))
        t.start()
        time.sleep(0.5)  # the sync is now waiting on the master for peer 1
        try:
            comm.update_topology()
            refused = None
        except pccl.PCCLError as e:
            refused = e.result
        finally:
            go.set()
        t.join(30)
        return refused, "info" in out

    with local_master() as addr:
        res = run_threaded_peers(2, fn, address=addr)
    assert res[0] == (pccl.Result.INVALID_USAGE, True)


@pytest.mark.parametrize("streams", ["1", "3"])
def test_outdated_keys_over_parallel_streams(streams, monkeypatch):
    """PCCL_SS_STREAMS: the outdated keys are fetched over that many connections at once (each an ordinary request
    for a size-balanced subset of the keys); contents, byte accounting and revision are the same as over one."""
    monkeypatch.setenv("PCCL_SS_STREAMS", streams)
    world = 3
    sizes = [100_000, 3, 50_000, 7, 20_000, 1]

    def fn(rank, comm):
        ts = {f"t{k}": torch.full((n,), float(k + 1)) for k, n in enumerate(sizes)}
        if rank == 2:  # the outdated peer: every key differs
            for t in ts.values():
                t.fill_(-5.0)
        st = _state(ts)
        st.revision = 0 if rank == 2 else 4
        info = comm.sync_shared_state(st)
        return {k: v.clone() for k, v in ts.items()}, info.rx_bytes, st.revision

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    state, rx, rev = res[2]
    assert rx == 4 * sum(sizes) and rev == 4
    for k, n in enumerate(sizes):
        assert torch.all(state[f"t{k}"] == float(k + 1))
