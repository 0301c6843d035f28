"""Shared-state distribution scenarios, ported from the reference's end-to-end suite
(/root/reference/ccoip/tests/end_to_end/test_shared_state_distribution.cpp, one test per TEST() there) to threaded
peers of this implementation. Values are 1 KiB uint8 entries unless noted; every assertion mirrors the reference's
EXPECTs (tx/rx byte accounting, final contents, kicks)."""
import threading
import time

import pytest
import torch

import pccl_amd as pccl
from pccl_amd.utils import local_master, peer_ports, wait_for_world

S = pccl.SharedStateSyncStrategy
VS = 1024


def _state(entries, revision=0, allow=()):
    st = pccl.SharedState([pccl.TensorInfo.from_torch(t, k, allow_content_inequality=k in allow)
                           for k, t in entries.items()])
    st.revision = revision
    return st


def _sync(comm, st, strategy=S.ENFORCE_POPULAR):
    """(ok, tx, rx); ok False if the master kicked this peer."""
    try:
        info = comm.sync_shared_state(st, strategy)
        return True, info.tx_bytes, info.rx_bytes
    except pccl.PCCLError:
        return False, 0, 0


def run_peers(groups, fn, timeout=90, stagger=None):
    """One thread per peer; peer r joins peer group groups[r]. fn(rank, comm) runs once every peer is admitted.
    stagger[r]: seconds to wait before peer r's fn starts (the reference's 'this client hits the master first')."""
    n = len(groups)
    results, errors = [None] * n, [None] * n
    ports = peer_ports(n)
    with local_master() as addr:
        comms = [None] * n

        def body(r):
            try:
                c = pccl.Communicator(addr, groups[r], **ports[r])
                comms[r] = c
                c.connect(n_attempts=20)
                wait_for_world(c, n, timeout=timeout)
                if stagger:
                    time.sleep(stagger[r])
                results[r] = fn(r, c)
            except BaseException as e:  # noqa: BLE001 - re-raised below
                errors[r] = e

        ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout)
        assert not any(t.is_alive() for t in ts), "peers hung"
        for e in errors:
            if e is not None:
                raise e
        for c in comms:
            if c is not None:
                c.destroy()
    return results


def _filled(v):
    return torch.full((VS,), v, dtype=torch.uint8)


def test_basic_tie_two_peers():
    """TestBasic: a 1:1 tie; exactly one full transfer in either direction, contents equal afterwards."""
    vals = [_filled(42), _filled(0)]

    def fn(r, c):
        return _sync(c, _state({"key1": vals[r]}))

    res = run_peers([0, 0], fn, stagger=[0, 0.5])
    assert all(ok for ok, _, _ in res)
    assert sorted((tx, rx) for _, tx, rx in res) in ([(0, VS), (VS, 0)],)
    assert torch.equal(vals[0], vals[1])


def test_no_sync_identical_shared_state():
    def fn(r, c):
        return _sync(c, _state({"key1": _filled(42)}))

    assert run_peers([0, 0], fn) == [(True, 0, 0)] * 2


def test_partial_sync_partially_dirty_state():
    """Two keys, only key2 differs: exactly VS bytes move."""
    vals = [{"key1": _filled(42), "key2": _filled(43)}, {"key1": _filled(42), "key2": _filled(0)}]

    def fn(r, c):
        return _sync(c, _state(vals[r]))

    res = run_peers([0, 0], fn)
    assert sum(tx for _, tx, _ in res) == VS and sum(rx for _, _, rx in res) == VS
    assert torch.equal(vals[0]["key2"], vals[1]["key2"])


def test_popular_hash_prevalence_unpopular_first():
    """TestPopularHashPrevelance: the unpopular peer votes first and must still receive the popular content."""
    vals = [_filled(0), _filled(42), _filled(42)]

    def fn(r, c):
        return _sync(c, _state({"key1": vals[r]}))

    res = run_peers([0, 0, 0], fn, stagger=[0, 0.5, 0.5])
    assert res[0] == (True, 0, VS)
    assert sum(tx for _, tx, _ in res[1:]) == VS and all(rx == 0 for _, _, rx in res[1:])
    assert all(torch.equal(v, _filled(42)) for v in vals)


def test_popular_hash_prevalence_multiple_keys():
    """Many keys; peer 0 differs in some of them and receives exactly those."""
    n_keys = 8
    base = {f"k{i}": _filled(i + 1) for i in range(n_keys)}
    vals = [{k: v.clone() for k, v in base.items()} for _ in range(3)]
    for i in (1, 4, 6):
        vals[0][f"k{i}"].fill_(200)

    def fn(r, c):
        return _sync(c, _state(vals[r]))

    res = run_peers([0, 0, 0], fn, stagger=[0, 0.3, 0.3])
    assert res[0] == (True, 0, 3 * VS)
    for k in base:
        assert torch.equal(vals[0][k], base[k])


@pytest.mark.parametrize("different_keys", [False, True])
@pytest.mark.parametrize("concurrent", [False, True])
def test_peer_groups_identical_within_group(different_keys, concurrent):
    """TestNoSyncIdenticalSharedStateMultiplePeerGroups(+DifferentKeys, +Concurrent): state differs across groups but
    is identical within each group, so no bytes move; groups never compare masks or contents with each other."""
    groups = [0, 0, 1, 1]

    def fn(r, c):
        g = groups[r]
        key = ("key1" if g == 1 else "key2") if different_keys else "key1"
        return _sync(c, _state({key: _filled(42 + g)}))

    res = run_peers(groups, fn, stagger=None if concurrent else [0, 0, 0.5, 0.5])
    assert res == [(True, 0, 0)] * 4


def test_multi_step_advancement():
    """Identical updates every step: revisions advance by one, nothing moves."""
    def fn(r, c):
        v = _filled(0)
        st = _state({"key1": v})
        out = []
        for step in range(1, 6):
            v.fill_(42 + step)
            st.revision = step
            out.append(_sync(c, st))
        return out

    for steps in run_peers([0, 0], fn):
        assert steps == [(True, 0, 0)] * 5


@pytest.mark.parametrize("advance_contents", [False, True])
def test_drag_along(advance_contents):
    """TestDragAlongClient{No,With}AdvancedStateContents: two leaders advance the revision (and optionally the
    contents) every step; a follower never updates its own state or revision. It receives the leaders' state at the
    first step (and at every step if the contents advance) and its revision follows the leaders'."""
    steps = 4
    leaders = [_filled(42), _filled(42)]
    follower = _filled(0)

    def fn(r, c):
        out = []
        if r < 2:
            st = _state({"key1": leaders[r]})
            for step in range(steps):
                if advance_contents:
                    leaders[r].fill_(42 + step)
                st.revision = step
                out.append(_sync(c, st))
        else:
            st = _state({"key1": follower})
            for step in range(steps):
                out.append(_sync(c, st) + (st.revision, follower.clone()))
        return out

    res = run_peers([0, 0, 0], fn)
    for step in range(steps):
        ok, tx, rx, rev, content = res[2][step]
        assert ok and tx == 0
        assert rev == step
        expect_rx = VS if (step == 0 or advance_contents) else 0
        assert rx == expect_rx, (step, rx)
        assert torch.equal(content, _filled(42 + step if advance_contents else 42))
        # exactly one leader served the follower whenever it was outdated
        assert sum(res[L][step][1] for L in range(2)) == expect_rx
        assert all(res[L][step][2] == 0 for L in range(2))


def test_one_increment_rule_violation():
    """TestOneIncrementRuleViolationSimple: a peer that jumps its revision by two is kicked."""
    def fn(r, c):
        v = _filled(42 if r == 0 else 0)
        st = _state({"key1": v})
        out = []
        for step in range(2):
            st.revision = step * 2 if r == 0 else st.revision
            out.append(_sync(c, st)[0])
        return out

    res = run_peers([0, 0], fn)
    assert res[0][0] is True and res[0][1] is False  # revision 2 after 0: kicked


def test_one_increment_rule_initialization_allows_resume():
    """TestOneIncrementRuleViolationInitialization: the first sync of a run may start at any revision (resume);
    a peer at revision 0 then receives it."""
    v0, v1 = _filled(42), _filled(0)

    def fn(r, c):
        st = _state({"key1": v0 if r == 0 else v1}, revision=13 if r == 0 else 0)
        res = _sync(c, st)
        return res + (st.revision,)

    res = run_peers([0, 0], fn, stagger=[0, 0.5])
    assert res[0][0] and res[1] == (True, 0, VS, 13)
    assert torch.equal(v0, v1)


def test_mask_mismatch_kick():
    """TestSharedStateMaskMismatchKick: two peers establish the key set; a third with a different key is kicked,
    and stays kicked; the others keep syncing."""
    def fn(r, c):
        if r < 2:
            st = _state({"key1": _filled(42)})
            a = _sync(c, st)[0]
            st.revision = 1
            b = _sync(c, st)[0]
            return a, b
        st = _state({"key3": _filled(42)})
        return _sync(c, st)[0], _sync(c, st)[0]

    res = run_peers([0, 0, 0], fn, stagger=[0, 0, 0.5])
    assert res[0] == (True, True) and res[1] == (True, True)
    assert res[2] == (False, False)


def test_concurrent_advancement_within_peer_groups():
    """Two groups advance their own state concurrently for several steps; nothing moves, nothing crosses groups."""
    groups = [0, 0, 1, 1]

    def fn(r, c):
        v = _filled(0)
        st = _state({"key": v})
        out = []
        for step in range(1, 5):
            v.fill_(42 + step + 10 * groups[r])
            st.revision = step
            out.append(_sync(c, st))
        return out

    for steps in run_peers(groups, fn):
        assert steps == [(True, 0, 0)] * 4


def test_concurrent_drag_along_across_peer_groups():
    """Per group: two leaders and a follower; followers of both groups are dragged along by their own group only."""
    groups = [0, 0, 0, 1, 1, 1]
    vals = [_filled(80 + g) if i % 3 < 2 else _filled(0) for i, g in enumerate(groups)]

    def fn(r, c):
        g = groups[r]
        st = _state({f"drag_key_{g}": vals[r]})
        out = []
        for step in range(3):
            if r % 3 < 2:
                vals[r].fill_(90 + g + step)
                st.revision = step
            out.append(_sync(c, st))
        return out

    res = run_peers(groups, fn)
    for r, g in enumerate(groups):
        assert all(ok for ok, _, _ in res[r])
        if r % 3 == 2:
            assert [rx for _, _, rx in res[r]] == [VS] * 3
            assert torch.equal(vals[r], _filled(90 + g + 2))


def test_overlapping_keys_across_peer_groups():
    """The same key name in two groups with different contents: groups are independent, nothing moves."""
    groups = [0, 0, 1, 1]

    def fn(r, c):
        return _sync(c, _state({"shared_key_overlapping": _filled(200 + groups[r])}))

    assert run_peers(groups, fn) == [(True, 0, 0)] * 4


def test_changing_group_membership_between_steps():
    """A third peer joins the group between synchronization steps and catches up without disturbing the others."""
    n_steps = 4
    ports = peer_ports(3)
    out, errors = {}, []
    joined = threading.Event()
    with local_master() as addr:
        def member(r):
            try:
                c = pccl.Communicator(addr, 0, **ports[r])
                c.connect(n_attempts=20)
                wait_for_world(c, 2)
                v = _filled(150)
                st = _state({"key": v})
                res = []
                for step in range(n_steps):
                    if step == 2:  # admit the newcomer between steps
                        deadline = time.time() + 30
                        while c.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE) < 3 and time.time() < deadline:
                            if c.are_peers_pending():
                                c.update_topology()
                            else:
                                time.sleep(0.01)
                    v.fill_(160 + step)
                    st.revision = step
                    res.append(_sync(c, st))
                    if step == 1:
                        joined.set()
                out[r] = res
                c.destroy()
            except BaseException as e:  # noqa: BLE001
                errors.append(e)

        def newcomer():
            try:
                joined.wait(30)
                c = pccl.Communicator(addr, 0, **ports[2])
                c.connect(n_attempts=30)
                v = _filled(0)
                st = _state({"key": v})
                res = []
                for _ in range(2, n_steps):
                    res.append(_sync(c, st) + (st.revision,))
                out[2] = (res, v.clone())
                c.destroy()
            except BaseException as e:  # noqa: BLE001
                errors.append(e)

        ts = [threading.Thread(target=member, args=(r,), daemon=True) for r in range(2)]
        ts.append(threading.Thread(target=newcomer, daemon=True))
        for t in ts:
            t.start()
        for t in ts:
            t.join(90)
    assert not errors, errors
    for r in range(2):
        assert all(ok for ok, _, _ in out[r])
        assert all(rx == 0 for _, _, rx in out[r])
    res, v = out[2]
    assert [x[0] for x in res] == [True, True]
    assert [x[2] for x in res] == [VS, VS]  # the leaders' contents advance every step
    assert [x[3] for x in res] == [2, 3]
    assert torch.equal(v, _filled(160 + n_steps - 1))


def test_both_send_only_different_content_one_kicked():
    vals = [_filled(42), _filled(0)]

    def fn(r, c):
        return _sync(c, _state({"key1": vals[r]}), S.SEND_ONLY)[0]

    res = run_peers([0, 0], fn)
    assert res.count(False) >= 1


@pytest.mark.parametrize("same_content", [False, True])
def test_both_receive_only_kicked(same_content):
    """Nobody puts content up for election: both peers are kicked."""
    def fn(r, c):
        return _sync(c, _state({"key1": _filled(42 if (r == 0 or same_content) else 0)}), S.RECEIVE_ONLY)[0]

    assert run_peers([0, 0], fn) == [False, False]


@pytest.mark.parametrize("others", [[S.RECEIVE_ONLY], [S.SEND_ONLY], [S.SEND_ONLY, S.SEND_ONLY],
                                    [S.SEND_ONLY, S.RECEIVE_ONLY]])
def test_enforce_popular_no_mixing(others):
    """TestEnforcePopularSyncStrategyNoMixingWith*: if one peer enforces popularity, every peer of the group must;
    the others are kicked and the enforcing peer's sync succeeds."""
    strategies = [S.ENFORCE_POPULAR] + others

    def fn(r, c):
        return _sync(c, _state({"key1": _filled(42)}), strategies[r])[0]

    res = run_peers([0] * len(strategies), fn)
    assert res[0] is True and res[1:] == [False] * len(others)


def test_cross_peer_group_local_mixing_local_kick():
    """TestCrossPeerGroupLocalMixingLocalKickWorldSize4PeerGroups2: group 0 mixes enforce-popular with send-only
    (the send-only peer is kicked); group 1 uses send-only on identical content, which is allowed."""
    groups = [0, 0, 1, 1]
    strategies = [S.ENFORCE_POPULAR, S.SEND_ONLY, S.SEND_ONLY, S.SEND_ONLY]

    def fn(r, c):
        return _sync(c, _state({"key1": _filled(42)}), strategies[r])[0]

    assert run_peers(groups, fn) == [True, False, True, True]
