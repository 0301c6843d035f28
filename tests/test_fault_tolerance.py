"""Fault tolerance: peers crash mid-run (no clean disconnect), survivors retry and continue; new peers rejoin.

Reference scenarios: python/tests/stress_tests/basic_stress_test (random peer kills / respawns),
BASELINE config 5 ("kill + rejoin 1 of N peers mid-all-reduce"). Every successful all-reduce is checked against
the world size it ran with (x = 1 on every peer => result == world).
"""
import json
import os
import subprocess
import time

import pytest

from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, spawn_python

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "workers", "allreduce_peer.py")


def _spawn(addr, world, rank, *extra, device="cpu"):
    return spawn_python([WORKER, addr, str(world), str(rank), "--device", device, *extra],
                        stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def _lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def _check_ok(lines):
    oks = [ln for ln in lines if "error" not in ln]
    assert oks and not any(ln.get("bad") for ln in oks), lines[-5:]
    return oks


@pytest.mark.parametrize("n", [1000, 1 << 20])
def test_peer_crash_survivors_continue(n):
    with local_master() as addr:
        ps = [_spawn(addr, 3, r, "--const", "--n", str(n), "--steps", "40", "--step-sleep", "0.01",
                     *(["--die-at", "10"] if r == 1 else [])) for r in range(3)]
        outs = communicate_all(ps, 240, DIAG_SIGNALS)
    assert ps[1].returncode == 17
    for r in (0, 2):
        assert ps[r].returncode == 0, outs[r][1][-3000:]
        oks = _check_ok(_lines(outs[r][0]))
        assert len(oks) == 40
        assert oks[0]["world"] == 3 and oks[-1]["world"] == 2


def test_crash_and_rejoin():
    with local_master() as addr:
        ps = [_spawn(addr, 3, r, "--const", "--n", "4096", "--steps", "150", "--step-sleep", "0.02",
                     *(["--die-at", "10"] if r == 2 else [])) for r in range(3)]
        time.sleep(1.0)
        deadline = time.time() + 60
        while ps[2].poll() is None and time.time() < deadline:
            time.sleep(0.1)
        assert ps[2].returncode == 17
        joiner = _spawn(addr, 3, 3, "--const", "--n", "4096", "--steps", "20", "--no-wait", "--leave-when-alone")
        (jo, je), = communicate_all([joiner], 150, DIAG_SIGNALS)
        outs = communicate_all(ps[:2], 240, DIAG_SIGNALS)
    assert joiner.returncode == 0, je[-3000:]
    jl = _check_ok(_lines(jo))
    assert all(ln["world"] == 3 for ln in jl)
    for r in (0, 1):
        assert ps[r].returncode == 0, outs[r][1][-3000:]
        oks = _check_ok(_lines(outs[r][0]))
        worlds = [ln["world"] for ln in oks]
        assert worlds[0] == 3 and 2 in worlds and worlds.count(3) > 20  # shrank to 2, grew back to 3
    print("rejoin latency (s):", jl[0]["first_ok_s"])
    assert jl[0]["first_ok_s"] < 20


def test_master_kill_peers_fail_cleanly():
    """Losing the master makes collectives fail with an error instead of hanging."""
    import pccl_amd as pccl
    master_port = None
    with local_master() as addr:
        master_port = addr
        ps = [_spawn(addr, 2, r, "--const", "--n", "1000", "--steps", "100000", "--step-sleep", "0.01")
              for r in range(2)]
        time.sleep(3.0)
    # master is gone: peers must exit (error) within a bounded time
    for p in ps:
        try:
            p.communicate(timeout=90)
        except subprocess.TimeoutExpired:
            p.kill()
            pytest.fail("peer hung after master loss")
        assert p.returncode != 0
    assert master_port and pccl is not None


@pytest.mark.gpu
def test_gpu_peer_crash_survivors_continue(hip):
    with local_master() as addr:
        ps = [_spawn(addr, 3, r, "--const", "--n", str(1 << 22), "--dtype", "bf16", "--steps", "30",
                     *(["--die-at", "8"] if r == 0 else []), device="cuda:0") for r in range(3)]
        outs = communicate_all(ps, 300, DIAG_SIGNALS)
    assert ps[0].returncode == 17
    for r in (1, 2):
        assert ps[r].returncode == 0, outs[r][1][-3000:]
        oks = _check_ok(_lines(outs[r][0]))
        assert len(oks) == 30 and oks[-1]["world"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("point,inplace,respawn,shareable", [
    ("ipc_kernel", False, False, False), ("ipc_kernel", True, False, False), ("ipc_vote", True, False, False),
    ("ipc_kernel", False, True, False), ("ipc_kernel", False, False, True), ("ipc_kernel", True, False, True)])
def test_gpu_ipc_sigkill_mid_op(hip, tmp_path, point, inplace, respawn, shareable):
    """xGMI/IPC path, 3 processes on one GPU, 512 MiB bf16: peer 0 SIGKILLs itself at a fixed protocol point of op
    300 (PCCL_FAULT_INJECT) - right after launching its push kernel (every peer's kernel is then reading / writing the
    victim's exported HBM) or right after publishing its vote. Survivors must abort that op, re-form the ring and
    keep producing exact results on the IPC path, with no GPU memory fault; with `respawn` a fresh replacement process
    joins the running ring afterwards (new arena, the BASELINE config 5 sequence). With `shareable` the peers' buffers
    live in fd-shareable memory (pccl_amd.memory): the kernels read / write the victim's own tensors (zero-copy), and
    those must survive its death just as the staged comm buffers do."""
    summary = _ipc_kill(tmp_path, point, inplace, respawn, shareable)
    for k in (1, 2):
        s_k = summary[f"peer{k}"]
        if shareable:  # the output (and, out of place, the input) went to the peers directly
            b = s_k["ipc_bufs"]
            assert b["direct_out"] > 300 and b["staged_out"] == 0, b
            assert (b["direct_in"] > 300 and b["staged_in"] == 0) if not inplace else b["direct_in"] == 0, b


@pytest.mark.gpu
@pytest.mark.parametrize("shareable", [False, True])
def test_gpu_ipc_sigkill_after_local_success(hip, tmp_path, shareable):
    """op_end on the xGMI path: op 300 finished on every peer (the gathered barrier passed, every output holds the
    result) and the victim dies before its completion packet. If the master aborts op 300 the survivors' in-place
    buffers must hold the input again (the staged original is kept until the verdict, OpState::settle), else the
    result stands and the next op fails; either way every failed op's buffer is re-read 200 ms later bit-exactly
    and the survivors continue on the IPC path."""
    summary = _ipc_kill(tmp_path, "op_end", True, False, shareable, "--verify-restore-ms", "200",
                        inject="op_end:300")
    for k in (1, 2):
        s_k = summary[f"peer{k}"]
        assert s_k["errors"] >= 1 and s_k["restore_bad"] == 0 and s_k["restore_checked"] >= 1, s_k


@pytest.mark.gpu
def test_gpu_ipc_sigkill_many_threads_restore_is_final(hip, tmp_path):
    """Abort quiescence keyed to GPU state, not process state: the victim runs 48 extra busy threads, so when it is
    SIGKILLed right after launching its push kernel its group leader turns zombie while the other threads still exit
    (and still hold the address space whose teardown evicts its GPU queues). In-place ops in shareable memory: the
    victim's kernel writes straight into the survivors' buffers. Each survivor waits for that teardown before it
    restores its buffer, re-reads the buffer 200 ms after the failed op and requires the original input bit-exactly,
    and the staged comm buffer of the aborted op is quarantined (never handed to a later op)."""
    summary = _ipc_kill(tmp_path, "ipc_kernel", True, False, True, "--victim-threads", "48",
                        "--verify-restore-ms", "200")
    for k in (1, 2):
        s_k = summary[f"peer{k}"]
        assert s_k["restore_checked"] >= 1 and s_k["restore_bad"] == 0, s_k
        assert s_k["ipc_bufs"]["quarantined"] >= 1, s_k


def _ipc_kill(tmp_path, point, inplace, respawn, shareable, *extra, inject=None, path=3, n=1 << 28, duration=None,
              min_ops=300):
    """Runs scripts/ipc_kill_probe.py (victim = peer 0, killed at `point` of op 300, or at `inject`) and checks the
    common outcome: the victim died of SIGKILL, the survivors exited cleanly with exact results over both world sizes
    on reduce path `path` (3 IPC, 2 device ring) and no GPU fault line. Returns the probe's JSON summary."""
    import sys
    probe = os.path.join(os.path.dirname(HERE), "scripts", "ipc_kill_probe.py")
    dur = duration if duration is not None else ("12" if respawn else "4")
    args = [sys.executable, probe, "--inject", inject or f"{point}:300", "--duration", str(dur), "--n", str(n),
            "--out", str(tmp_path / "ipc_kill")]
    args += (["--inplace"] if inplace else []) + (["--respawn"] if respawn else []) + \
        (["--shareable"] if shareable else []) + list(extra)
    r = subprocess.run(args, capture_output=True, text=True, timeout=240)
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["victim_rc"] == -9, summary
    assert summary["survivor_rcs"] == [0, 0] + ([0] if respawn else []), (summary, r.stderr[-2000:])
    if respawn:
        j = summary["peer3"]
        assert j["bad"] == 0 and not j["fault_lines"] and j["ops_ok"] > 0 and 3 in j["worlds"], j
    for k in (1, 2):
        s_k = summary[f"peer{k}"]
        assert s_k["bad"] == 0 and not s_k["fault_lines"], s_k
        assert 2 in s_k["worlds"] and 3 in s_k["worlds"] and s_k["ops_ok"] > min_ops and s_k["paths"] == [path], s_k
    return summary


# Device TCP ring (PCCL_DISABLE_IPC=1), 3 processes on one GPU, 64 Mi bf16 elements: the victim SIGKILLs itself at a
# global ring step (0-1 reduce-scatter, 2-3 all-gather) of op 12 in a given phase (csrc/common/types.hpp): `publish`
# (its step's sends just handed to the stripe threads), `rx` (first received piece handed to the copy engine /
# kernels), `ahead` (the next step's sinks posted while this step still receives), `end`; quantized ring: `meta`
# (its metadata packet sent, waiting for the peer's), `rx`.
RING_KILLS = [("ring", 0, "ahead", False), ("ring", 1, "rx", True), ("ring", 2, "rx", False),
              ("ring", 3, "publish", True), ("ring", 1, "end", False), ("qring", 1, "meta", True),
              ("qring", 2, "rx", False), ("qring", 0, "rx", True),
              # the victim dies after its last step: survivors finish their part, the master aborts the op anyway and
              # the in-place input comes back from the backup kept until the verdict (OpState::settle)
              ("ring", 3, "end", True), ("qring", 3, "end", True),
              # after the victim's whole part (the op_end point, before its completion packet), plain and quantized
              ("op_end", None, None, True), ("op_end", None, "q", True)]


@pytest.mark.gpu
@pytest.mark.parametrize("point,step,phase,inplace", RING_KILLS)
def test_gpu_ring_sigkill_mid_op(hip, tmp_path, point, step, phase, inplace):
    """Abort safety of the pipelined device ring (plain and quantized): survivors drain every copy / kernel of the
    aborted op before their in-place buffer is restored (re-read 200 ms later, bit-exact), re-form the ring and keep
    producing exact results for at least 20 more ops in the smaller world (reference reduce.cpp:551-580,657-660)."""
    quant = point == "qring" or phase == "q"
    inject = "op_end:12" if point == "op_end" else f"{point}:12:{step}:{phase}"
    summary = _ipc_kill(tmp_path, point, inplace, False, False, "--disable-ipc", "--verify-restore-ms", "200",
                        "--pool", "2", *(["--quant", "u8"] if quant else []), inject=inject,
                        path=2, n=1 << 26, duration=12, min_ops=30)
    for k in (1, 2):
        s_k = summary[f"peer{k}"]
        assert s_k["errors"] >= 1 and s_k["restore_bad"] == 0, s_k
        if inplace:
            assert s_k["restore_checked"] >= 1, s_k
        assert s_k["ops_ok_by_world"].get("2", 0) >= 20, s_k


@pytest.mark.gpu
@pytest.mark.parametrize("shareable", [False, True])
def test_gpu_shared_state_distributor_sigkill_mid_handoff(hip, shareable):
    """Same-host shared-state hand-off (HBM entries passed as VMM fd shares): the distributor SIGKILLs itself 300 ms
    after sending its IPC response (PCCL_FAULT_INJECT=ss_serve:5 + PCCL_FAULT_INJECT_DELAY_MS) while the joiner has
    mapped its copy and waits 1 s before copying (PCCL_SS_COPY_DELAY_MS). The joiner's import holds its own reference
    to the pages, so the copy reads valid memory of a dead process: exact data, no GPU fault, and the survivors then
    all-reduce in the shrunken world. Both distributors carry the injection; only the one that serves dies."""
    worker = os.path.join(HERE, "workers", "ss_peer.py")
    extra = ["--n", str(1 << 26)] + (["--shareable"] if shareable else [])
    kill = {"PCCL_FAULT_INJECT": "ss_serve:5", "PCCL_FAULT_INJECT_DELAY_MS": "300"}
    with local_master() as addr:
        ds = [spawn_python([worker, addr, "dist", *extra], env=kill, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True) for _ in range(2)]
        time.sleep(1.0)
        j = spawn_python([worker, addr, "join", *extra], env={"PCCL_SS_COPY_DELAY_MS": "1000"},
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        outs = communicate_all(ds + [j], 180, DIAG_SIGNALS)
    rcs = [p.returncode for p in ds + [j]]
    assert sorted(rcs[:2]) == [-9, 0], (rcs, [o[1][-2000:] for o in outs])
    assert rcs[2] == 0, outs[2][1][-3000:]
    for _, err in outs:
        assert "memory access fault" not in err.lower() and "illegal address" not in err.lower(), err[-2000:]
    jl = _lines(outs[2][0])
    sync = next(x for x in jl if x["phase"] == "sync")
    assert sync["lo"] == sync["hi"] == 7.0 and sync["rx"] == (1 << 26) * 4 and sync["revision"] == 5, jl
    ar = next(x for x in jl if x["phase"] == "all_reduce")
    assert ar["world"] == 2 and ar["lo"] == ar["hi"] == 2.0, jl


@pytest.mark.gpu
def test_gpu_shared_state_many_tensors_packed_handoff(hip):
    """A joiner in another process receives 300 small HBM tensors of odd sizes plus one 256 MiB tensor over the
    fault-safe IPC hand-off: the small ones are packed into shared VMM segments (one fd / import per segment), the
    large one has its own; every byte arrives."""
    worker = os.path.join(HERE, "workers", "ss_peer.py")
    extra = ["--n", str(1 << 26), "--extra-tensors", "300"]
    with local_master() as addr:
        ds = [spawn_python([worker, addr, "dist", *extra], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
              for _ in range(2)]
        time.sleep(1.0)
        j = spawn_python([worker, addr, "join", *extra], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        outs = communicate_all(ds + [j], 180, DIAG_SIGNALS)
    assert [p.returncode for p in ds + [j]] == [0, 0, 0], [o[1][-2000:] for o in outs]
    sync = next(x for x in _lines(outs[2][0]) if x["phase"] == "sync")
    assert sync["lo"] == sync["hi"] == 7.0 and sync["extra_ok"] and sync["revision"] == 5, sync
    assert sync["sec"] < 5.0, sync


@pytest.mark.gpu
def test_gpu_ipc_quarantine_reclaimed_on_unchanged_ring(hip):
    """50 aborted staged xGMI ops on a ring whose membership never changes (the arena is reused): peer 1 stalls
    300 ms before publishing its vote for ops seq <= 49 (PCCL_FAULT_STALL) while peer 0's vote barrier gives up after
    100 ms (PCCL_IPC_TIMEOUT_MS), so every such op aborts on both peers and quarantines its staged comm buffers. Each
    later acquire reclaims them once no peer can still touch them for the aborted op: HBM use stays flat over the
    aborts, the reclaim counter moves, and the ops after the stall succeed with exact results."""
    n = 1 << 24  # 64 MiB fp32 per buffer
    env = {"PCCL_IPC_TIMEOUT_MS": "100"}
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "2", str(r), "--device", "cuda:0", "--const", "--inplace", "--n", str(n),
                            "--steps", "10", "--max-failures", "60", "--report-mem"],
                           env=dict(env, **({"PCCL_FAULT_STALL": "ipc_vote:49:300"} if r == 1 else {})),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = communicate_all(ps, 240, DIAG_SIGNALS)
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, e[-3000:]
        lines = _lines(o)
        errs = [x for x in lines if "error" in x]
        oks = _check_ok(lines)
        assert len(errs) >= 45 and len(oks) == 10, (len(errs), len(oks))
        assert all(x["path"] == 3 and x["world"] == 2 for x in oks), oks[-1]
        used = [x["hbm_used"] for x in errs]
        # flat: no growth by a buffer per aborted op (64 MiB x 2 buffers x 2 peers each)
        assert max(used[5:]) - used[5] < 3 * (n * 4), used
        b = oks[-1]["ipc_bufs"]
        assert b["quarantined"] >= 45 and b["reclaimed"] >= 40, b


# Host ring (CPU tensors): the victim SIGKILLs itself in op 8 at a global ring step (0-1 reduce-scatter, 2-3
# all-gather) after its first received bytes were reduced (`rx`) or after the step completed (`end`).
HRING_KILLS = [(0, "rx", True, False), (1, "end", False, False), (2, "rx", True, False), (3, "rx", False, False),
               (1, "rx", True, True), (2, "end", True, True), (3, "end", True, False), (3, "end", True, True),
               # op_end: the victim finished its part of op 8 and dies before its completion packet. Depending on
               # when the master sees the disconnect, op 8 either completes for the survivors (their results stand)
               # or is aborted after their rings succeeded (the input comes back from the backup kept until the
               # verdict); either way the next op fails and restores. (2, "end", True, True) above is the case that
               # needs the late restore every time: one survivor's ring succeeded, the other's failed.
               (None, "op_end", True, False), (None, "op_end", True, True)]


# the host-emulated device backend (PCCL_TEST_HOSTDEV: another build of it, e.g. the TSan one)
HOSTDEV = os.environ.get("PCCL_TEST_HOSTDEV") or os.path.join(os.path.dirname(HERE), "pccl_amd", "lib",
                                                              "libpccl_hostdev.so")


@pytest.mark.parametrize("point,step,phase,inplace", RING_KILLS)
def test_emulated_device_ring_sigkill_mid_op(point, step, phase, inplace):
    """The device ring's kill matrix (RING_KILLS) on CPU: 3 peer processes on the host-emulated device backend
    (csrc/testing/hostdev_backend.cpp: every buffer taken for device memory, streams as worker threads, the host twins
    of the kernels) run the plain and quantized device rings; the victim SIGKILLs itself at the point of op 8. The
    survivors fail that op, drain every copy / kernel of it before the in-place input is restored (re-read 100 ms
    later, bit-exact), re-form the ring and finish every step exactly in the smaller world, on the device ring."""
    if not os.path.exists(HOSTDEV) or os.environ.get("PCCL_DISABLE_HIP") == "1":
        pytest.skip("libpccl_hostdev.so not built, or device plugins disabled (PCCL_DISABLE_HIP)")
    quant = point == "qring" or phase == "q"
    inject = "op_end:8" if point == "op_end" else f"{point}:8:{step}:{phase}"
    dev = {"PCCL_HIP_PLUGIN": HOSTDEV, "PCCL_HOSTDEV_ALL_DEVICE": "1", "PCCL_DISABLE_IPC": "1"}
    extra = (["--inplace"] if inplace else []) + (["--quant", "u8"] if quant else [])
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "3", str(r), "--device", "cpu", "--const", "--n", str(1 << 22), "--steps",
                            "30", "--pool", "2", *extra, *(["--verify-restore-ms", "100"] if r else [])],
                           env=dict(dev, PCCL_FAULT_INJECT=inject) if r == 0 else dev,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
        outs = communicate_all(ps, 240, DIAG_SIGNALS)
    assert ps[0].returncode == -9, outs[0][1][-2000:]
    for r in (1, 2):
        assert ps[r].returncode == 0, outs[r][1][-3000:]
        lines = _lines(outs[r][0])
        oks = _check_ok(lines)
        errs = [x for x in lines if "error" in x]
        assert len(oks) == 30 and oks[0]["world"] == 3 and oks[-1]["world"] == 2, (len(oks), oks[-1])
        assert all(x["path"] == 2 for x in oks), oks[-1]
        assert errs and not any(x.get("restore_bad") for x in errs), errs


@pytest.mark.parametrize("step,phase,inplace,quant", HRING_KILLS)
def test_host_ring_sigkill_mid_op(step, phase, inplace, quant):
    """Abort safety of the host ring (the reference's data path, reduce.cpp:551-580,657-660): survivors of a peer
    killed mid-op get an error for that op, find their in-place buffer restored bit-exactly 100 ms later, re-form the
    ring and finish every step with exact results in the smaller world."""
    n = 1 << 22
    extra = (["--inplace"] if inplace else []) + (["--quant", "u8"] if quant else [])
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "3", str(r), "--device", "cpu", "--const", "--n", str(n), "--steps", "30",
                            "--pool", "2", *extra, *(["--verify-restore-ms", "100"] if r else [])],
                           env={"PCCL_FAULT_INJECT": "op_end:8" if phase == "op_end" else f"hring:8:{step}:{phase}"}
                           if r == 0 else None,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
        outs = communicate_all(ps, 240, DIAG_SIGNALS)
    assert ps[0].returncode == -9, outs[0][1][-2000:]
    for r in (1, 2):
        assert ps[r].returncode == 0, outs[r][1][-3000:]
        lines = _lines(outs[r][0])
        oks = _check_ok(lines)
        errs = [x for x in lines if "error" in x]
        assert len(oks) == 30 and oks[0]["world"] == 3 and oks[-1]["world"] == 2, (len(oks), oks[-1])
        assert errs and not any(x.get("restore_bad") for x in errs), errs
        if inplace:
            assert any("restore_bad" in x for x in errs), errs
