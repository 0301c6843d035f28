"""Bounded-time failure detection for peers that stop without closing their sockets.

The reference detects a failed peer only by TCP close / RST and SO_KEEPALIVE (tinysockets multiplexed_socket.cpp:
29-49, server_socket.cpp): a SIGSTOPped peer, a wedged driver call or a black-holed path hangs its whole group for
ever (its kernel keeps ACKing; keepalive never probes while data is outstanding). pccl-amd adds a negotiated liveness
protocol (docs/ARCHITECTURE.md "Failure detection"): peer heartbeats with a master-side timeout, an op-progress
watchdog whose stall reports let the master name and drop the peer at fault, and teardown that never joins a sender
blocked in sendmsg. These tests SIGSTOP a peer mid-op (PCCL_FAULT_SIGNAL=STOP at a PCCL_FAULT_INJECT point) or
black-hole one ring link in the WAN relay, and require: survivors get a failed op within the timeout + 2 s, re-form
the ring one smaller with exact results (in-place buffers restored), and the stopped peer, once resumed, gets a
clean error (MASTER_CONNECTED == 0) and joins again as a new peer.
"""
import json
import os
import signal
import subprocess
import threading
import time

import pytest

from pccl_amd.utils import DIAG_SIGNALS, communicate_all, free_ports, local_master, spawn_python

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "workers", "allreduce_peer.py")
RELAY = os.path.join(os.path.dirname(HERE), "pccl_amd", "lib", "pccl_wan_relay")

PEER_TIMEOUT_S = 2.0  # PCCL_PEER_TIMEOUT_MS for these tests; the op-stall timeout defaults to 1.5x (3 s)


def _lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def _proc_state(pid):
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0]
    except (OSError, IndexError):
        return None


def _wait_until(pred, timeout, what):
    t0 = time.time()
    while not pred():
        if time.time() - t0 > timeout:
            raise AssertionError(f"timed out waiting for {what}")
        time.sleep(0.01)


class _Run:
    """Peers whose output is drained in the background while the test stops / resumes / black-holes them."""

    def __init__(self, procs, timeout):
        self.procs = procs
        self.outs = None
        self.err = None

        def body():
            try:
                self.outs = communicate_all(procs, timeout, DIAG_SIGNALS)
            except Exception as e:  # noqa: BLE001 - reported by join()
                self.err = e
        self.t = threading.Thread(target=body, daemon=True)
        self.t.start()

    def join(self):
        self.t.join()
        if self.err:
            raise self.err
        return self.outs


def _check_survivor(lines, t_fault, bound_s, world_before=3, smaller_ring=True):
    oks = [x for x in lines if "error" not in x and "world" in x]
    assert oks and not any(x.get("bad") for x in oks), lines[-5:]
    errs = [x for x in lines if "error" in x]
    assert errs, "the survivor never saw the failure"
    assert not any(x.get("restore_bad") for x in errs), errs
    assert not any(x.get("kicked") for x in errs), errs
    first_err = min(x["t"] for x in errs if x["t"] >= t_fault - 0.5)
    detect = first_err - t_fault
    assert detect <= bound_s, f"failed op {detect:.2f} s after the fault (bound {bound_s} s)"
    assert oks[0]["world"] == world_before
    after = [x for x in oks if x["t"] > first_err]
    if smaller_ring and not any(x["world"] < world_before for x in after):
        print("survivor timeline:", [(round(x["t"] - t_fault, 2), x.get("world", x.get("error", "")[:50]))
                                     for x in lines if x["t"] > t_fault - 0.5])
        raise AssertionError("the ring did not re-form without the stopped peer")
    return detect, after


@pytest.mark.parametrize("quant,inplace", [(False, True), (True, True), (False, False)])
def test_sigstopped_peer_host_ring(monkeypatch, quant, inplace):
    """3 CPU peers on the host ring; peer 0 SIGSTOPs itself after the first received bytes of ring step 1 of op seq
    20 and is resumed 5 s later. Its heartbeats stop with it: the master drops it after PCCL_PEER_TIMEOUT_MS and aborts
    the op, the survivors' op fails within the timeout + 2 s (their senders blocked on its full socket are
    interrupted, not joined), their in-place input is restored bit-exactly, and they continue at W = 2 with exact
    results. Once resumed the stopped peer fails cleanly (MASTER_CONNECTED == 0), joins again as a new peer and the
    ring grows back to 3."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", str(int(PEER_TIMEOUT_S * 1000)))
    extra = ["--const", "--n", str(1 << 20), "--pool", "2", "--duration", "16", "--rejoin", "--max-failures", "30"]
    extra += (["--inplace", "--verify-restore-ms", "100"] if inplace else []) + (["--quant", "u8"] if quant else [])
    stop = {"PCCL_FAULT_INJECT": "hring:20:1:rx", "PCCL_FAULT_SIGNAL": "STOP"}
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "3", str(r), "--device", "cpu", *extra], env=stop if r == 0 else None,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
        run = _Run(ps, 150)
        _wait_until(lambda: _proc_state(ps[0].pid) == "T" or ps[0].poll() is not None, 60, "the victim to stop")
        t_stop = time.time()
        assert ps[0].poll() is None
        time.sleep(5.0)
        os.kill(ps[0].pid, signal.SIGCONT)
        outs = run.join()
    for r in range(3):
        assert ps[r].returncode == 0, (r, outs[r][1][-3000:])
    for r in (1, 2):
        detect, after = _check_survivor(_lines(outs[r][0]), t_stop, PEER_TIMEOUT_S + 2.0)
        print(f"peer {r}: failed op {detect:.2f} s after the stop")
        assert any(x["world"] == 3 for x in after), "the resumed peer did not rejoin"
    vl = _lines(outs[0][0])
    kicked = [x for x in vl if x.get("kicked")]
    assert kicked and kicked[0]["t"] > t_stop + 4.0, vl[:5]
    rej = [x for x in vl if x.get("rejoined")]
    assert rej, vl[-5:]
    oks_after = [x for x in vl if "world" in x and x["t"] > rej[0]["t"]]
    assert oks_after and not any(x.get("bad") for x in oks_after), vl[-5:]


def test_blackholed_link_host_ring(monkeypatch):
    """3 CPU peers whose P2P connections pass a relay (pccl_wan_relay, 1 ms); after ops run, the relay black-holes
    the link into peer 1 (SIGUSR1: both directions stop forwarding, sockets stay open). Heartbeats to the master
    continue, so only the op watchdog sees it: every peer reports its stalled op after PCCL_OP_STALL_MS, the master
    drops the peer the reports name (the sender in front of the broken link, or its receiver when a send is blocked)
    and the survivors' op fails within the stall timeout + 2 s; they continue at W = 2 with exact results, the
    dropped peer joins again over fresh connections and the ring grows back to 3."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", str(int(PEER_TIMEOUT_S * 1000)))
    stall_s = 1.5 * PEER_TIMEOUT_S
    ports = free_ports(6)
    listen, adv = ports[:3], ports[3:]
    relay = subprocess.Popen([RELAY, "--delay-ms", "1", "--flow-mbit", "40000",
                              *sum([["--map", f"{adv[r]}:{listen[r]}"] for r in range(3)], []),
                              "--blackhole-port", str(adv[1])], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                             text=True)
    try:
        assert json.loads(relay.stdout.readline())["relay"] == "ready"
        extra = ["--const", "--n", str(1 << 20), "--pool", "2", "--duration", "14", "--rejoin", "--max-failures", "30"]
        with local_master() as addr:
            ps = [spawn_python([WORKER, addr, "3", str(r), "--device", "cpu", "--p2p-port", str(listen[r]),
                                "--adv-port", str(adv[r]), *extra],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
            run = _Run(ps, 150)
            time.sleep(5.0)  # import, connect, admit, and some ops
            t_bh = time.time()
            relay.send_signal(signal.SIGUSR1)
            outs = run.join()
    finally:
        relay.terminate()
        relay.wait(10)
    for r in range(3):
        assert ps[r].returncode == 0, (r, outs[r][1][-3000:])
    lines = [_lines(o) for o, _ in outs]
    # Peer 0 (in front of the broken link into peer 1) or peer 1 is dropped first. Every connection of the relay map
    # that existed at SIGUSR1 is black: if the smaller ring reuses one (peer 2's pool to peer 1, opened when it was
    # a neighbour), that op stalls as well and the master drops one of its endpoints too; fresh connections work.
    dropped = [r for r in range(3) if any(x.get("kicked") for x in lines[r])]
    assert 1 <= len(dropped) <= 2, dropped
    for r in dropped:
        rej = [x for x in lines[r] if x.get("rejoined")]
        assert rej and any(x.get("world") == 3 and x["t"] > rej[-1]["t"] for x in lines[r]), lines[r][-3:]
    for r in range(3):
        if r in dropped:
            continue
        oks_before = [x for x in lines[r] if "world" in x and x["t"] < t_bh]
        assert len(oks_before) >= 3, "no ops before the black hole"
        # With a second peer dropped (a reused black connection) both may be admitted again by the survivor's next
        # update_topology, so it need not run an op in a smaller ring: the ring growing back to 3 is checked below.
        detect, after = _check_survivor(lines[r], t_bh, stall_s + 2.0, smaller_ring=len(dropped) == 1)
        print(f"peer {r}: failed op {detect:.2f} s after the black hole (dropped: {dropped}, "
              f"worlds after: {sorted(set(x['world'] for x in after))})")
        assert any(x["world"] == 3 for x in after), "the dropped peer did not rejoin"


def test_sigstopped_idle_peer_consensus(monkeypatch):
    """A peer stopped between collectives (SIGSTOP from outside while it idles) holds no op the watchdog could see;
    the consensus rounds that need its vote - the shared-state sync (every accepted peer must vote) and the next
    all-reduce - would wait for it forever without heartbeats. The master drops it after PCCL_PEER_TIMEOUT_MS, and
    the survivors complete a round at W = 2 within the timeout + 2 s of the stop; once resumed, the stopped peer
    finds itself dropped (MASTER_CONNECTED == 0)."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", str(int(PEER_TIMEOUT_S * 1000)))
    worker = os.path.join(HERE, "workers", "consensus_peer.py")
    with local_master() as addr:
        ps = [spawn_python([worker, addr, "3", str(r), "--duration", "14", "--step-sleep", "0.3"],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
        run = _Run(ps, 120)
        time.sleep(6.0)  # import, connect, admit, some rounds
        t_stop = time.time()
        os.kill(ps[0].pid, signal.SIGSTOP)
        time.sleep(5.0)
        os.kill(ps[0].pid, signal.SIGCONT)
        outs = run.join()
    for r in range(3):
        assert ps[r].returncode == 0, (r, outs[r][1][-3000:])
    for r in (1, 2):
        lines = _lines(outs[r][0])
        before = [x for x in lines if x["t"] < t_stop and x.get("world") == 3]
        assert len(before) >= 2, lines[:5]
        after = [x for x in lines if x["t"] > t_stop and x.get("world") == 2 and x.get("ar")]
        assert after, lines[-5:]
        # a round that started before the drop ends once the master dropped the peer (+ its own duration)
        done = min(x["t"] for x in after) - t_stop
        assert done <= PEER_TIMEOUT_S + 2.0 + 0.5, f"first W = 2 round {done:.2f} s after the stop"
        print(f"peer {r}: first round at W = 2 {done:.2f} s after the stop")
    assert any(x.get("kicked") for x in _lines(outs[0][0])), outs[0][0][-1000:]


def test_sigstopped_shared_state_distributor(monkeypatch):
    """The shared-state distributor stops (SIGSTOP at the ss_serve fault point: response sent, entries not yet
    streamed) while a late joiner fetches 256 MiB from it over TCP. Its kernel keeps the connections alive, so
    neither keepalive nor TCP_USER_TIMEOUT would end the joiner's receives: the fetch sockets time out after
    PCCL_OP_STALL_MS without a byte, and the joiner's sync fails within that + 2 s of the stop instead of hanging."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", str(int(PEER_TIMEOUT_S * 1000)))
    stall_s = 1.5 * PEER_TIMEOUT_S
    worker = os.path.join(HERE, "workers", "ss_peer.py")
    extra = ["--device", "cpu", "--n", str(1 << 26), "--world", "2", "--no-all-reduce"]
    stop = {"PCCL_FAULT_INJECT": "ss_serve:5", "PCCL_FAULT_SIGNAL": "STOP"}
    with local_master() as addr:
        d = spawn_python([worker, addr, "dist", *extra], env=stop, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
        time.sleep(1.0)
        j = spawn_python([worker, addr, "join", *extra], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        run = _Run([j], 120)
        try:
            _wait_until(lambda: _proc_state(d.pid) == "T" or d.poll() is not None, 60, "the distributor to stop")
            t_stop = time.time()
            (jo, je), = run.join()
        finally:
            d.kill()
            d.communicate(timeout=30)
    assert j.returncode == 0, je[-3000:]
    sync = next(x for x in _lines(jo) if x["phase"] == "sync")
    assert "error" in sync, (sync, je[-3000:])
    detect = sync["t"] - t_stop
    assert detect <= stall_s + 2.0, f"sync failed {detect:.2f} s after the stop"
    print(f"joiner: sync failed {detect:.2f} s after the distributor stopped")


def test_reference_wire_peer_is_exempt_from_heartbeats(monkeypatch):
    """A peer speaking the reference protocol (PCCL_WIRE=reference) sends no heartbeats and must not be dropped for
    it: with a 1 s peer timeout, a mixed pair keeps all-reducing for 4 s without an error."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", "1000")
    extra = ["--const", "--n", "4096", "--duration", "4", "--step-sleep", "0.2"]
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "2", str(r), "--device", "cpu", *extra],
                           env={"PCCL_WIRE": "reference"} if r == 0 else None,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = communicate_all(ps, 120, DIAG_SIGNALS)
    for r in range(2):
        assert ps[r].returncode == 0, outs[r][1][-2000:]
        lines = _lines(outs[r][0])
        assert lines and not any("error" in x for x in lines), lines[-3:]
        assert all(x["world"] == 2 for x in lines)


def test_stopped_master_is_detected(monkeypatch):
    """The master sends heartbeats too: a peer whose master stops answering (SIGSTOP of a separate master process)
    fails its next collective within 2 x PCCL_PEER_TIMEOUT_MS instead of hanging, and reports the master lost."""
    import sys
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", "1000")
    port = free_ports(1)[0]
    master = subprocess.Popen([sys.executable, "-m", "pccl_amd.master", "--port", str(port)],
                              env=dict(os.environ, PYTHONPATH=os.path.dirname(HERE)), stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, text=True)
    try:
        assert "listening" in master.stdout.readline()
        addr = f"127.0.0.1:{port}"
        extra = ["--const", "--n", "4096", "--steps", "100000", "--step-sleep", "0.01", "--max-failures", "0"]
        ps = [spawn_python([WORKER, addr, "2", str(r), "--device", "cpu", *extra],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        run = _Run(ps, 90)
        time.sleep(6.0)  # import, connect, admit, ops
        t_stop = time.time()
        master.send_signal(signal.SIGSTOP)
        outs = run.join()
        t_end = time.time()
    finally:
        master.send_signal(signal.SIGCONT)
        master.kill()
        master.wait(10)
    for r in range(2):
        assert ps[r].returncode != 0
    assert t_end - t_stop < 2 * 1.0 + 5.0, t_end - t_stop


def _gpu_stop_run(monkeypatch, inject, extra_env, n, extra_args=()):
    """3 peer processes on cuda:0, in place, the victim (peer 0) SIGSTOPped at `inject` and resumed 5 s later;
    returns (t_stop, outs) after the common checks of a survivor / rejoin run."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", str(int(PEER_TIMEOUT_S * 1000)))
    args = ["--device", "cuda:0", "--const", "--inplace", "--verify-restore-ms", "200", "--n", str(n), "--dtype",
            "bf16", "--duration", "18", "--rejoin", "--max-failures", "30", *extra_args]
    stop = dict(extra_env, PCCL_FAULT_INJECT=inject, PCCL_FAULT_SIGNAL="STOP")
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "3", str(r), *args], env=stop if r == 0 else extra_env,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
        run = _Run(ps, 200)
        _wait_until(lambda: _proc_state(ps[0].pid) == "T" or ps[0].poll() is not None, 120, "the victim to stop")
        t_stop = time.time()
        assert ps[0].poll() is None
        time.sleep(5.0)
        os.kill(ps[0].pid, signal.SIGCONT)
        outs = run.join()
    for r in range(3):
        assert ps[r].returncode == 0, (r, outs[r][1][-3000:])
        assert "memory access fault" not in outs[r][1].lower(), outs[r][1][-2000:]
    for r in (1, 2):
        detect, after = _check_survivor(_lines(outs[r][0]), t_stop, PEER_TIMEOUT_S + 2.0)
        print(f"peer {r}: failed op {detect:.2f} s after the stop")
        assert any(x["world"] == 3 for x in after), "the resumed peer did not rejoin"
    vl = _lines(outs[0][0])
    assert any(x.get("kicked") for x in vl) and any(x.get("rejoined") for x in vl), vl[-5:]
    return t_stop, outs


# the host-emulated device backend (PCCL_TEST_HOSTDEV: another build of it, e.g. the TSan one)
HOSTDEV = os.environ.get("PCCL_TEST_HOSTDEV") or os.path.join(os.path.dirname(HERE), "pccl_amd", "lib",
                                                              "libpccl_hostdev.so")


@pytest.mark.parametrize("point", ["ring:8:1:rx", "qring:8:1:meta"])  # (op 8: reached early under TSan too)
def test_sigstopped_peer_emulated_device_ring(monkeypatch, point):
    """The device ring's stop points on CPU: peers on the host-emulated device backend (every buffer taken for device
    memory, streams as worker threads; csrc/testing/hostdev_backend.cpp) run the plain and quantized device rings, and
    peer 0 stops inside a ring step; survivors fail within the peer timeout + 2 s, drain, restore their in-place input
    and continue at W = 2 on the device ring; the resumed peer rejoins."""
    if not os.path.exists(HOSTDEV) or os.environ.get("PCCL_DISABLE_HIP") == "1":
        pytest.skip("libpccl_hostdev.so not built, or device plugins disabled (PCCL_DISABLE_HIP)")
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", str(int(PEER_TIMEOUT_S * 1000)))
    dev = {"PCCL_HIP_PLUGIN": HOSTDEV, "PCCL_HOSTDEV_ALL_DEVICE": "1", "PCCL_DISABLE_IPC": "1"}
    scale = float(os.environ.get("PCCL_TEST_TIME_SCALE", "1"))  # (sanitizer builds run slower)
    extra = ["--const", "--inplace", "--verify-restore-ms", "100", "--n", str(1 << 19), "--pool", "2", "--duration",
             str(16 * scale), "--rejoin", "--max-failures", "30"] + (["--quant", "u8"] if point.startswith("qring") else [])
    stop = dict(dev, PCCL_FAULT_INJECT=point, PCCL_FAULT_SIGNAL="STOP")
    with local_master() as addr:
        ps = [spawn_python([WORKER, addr, "3", str(r), "--device", "cpu", *extra], env=stop if r == 0 else dev,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
        run = _Run(ps, 150 * scale)
        _wait_until(lambda: _proc_state(ps[0].pid) == "T" or ps[0].poll() is not None, 60 * scale,
                    "the victim to stop")
        t_stop = time.time()
        assert ps[0].poll() is None
        time.sleep(5.0)
        os.kill(ps[0].pid, signal.SIGCONT)
        outs = run.join()
    for r in range(3):
        assert ps[r].returncode == 0, (r, outs[r][1][-3000:])
    for r in (1, 2):
        lines = _lines(outs[r][0])
        assert all(x["path"] == 2 for x in lines if "path" in x), lines[-3:]
        detect, after = _check_survivor(lines, t_stop, PEER_TIMEOUT_S + 2.0)
        print(f"peer {r}: failed op {detect:.2f} s after the stop")
        assert any(x["world"] == 3 for x in after), "the resumed peer did not rejoin"


@pytest.mark.gpu
@pytest.mark.parametrize("point", ["ring:20:1:rx", "ring:20:2:publish", "qring:20:1:meta"])
def test_gpu_sigstopped_peer_device_ring(hip, monkeypatch, point):
    """TCP device ring (PCCL_DISABLE_IPC=1), 16 Mi bf16 in place, plain and uint8-quantized: peer 0 stops inside a
    ring step (its copies / kernels of that step in flight, or its step's sends published, or its metadata packet
    sent); survivors fail within the peer timeout + 2 s, drain their own copies and kernels before restoring the
    input (re-read 200 ms later, bit-exact), continue at W = 2 on the device ring, and the resumed peer rejoins."""
    extra = ("--quant", "u8") if point.startswith("qring") else ()
    _, outs = _gpu_stop_run(monkeypatch, point, {"PCCL_DISABLE_IPC": "1"}, 1 << 24, extra)
    for r in (1, 2):
        assert all(x["path"] == 2 for x in _lines(outs[r][0]) if "path" in x)


@pytest.mark.gpu
def test_gpu_sigstopped_peer_ipc(hip, monkeypatch):
    """xGMI / IPC path, 3 processes on one GPU, 64 Mi bf16 in place: peer 0 stops right after publishing its vote
    for op seq 20, so the survivors pass the vote barrier and run their push kernels into its exported buffers, then
    wait for it in the gathered barrier. The master drops it after PCCL_PEER_TIMEOUT_MS; the survivors abort, do not
    wait for the stopped peer (it stopped before its pre-launch check, so on resume it sees the abort and never
    launches into their restored buffers: IpcArena::run), restore their input bit-exactly and continue on the IPC path
    at W = 2; the resumed peer fails cleanly and rejoins."""
    _, outs = _gpu_stop_run(monkeypatch, "ipc_vote:20", {}, 1 << 26)
    for r in (1, 2):
        assert all(x["path"] == 3 for x in _lines(outs[r][0]) if "path" in x)
