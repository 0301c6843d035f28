"""Elastic stress test: peers with cross-step background reduces are killed (SIGKILL) and respawned at random while
the run continues (reference python/tests/stress_tests/*/stresstest_orchestrator.py). Asserts: no wrong reduce result
ever, survivors keep making progress, every peer alive at the end exits cleanly.

Soak mode (the reference orchestrator runs 8 h): PCCL_STRESS_SECONDS=28800 [PCCL_STRESS_PEERS=8] runs the same loop
for that long with the reference's schedule (every 0.5-2 s: spawn with p = 0.6, SIGKILL with p = 0.4, never below 2
alive); the GPU variant puts every peer's tensors on cuda:0 (xGMI/IPC path, kills land mid-kernel).
"""
import json
import os
import random
import signal
import subprocess
import time

import pytest

from pccl_amd.utils import local_master, spawn_python

HERE = os.path.dirname(os.path.abspath(__file__))
PEER = os.path.join(HERE, "workers", "stress_peer.py")


def _run_stress(tmp_path, duration, target, device="cpu", soak=False, env=None, stop_p=0.0):
    """`stop_p`: share of the victims that are SIGSTOPped instead (a hung peer: its sockets stay open, only the
    liveness protocol notices) and SIGKILLed 4 s later."""
    rng = random.Random(int(os.environ.get("PCCL_STRESS_SEED", "1234")))
    stop = tmp_path / "stop"
    procs, killed, signalled = [], 0, set()
    hung = []  # (process, time to SIGKILL it)

    def hit(victim):
        if rng.random() < stop_p:
            victim.send_signal(signal.SIGSTOP)
            hung.append((victim, time.time() + 4.0))
        else:
            victim.send_signal(signal.SIGKILL)
    with local_master() as addr:
        def spawn():
            # stdout to a file: a long soak must never block a peer on a full pipe
            out = open(tmp_path / f"peer{len(procs)}.out", "w+")
            procs.append((spawn_python([PEER, addr, str(stop)], env={"OMP_NUM_THREADS": "1", "STRESS_DEVICE": device,
                                                                     **(env or {})},
                                       stdout=out, stderr=subprocess.STDOUT, text=True), out))
        for _ in range(target):
            spawn()
        t_end = time.time() + duration
        t_report = time.time() + 30
        while time.time() < t_end:
            for v, t_kill in [h for h in hung if time.time() >= h[1]]:
                v.send_signal(signal.SIGKILL)
                hung.remove((v, t_kill))
            # a SIGKILLed GPU process can take a while to exit: never pick (or count) it twice
            alive = [p for p, _ in procs if p.poll() is None and p.pid not in signalled]
            if soak and time.time() >= t_report:  # progress of a long soak (run pytest with -s to see it live)
                t_report = time.time() + 30
                print(f"[soak] {duration - (t_end - time.time()):.0f}/{duration:.0f} s: {len(alive)} alive, "
                      f"{killed} killed, {len(procs)} spawned", flush=True)
            if soak:  # reference schedule
                time.sleep(rng.uniform(0.5, 2.0))
                if rng.random() < 0.4 and len(alive) > 2:
                    victim = rng.choice(alive)
                    hit(victim)
                    signalled.add(victim.pid)
                    killed += 1
                if rng.random() < 0.6 and len(alive) < 2 * target:
                    spawn()
                continue
            time.sleep(rng.uniform(2.0, 4.0))
            if len(alive) > 2:
                victim = rng.choice(alive)
                hit(victim)
                signalled.add(victim.pid)
                killed += 1
            if len([p for p, _ in procs if p.poll() is None and p.pid not in signalled]) < target:
                spawn()
        for v, _ in hung:
            v.send_signal(signal.SIGKILL)
        stop.write_text("1")
        for p, out in procs:
            try:
                p.wait(timeout=90)
            except subprocess.TimeoutExpired:
                # stacks of every peer still running (the one that does not stop may wait for another one)
                alive = [q for q, _ in procs if q.poll() is None]
                for q in alive:
                    q.send_signal(signal.SIGUSR1)  # faulthandler: dump every thread's Python stack
                time.sleep(1)
                for q in alive:
                    q.send_signal(signal.SIGUSR2)  # native backtraces of every thread (PCCL_DEBUG_BACKTRACE_SIGNAL)
                time.sleep(2)
                for q in alive:
                    q.kill()
                    q.wait()
                dump = os.environ.get("PCCL_STRESS_DUMP_DIR")  # every peer's whole output, for the post-mortem
                if dump:
                    os.makedirs(dump, exist_ok=True)
                    for k, (q, o) in enumerate(procs):
                        o.seek(0)
                        with open(os.path.join(dump, f"peer{k}{'_alive' if q in alive else ''}.out"), "w") as f:
                            f.write(f"pid {q.pid}\n" + o.read())
                out.seek(0)
                raise AssertionError("peer did not stop:\n" + out.read()[-6000:])
    summaries, progress = [], 0
    for p, out in procs:
        out.seek(0)
        text = out.read()
        out.close()
        lines = [json.loads(x) for x in text.splitlines() if x.startswith("{")]
        progress += max([x["progress"] for x in lines if "progress" in x], default=0)
        if p.returncode == -signal.SIGKILL:
            continue
        assert p.returncode == 0, text[-3000:]
        ends = [x for x in lines if "steps" in x or "kicked" in x]
        assert ends, text[-2000:]
        summaries.append(ends[-1])
    print(f"[stress] {killed} hit, {len(procs)} spawned, progress {progress} peer-steps", flush=True)
    return killed, summaries, progress


def test_random_kill_respawn(tmp_path):
    duration = float(os.environ.get("PCCL_STRESS_SECONDS", "25"))
    soak = duration > 60
    killed, summaries, progress = _run_stress(tmp_path, duration, int(os.environ.get("PCCL_STRESS_PEERS", "4")),
                                              soak=soak)
    assert killed >= 3
    assert summaries and all(s["bad"] == 0 for s in summaries), summaries
    assert progress > 10, (progress, summaries)  # successful steps of every peer of the run, the killed ones too


def test_random_stop_kill_respawn(tmp_path, monkeypatch):
    """The same churn with half of the victims hung instead of killed (SIGSTOP, SIGKILLed 4 s later): the master drops a
    hung peer after PCCL_PEER_TIMEOUT_MS (2 s here) while its sockets are still open, and the survivors keep making
    progress with exact results."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", "2000")
    duration = float(os.environ.get("PCCL_STRESS_SECONDS", "30"))
    killed, summaries, progress = _run_stress(tmp_path, duration, 4, soak=duration > 60, stop_p=0.5)
    assert killed >= 3
    assert summaries and all(s["bad"] == 0 for s in summaries), summaries
    assert progress > 10, (progress, summaries)  # successful steps of every peer of the run, the killed ones too


HOSTDEV = os.environ.get("PCCL_TEST_HOSTDEV") or os.path.join(os.path.dirname(HERE), "pccl_amd", "lib",
                                                              "libpccl_hostdev.so")


def test_random_stop_kill_respawn_emulated_device(tmp_path, monkeypatch):
    """The hung / killed peer churn on the device rings, on the CPU: the host-emulated device backend (every pointer is
    device memory, streams are worker threads) runs the small-message path for the 16-96 KiB tensors and the staged
    pipeline for a 4 MiB one, with their abort polls - the code a GPU soak hung in when a poll took the master's abort
    packet and the op still finished (docs/ROUND6_RESPONSE.md)."""
    if not os.path.exists(HOSTDEV) or os.environ.get("PCCL_DISABLE_HIP") == "1":
        pytest.skip("libpccl_hostdev.so not built, or device plugins disabled (PCCL_DISABLE_HIP)")
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", "2000")
    duration = float(os.environ.get("PCCL_STRESS_SECONDS", "30"))
    env = {"PCCL_HIP_PLUGIN": HOSTDEV, "PCCL_HOSTDEV_ALL_DEVICE": "1", "PCCL_DISABLE_IPC": "1", "STRESS_BIG_MIB": "4"}
    killed, summaries, progress = _run_stress(tmp_path, duration, 4, soak=duration > 60, env=env, stop_p=0.5)
    assert killed >= 3
    assert summaries and all(s["bad"] == 0 for s in summaries), summaries
    assert progress > 10, (progress, summaries)  # successful steps of every peer of the run, the killed ones too


@pytest.mark.gpu
def test_random_kill_respawn_gpu_ipc(tmp_path, hip):
    """Device tensors on cuda:0: the peers reduce over the xGMI/IPC path, so SIGKILLs land during IPC votes and
    kernels; no wrong result, survivors progress, everyone alive at the end exits cleanly."""
    duration = float(os.environ.get("PCCL_STRESS_SECONDS", "30"))
    killed, summaries, progress = _run_stress(tmp_path, duration, 4, device="cuda:0", soak=duration > 60)
    assert killed >= 3
    assert summaries and all(s["bad"] == 0 for s in summaries), summaries
    assert progress > 10, (progress, summaries)  # successful steps of every peer of the run, the killed ones too


@pytest.mark.gpu
def test_random_kill_respawn_gpu_ring(tmp_path, hip):
    """The same random SIGKILL / respawn schedule on the loopback-TCP device ring (PCCL_DISABLE_IPC=1) with a 64 MiB
    tensor per step next to the small ones, so kills land mid-pipeline (staging copies, fused reduce kernels and
    send-ahead stripes in flight): no wrong result, survivors progress, everyone alive at the end exits cleanly."""
    duration = float(os.environ.get("PCCL_STRESS_SECONDS", "30"))
    killed, summaries, progress = _run_stress(tmp_path, duration, 4, device="cuda:0", soak=duration > 60,
                                    env={"PCCL_DISABLE_IPC": "1", "STRESS_BIG_MIB": "64"})
    assert killed >= 3
    assert summaries and all(s["bad"] == 0 for s in summaries), summaries
    assert progress > 10, (progress, summaries)  # successful steps of every peer of the run, the killed ones too


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["ring", "ipc"])
def test_random_stop_kill_respawn_gpu(tmp_path, hip, monkeypatch, path):
    """Hung and killed peers at random on cuda:0 (PCCL_PEER_TIMEOUT_MS 2 s): on the TCP device ring with a 64 MiB
    tensor per step (hangs land mid-pipeline) and on the xGMI path (hangs land around votes and kernels); no wrong
    result, survivors progress, everyone alive at the end exits cleanly."""
    monkeypatch.setenv("PCCL_PEER_TIMEOUT_MS", "2000")
    duration = float(os.environ.get("PCCL_STRESS_SECONDS", "30"))
    env = {"PCCL_DISABLE_IPC": "1", "STRESS_BIG_MIB": "64"} if path == "ring" else None
    killed, summaries, progress = _run_stress(tmp_path, duration, 4, device="cuda:0", soak=duration > 60, env=env,
                                              stop_p=0.5)
    assert killed >= 3
    assert summaries and all(s["bad"] == 0 for s in summaries), summaries
    assert progress > 10, (progress, summaries)  # successful steps of every peer of the run, the killed ones too
