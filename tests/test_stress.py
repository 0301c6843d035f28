"""Elastic stress test: peers with cross-step background reduces are killed (SIGKILL) and respawned at random while
the run continues (reference python/tests/stress_tests/*/stresstest_orchestrator.py). Asserts: no wrong reduce result
ever, survivors keep making progress, every peer alive at the end exits cleanly."""
import json
import os
import random
import signal
import subprocess
import time

from pccl_amd.utils import local_master, spawn_python

HERE = os.path.dirname(os.path.abspath(__file__))
PEER = os.path.join(HERE, "workers", "stress_peer.py")


def test_random_kill_respawn(tmp_path):
    rng = random.Random(1234)
    stop = tmp_path / "stop"
    duration, target = 25.0, 4
    procs, killed = [], 0
    with local_master() as addr:
        def spawn():
            procs.append(spawn_python([PEER, addr, str(stop)], env={"OMP_NUM_THREADS": "1"},
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        for _ in range(target):
            spawn()
        t_end = time.time() + duration
        while time.time() < t_end:
            time.sleep(rng.uniform(2.0, 4.0))
            alive = [p for p in procs if p.poll() is None]
            if len(alive) > 2:
                victim = rng.choice(alive)
                victim.send_signal(signal.SIGKILL)
                killed += 1
            if len([p for p in procs if p.poll() is None]) < target:
                spawn()
        stop.write_text("1")
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=90))
            except subprocess.TimeoutExpired:
                p.send_signal(signal.SIGUSR1)  # faulthandler: dump every thread's Python stack
                time.sleep(1)
                p.kill()
                o, e = p.communicate()
                raise AssertionError("peer did not stop:\n" + e[-6000:])
    summaries = []
    for p, (o, e) in zip(procs, outs):
        if p.returncode == -signal.SIGKILL:
            continue
        assert p.returncode == 0, e[-3000:]
        lines = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
        assert lines, e[-2000:]
        summaries.append(lines[-1])
    assert killed >= 3
    assert summaries and all(s["bad"] == 0 for s in summaries), summaries
    assert sum(s["ok_ops"] for s in summaries) > 10, summaries
