"""BASELINE config 5: kill + rejoin 1 of 8 peers mid-all-reduce, then re-solve the ring topology (ATSP).

    python benchmarks/fault_tolerance.py [--peers 8] [--mib 64] [--device cuda:0|cpu]

Peer processes and an in-process master on 127.0.0.1 run a loop of AVG all-reduces of --mib MiB (constant inputs,
so every result is checkable: value 1.0 -> result 1.0 whatever the world size) and log a timestamp per completed or
failed op. The driver
  1. lets the 8 peers run, then SIGKILLs one of them mid-run (no clean disconnect),
  2. starts a replacement peer after --respawn-after seconds,
  3. once the replacement has completed an all-reduce, every peer calls pcclOptimizeTopology (bandwidth probes
     between peers + asymmetric TSP solve on the master) and keeps reducing on the new ring.
Reported: ops that failed because of the kill, recovery time (kill -> first successful op of the 7 survivors),
rejoin time (replacement process started -> its first successful op; and from its connect() call, i.e. without the
Python/torch start-up), topology re-solve time, steady-state ms/op before
the kill, with 7 peers and after the rejoin, and whether every result was exact.
The reference publishes no number for this configuration.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def peer(a):
    import torch

    import pccl_amd as pccl
    from pccl_amd.utils import wait_for_world
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    print(json.dumps({"rank": a.rank, "t": time.time(), "event": "connecting"}), flush=True)
    comm = pccl.Communicator(a.master, 0, p2p_connection_pool_size=a.pool)
    comm.connect(n_attempts=120)
    if not a.joiner:
        wait_for_world(comm, a.peers, timeout=300)
    n = (a.mib << 20) // 4
    x = torch.ones(n, device=dev)
    y = torch.empty_like(x)

    def log(**kw):
        print(json.dumps({"rank": a.rank, "t": time.time(), **kw}), flush=True)

    log(event="start")
    optimized = False
    seen_small_world = False
    left = a.stop_after_optimize
    it = 0
    while time.time() < a.deadline:
        if it > 0 and comm.are_peers_pending():
            comm.update_topology()
        it += 1
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        if ws < 2:
            time.sleep(0.01)
            continue
        seen_small_world |= ws < a.peers
        try:
            t0 = time.perf_counter()
            info = comm.all_reduce(x, y, op=pccl.ReduceOp.AVG, tag=0)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ok = bool(torch.all(y == 1.0))
            log(event="ok", world=info.local_world_size, sec=dt, exact=ok)
        except pccl.PCCLError as e:
            log(event="fail", error=e.result.name)
            continue
        # the first op in which the replacement took part: everyone (incl. the replacement) re-solves the ring
        if not optimized and info.local_world_size == a.peers and (a.joiner or seen_small_world):
            t0 = time.perf_counter()
            try:
                comm.optimize_topology()
                log(event="optimized", sec=time.perf_counter() - t0)
            except pccl.PCCLError as e:
                log(event="optimize_failed", error=e.result.name, sec=time.perf_counter() - t0)
            optimized = True
        if optimized:
            left -= 1
            if left <= 0:
                break
    comm.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--pool", type=int, default=2)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--kill-after", type=float, default=3.0)
    ap.add_argument("--respawn-after", type=float, default=1.0)
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--master", default=None)
    ap.add_argument("--joiner", action="store_true")
    ap.add_argument("--deadline", type=float, default=0)
    ap.add_argument("--stop-after-optimize", type=int, default=20)
    ap.add_argument("--no-ipc", action="store_true",
                    help="device ring over TCP instead of the xGMI IPC path (default: IPC, which survives a peer "
                         "SIGKILLed mid-kernel since round 2; tests/test_fault_tolerance.py::test_gpu_ipc_sigkill_mid_op)")
    ap.add_argument("--log-dir", default=None, help="keep every peer's stderr here")
    a = ap.parse_args()
    if a.rank is not None:
        return peer(a)

    from pccl_amd.utils import local_master, spawn_python
    me = os.path.abspath(__file__)
    deadline = time.time() + 240
    common = ["--peers", str(a.peers), "--mib", str(a.mib), "--pool", str(a.pool), "--device", a.device,
              "--deadline", str(deadline), "--stop-after-optimize", str(a.stop_after_optimize)]
    env = {"PCCL_BENCHMARK_MILLIS": "300", "PCCL_NUM_BENCHMARK_CONNECTIONS": "2", "PCCL_SAME_HOST_MBPS": "0"}
    if a.no_ipc:
        env["PCCL_DISABLE_IPC"] = "1"
    lines = []
    lock = threading.Lock()
    if a.log_dir:
        os.makedirs(a.log_dir, exist_ok=True)

    def reader(p):
        for ln in p.stdout:
            if ln.startswith("{"):
                with lock:
                    lines.append(json.loads(ln))

    with local_master() as addr:
        procs, threads = [], []

        def start(rank, joiner=False):
            # a file, not a pipe: a chatty peer must never block on stderr
            err = open(os.path.join(a.log_dir, f"peer{rank}.err"), "w+") if a.log_dir else \
                tempfile.TemporaryFile(mode="w+")
            p = spawn_python([me, "--rank", str(rank), "--master", addr, *common] + (["--joiner"] if joiner else []),
                             env=env, stdout=subprocess.PIPE, stderr=err, text=True, start_new_session=True)
            p.err_file = err
            t = threading.Thread(target=reader, args=(p,), daemon=True)
            t.start()
            procs.append(p)
            threads.append(t)
            return p

        for r in range(a.peers):
            start(r)

        def oks(rank=None, world=None, after=0.0):
            with lock:
                return [x for x in lines if x["event"] == "ok" and (rank is None or x["rank"] == rank)
                        and (world is None or x["world"] == world) and x["t"] > after]

        def progress(what):
            print(json.dumps({"progress": what, "t": time.time(), "ops": len(oks())}), flush=True)

        while len(oks(world=a.peers)) < 3 * a.peers and time.time() < deadline:
            time.sleep(0.05)
        progress("running")
        time.sleep(a.kill_after)
        victim = procs[a.peers - 1]
        t_kill = time.time()
        os.killpg(victim.pid, signal.SIGKILL)  # its own session: only that peer's process group
        victim.wait()
        progress("killed")
        while not oks(world=a.peers - 1, after=t_kill) and time.time() < deadline:
            time.sleep(0.01)
        progress("recovered")
        time.sleep(a.respawn_after)
        t_spawn = time.time()
        start(a.peers, joiner=True)
        while not oks(rank=a.peers) and time.time() < deadline:
            time.sleep(0.01)
        progress("rejoined")
        for p in procs[:a.peers - 1] + procs[a.peers:]:
            try:
                p.wait(timeout=max(1.0, deadline - time.time() + 30))
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        for t in threads:
            t.join(timeout=5)
        errs = []
        for p in procs:
            if p.returncode not in (0, -signal.SIGKILL):
                p.err_file.seek(0)
                errs.append(p.err_file.read()[-2000:])

    def ms_per_op(sel):
        return round(1e3 * sorted(x["sec"] for x in sel)[len(sel) // 2], 3) if sel else None

    before = [x for x in oks(world=a.peers) if x["t"] < t_kill]
    seven = [x for x in oks(world=a.peers - 1) if x["t"] > t_kill]
    rejoin = oks(rank=a.peers)
    after = [x for x in oks(world=a.peers) if x["t"] > t_spawn]
    fails = [x for x in lines if x["event"] == "fail" and x["t"] > t_kill]
    opt = [x for x in lines if x["event"] in ("optimized", "optimize_failed")]
    connecting = [x["t"] for x in lines if x["event"] == "connecting" and x["rank"] == a.peers]
    print(json.dumps({
        "metric": "fault tolerance: kill + rejoin", "config": "Fault tolerance: kill + rejoin 1 of 8 peers "
        "mid-all-reduce, TSP topology re-solve", "peers": a.peers, "mib": a.mib, "device": a.device,
        "failed_ops_after_kill": len(fails),
        "recovery_ms": round(1e3 * (min(x["t"] for x in seven) - t_kill), 1) if seven else None,
        "rejoin_ms": round(1e3 * (min(x["t"] for x in rejoin) - t_spawn), 1) if rejoin else None,
        "rejoin_from_connect_ms": round(1e3 * (min(x["t"] for x in rejoin) - connecting[0]), 1)
        if rejoin and connecting else None,
        "topology_resolve_ms": round(1e3 * max(x["sec"] for x in opt), 1) if opt else None,
        "topology_resolve_ok": bool(opt) and all(x["event"] == "optimized" for x in opt),
        "ms_per_op": {"before_kill": ms_per_op(before), "after_kill": ms_per_op(seven),
                      "after_rejoin": ms_per_op(after)},
        "all_results_exact": all(x["exact"] for x in oks()), "peer_errors": errs}), flush=True)


if __name__ == "__main__":
    main()
