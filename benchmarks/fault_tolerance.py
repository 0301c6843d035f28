"""BASELINE config 5: kill + rejoin 1 of 8 peers mid-all-reduce, then re-solve the ring topology (ATSP).

    python benchmarks/fault_tolerance.py [--peers 8] [--mib 1024] [--device cuda:0|cpu] [--transport tcp|ipc]

One process per peer (the deployment shape) and a master in this process on 127.0.0.1. Every peer runs a loop of
in-place SUM all-reduces of --mib MiB (bf16 on a GPU, fp32 on the CPU) whose input is 1.0 everywhere, so every result
is checkable (== the op's world size) and every failed op's buffer must hold the input again (1.0: the in-place
restore). The sequence (reference python/tests/stress_tests/basic_stress_test/stresstest_orchestrator.py:88-262,
ccoip/src/cpp/ccoip_master_handler.cpp:1312-1400):
  1. the last peer SIGKILLs itself in the middle of op --kill-op (PCCL_FAULT_INJECT: on the TCP device ring when its
     first received piece of reduce-scatter step 1 is in flight, on the xGMI path right after launching its push
     kernel, on the host ring after its first received frame of step 1); the fault line carries the kill's wall time;
  2. the master sees the connection drop and aborts the op; the survivors' op fails, they re-form the ring without
     the dead peer and keep reducing with W-1 peers;
  3. once every survivor completed an op at W-1, a replacement process starts; the survivors admit it at their next
     op boundary (pcclArePeersPending / pcclUpdateTopology);
  4. at the first op with W peers again every peer calls pcclOptimizeTopology (pairwise bandwidth probes, then the
     master's asymmetric-TSP solve) and keeps reducing on the new ring.
With --signal stop the victim SIGSTOPs itself instead (PCCL_FAULT_SIGNAL=STOP: its sockets stay open and its kernel
keeps ACKing, so no connection ever closes): the master drops it once its heartbeats stop (PCCL_PEER_TIMEOUT_MS,
--peer-timeout-ms) and the survivors' op fails through the liveness path (docs/ARCHITECTURE.md); the stopped victim is
SIGKILLed after the survivors' first op at W-1 (cleanup) and the replacement joins as above. The fields are then named
stop_to_* instead of kill_to_*.
Reported (ms): kill -> survivors' failed op returned (abort received + ring re-formed), kill -> survivors' first exact
op at W-1, replacement's connect() -> its first exact op at W (its process start too), the admission vote, the
optimize call and the master's ATSP solve alone; ms per op in each phase (``after_rejoin`` holds each peer's first op
at W again, which waits for the replacement's first initiate: ~87 ms of a 111 ms xGMI op, profiles/r5/b6/
ft_ipc_traces/, the later ops are as fast as before the kill); the replacement's first op and the staging memory it had
to allocate; whether every result and every restore was exact. The reference publishes no number for this
configuration.
"""
from __future__ import annotations

import time

T_PROC = time.time()  # before any import: a replacement's process start

import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import re  # noqa: E402
import signal  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402
import tempfile  # noqa: E402
import threading  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def peer(a):
    import torch

    import pccl_amd as pccl
    from pccl_amd.utils import wait_for_world
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)

    def log(**kw):
        print(json.dumps({"rank": a.rank, "t": time.time(), **kw}), flush=True)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    log(event="proc_start", t_proc=T_PROC)
    # the peer's tensor exists before it connects, as in the reference's stress-test peer (its weights are created
    # before connect(), stresstest_peer.py:134-144): allocating and first touching 1 GiB of HBM is the application's
    # start-up, not part of the rejoin
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    x = torch.empty((a.mib << 20) // (2 if dtype == torch.bfloat16 else 4), device=dev, dtype=dtype)
    x.fill_(1.0)
    sync()
    comm = pccl.Communicator(a.master, 0, p2p_connection_pool_size=a.pool)
    t0 = time.time()
    log(event="connect_call")
    # the device ring's staging for this op size fills the library's pools while connect() waits for admission
    # (inside the measured connect -> first op window; a fresh process otherwise allocates it in its first op)
    reserve = None
    if dev.type == "cuda" and a.transport == "tcp" and not a.no_reserve:
        reserve = threading.Thread(target=pccl.memory.reserve_device_ring_staging,
                                   args=(a.mib << 20, a.peers), kwargs={"device": dev, "in_place": True}, daemon=True)
        reserve.start()
    comm.connect(n_attempts=120)
    log(event="connected", sec=time.time() - t0)
    if reserve is not None:
        reserve.join()
    if not a.joiner:
        wait_for_world(comm, a.peers, timeout=300)
    optimized = False
    saw_small = False
    post = 0
    it = 0
    while time.time() < a.deadline:
        # the pending query is a vote of every member at the same point of an iteration: a replacement enters right
        # after the others' admission (their update_topology of this iteration), so nobody asks in iteration 0
        it += 1
        if it > 1 and comm.are_peers_pending():
            t0 = time.perf_counter()
            comm.update_topology()
            log(event="admit", sec=time.perf_counter() - t0)
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        if ws < 2:
            time.sleep(0.005)
            continue
        x.fill_(1.0)
        sync()
        pools0 = pccl.memory.staging_pool_stats()
        t0 = time.perf_counter()
        try:
            info = comm.all_reduce(x, x, op=pccl.ReduceOp.SUM, tag=0)  # in place
            sync()
            dt = time.perf_counter() - t0
            w = info.local_world_size
            exact = bool((x == float(w)).all())
            pools = pccl.memory.staging_pool_stats()
            # staging memory the op had to allocate (pool misses: a fresh process's first ops)
            alloc_ms = sum(pools[k].get("alloc_us", 0) - pools0[k].get("alloc_us", 0) for k in pools) / 1e3
            log(event="ok", world=w, sec=dt, exact=exact, path=comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH),
                alloc_ms=alloc_ms)
        except pccl.PCCLError as e:
            t_fail = time.time()
            sync()
            restore_ok = bool((x == 1.0).all())  # the failed in-place op's buffer holds its input again
            log(event="fail", t_fail=t_fail, sec=time.perf_counter() - t0, error=e.result.name, restore_ok=restore_ok)
            continue
        saw_small |= w < a.peers
        # the first op with the full world again (the replacement's first op): everyone re-solves the ring
        if not optimized and w == a.peers and (a.joiner or saw_small):
            t0 = time.perf_counter()
            try:
                comm.optimize_topology()
                log(event="optimized", sec=time.perf_counter() - t0)
            except pccl.PCCLError as e:
                log(event="optimize_failed", error=e.result.name, sec=time.perf_counter() - t0)
            optimized = True
            continue
        if optimized:
            post += 1
            if post >= a.post_ops:
                break
    comm.destroy()


def _proc_state(pid: int):
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0]
    except (OSError, IndexError):
        return None


def inject_spec(device: str, transport: str, op: int) -> str:
    """PCCL_FAULT_INJECT of the victim: where in op `op` (the master's sequence number) it SIGKILLs itself."""
    if not device.startswith("cuda"):
        return f"hring:{op}:1:rx"
    return f"ipc_kernel:{op}" if transport == "ipc" else f"ring:{op}:1:rx"


def run(a) -> dict:
    import pccl_amd as pccl
    from pccl_amd.utils import free_port, spawn_python
    me = os.path.abspath(__file__)
    deadline = time.time() + a.timeout
    port = free_port()
    addr = f"127.0.0.1:{port}"
    if a.peer_timeout_ms is not None:  # read by the master (this process) when it is created
        os.environ["PCCL_PEER_TIMEOUT_MS"] = str(a.peer_timeout_ms)
    master = pccl.MasterNode(addr)
    master.run()
    common = ["--peers", str(a.peers), "--mib", str(a.mib), "--pool", str(a.pool), "--device", a.device,
              "--deadline", str(deadline), "--post-ops", str(a.post_ops), "--master", addr, "--transport", a.transport,
              *(["--no-reserve"] if a.no_reserve else [])]
    # short bandwidth probes (the reference's 10 s per pair is a WAN setting); several processes on one GPU: 2 hardware
    # queues each (README)
    env = {"PCCL_BENCHMARK_MILLIS": str(a.probe_ms), "PCCL_NUM_BENCHMARK_CONNECTIONS": "2",
           "PCCL_SAME_HOST_MBPS": "0", "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "2")}
    if a.transport == "tcp":
        env["PCCL_DISABLE_IPC"] = "1"
    spec = inject_spec(a.device, a.transport, a.kill_op)
    stop = a.signal == "stop"
    victim_env = {"PCCL_FAULT_INJECT": spec, **({"PCCL_FAULT_SIGNAL": "STOP"} if stop else {})}
    lines, procs, errs_files = [], [], []
    lock = threading.Lock()

    def reader(p):
        for ln in p.stdout:
            if ln.startswith("{"):
                with lock:
                    lines.append(json.loads(ln))

    def start(rank, joiner=False, extra_env=None):
        # a file, not a pipe: a chatty peer never blocks on stderr
        err = open(os.path.join(a.log_dir, f"peer{rank}.err"), "w+") if a.log_dir else tempfile.TemporaryFile(mode="w+")
        p = spawn_python([me, "--rank", str(rank), *common] + (["--joiner"] if joiner else []),
                         env=dict(env, **(extra_env or {})), stdout=subprocess.PIPE, stderr=err, text=True,
                         start_new_session=True)
        errs_files.append(err)
        threading.Thread(target=reader, args=(p,), daemon=True).start()
        procs.append(p)
        return p

    def sel(event, rank=None, world=None, after=0.0):
        with lock:
            return [x for x in lines if x["event"] == event and (rank is None or x["rank"] == rank)
                    and (world is None or x.get("world") == world) and x["t"] > after]

    victim_rank = a.peers - 1
    t_kill = None
    t_spawn = None
    t_victim_gone = None
    try:
        for r in range(a.peers):
            start(r, extra_env=victim_env if r == victim_rank else None)
        victim = procs[victim_rank]
        while victim.poll() is None and time.time() < deadline and not (stop and _proc_state(victim.pid) == "T"):
            time.sleep(0.002)
        t_victim_gone = time.time()  # reaped (its address space torn down, then its sockets closed) / stopped
        errs_files[victim_rank].seek(0)
        m = re.search(r"fault injection: SIG(?:KILL|STOP) at .* t=(\d+\.\d+)", errs_files[victim_rank].read())
        t_kill = float(m.group(1)) if m else None
        survivors = [r for r in range(a.peers) if r != victim_rank]
        while t_kill is not None and time.time() < deadline and \
                not all(sel("ok", rank=r, world=a.peers - 1, after=t_kill) for r in survivors):
            time.sleep(0.01)
        if stop and victim.poll() is None:  # stopped, dropped by the master: clean it up before the replacement
            os.killpg(victim.pid, signal.SIGKILL)
            victim.wait()
        t_spawn = time.time()
        start(a.peers, joiner=True)
        for p in procs:
            try:
                p.wait(timeout=max(1.0, deadline - time.time() + 30))
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        time.sleep(0.2)  # readers drain
        topo = master.topology_stats()
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        master.interrupt()
        master.await_termination()

    errs = []
    for k, p in enumerate(procs):
        if p.returncode not in (0, -signal.SIGKILL) or (k != victim_rank and p.returncode != 0):
            errs_files[k].seek(0)
            errs.append({"rank": k, "rc": p.returncode, "stderr": errs_files[k].read()[-1500:]})

    def ms(v):
        return round(v * 1e3, 1) if v is not None else None

    def med_ms(xs):
        return round(1e3 * sorted(x["sec"] for x in xs)[len(xs) // 2], 2) if xs else None

    survivors = [r for r in range(a.peers) if r != victim_rank]
    joiner = a.peers
    fails = [x for x in sel("fail") if t_kill is not None and x["t"] > t_kill]
    first_fail = [min((x["t_fail"] for x in fails if x["rank"] == r), default=None) for r in survivors]
    first_small = [min((x["t"] for x in sel("ok", rank=r, world=a.peers - 1, after=t_kill or 0)), default=None)
                   for r in survivors]
    j_ok = sel("ok", rank=joiner, world=a.peers)
    j_first = min((x["t"] for x in j_ok), default=None)
    j_connect = [x["t"] for x in sel("connect_call", rank=joiner)]
    j_proc = [x["t_proc"] for x in sel("proc_start", rank=joiner)]
    opt = sel("optimized") + sel("optimize_failed")
    admits = [x for x in sel("admit") if t_spawn is not None and x["t"] > t_spawn]
    t_opt_end = max((x["t"] for x in opt), default=None)
    oks = sel("ok")
    full_before = [x for x in oks if x["world"] == a.peers and t_kill is not None and x["t"] < t_kill]
    small = [x for x in oks if x["world"] == a.peers - 1]
    rejoined = [x for x in oks if x["world"] == a.peers and t_spawn is not None and x["t"] > t_spawn
                and (t_opt_end is None or x["t"] < t_opt_end)]
    after_opt = [x for x in oks if x["world"] == a.peers and t_opt_end is not None and x["t"] > t_opt_end]
    complete = t_kill is not None and None not in first_fail and None not in first_small and j_first is not None
    ev = "stop" if stop else "kill"
    return {
        "config": f"BASELINE config 5: {'SIGSTOP (no socket closes)' if stop else 'kill'} + rejoin 1 of {a.peers} "
                  f"peers mid-all-reduce, TSP topology re-solve",
        "fault_signal": "SIGSTOP" if stop else "SIGKILL",
        "peer_timeout_ms": (a.peer_timeout_ms if a.peer_timeout_ms is not None else
                            int(os.environ.get("PCCL_PEER_TIMEOUT_MS", "10000"))) if stop else None,
        "transport": "xGMI/IPC" if a.transport == "ipc" and a.device.startswith("cuda") else
        ("TCP device ring" if a.device.startswith("cuda") else "TCP host ring"),
        "peers": a.peers, "processes": "one per peer", "mib": a.mib, "device": a.device, "inject": spec,
        "complete": complete,
        f"{ev}_to_victim_{'stopped' if stop else 'reaped'}_ms": ms(t_victim_gone - t_kill) if t_kill is not None else None,
        f"{ev}_to_survivors_failed_op_ms": ms(max(first_fail) - t_kill) if complete else None,
        f"{ev}_to_survivors_first_exact_op_ms": ms(max(first_small) - t_kill) if complete else None,
        "joiner_connect_to_first_exact_op_ms": ms(j_first - j_connect[0]) if j_first and j_connect else None,
        "joiner_process_start_to_first_exact_op_ms": ms(j_first - j_proc[0]) if j_first and j_proc else None,
        # connect() returns once the survivors admitted the replacement at their next op boundary and the ring with it
        # is established
        "joiner_connect_call_ms": ms(sel("connected", rank=joiner)[0]["sec"]) if sel("connected", rank=joiner) else None,
        "joiner_first_op_ms": round(1e3 * min(j_ok, key=lambda x: x["t"])["sec"], 1) if j_ok else None,
        "joiner_first_op_staging_alloc_ms": round(min(j_ok, key=lambda x: x["t"]).get("alloc_ms", 0), 1) if j_ok else None,
        "survivors_admission_vote_ms": ms(max(x["sec"] for x in admits)) if admits else None,
        "optimize_topology_call_ms": ms(max(x["sec"] for x in opt)) if opt else None,
        "optimize_ok": bool(opt) and all(x["event"] == "optimized" for x in opt) and len(opt) == a.peers,
        "master_atsp_solve_ms": round(topo["last_solve_us"] / 1e3, 3) if topo["solves"] else None,
        "master_topology": topo,
        "failed_ops_per_survivor": max((sum(1 for x in fails if x["rank"] == r) for r in survivors), default=0),
        "in_place_restore_exact": bool(fails) and all(x["restore_ok"] for x in fails),
        "all_results_exact": bool(oks) and all(x["exact"] for x in oks),
        "paths": sorted({x["path"] for x in oks}),
        "ms_per_op": {"before_kill": med_ms(full_before), f"w{a.peers - 1}": med_ms(small),
                      "after_rejoin": med_ms(rejoined), "after_optimize": med_ms(after_opt)},
        "ops": {"before_kill": len(full_before), f"w{a.peers - 1}": len(small), "after_rejoin": len(rejoined),
                "after_optimize": len(after_opt)},
        "peer_errors": errs,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--pool", type=int, default=2)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--transport", default="tcp", choices=["tcp", "ipc"],
                    help="tcp: the device ring over loopback TCP (PCCL_DISABLE_IPC=1; the reference's data path); "
                         "ipc: the xGMI path for peers on one host")
    ap.add_argument("--kill-op", type=int, default=6, help="sequence number of the op the victim dies in")
    ap.add_argument("--signal", default="kill", choices=["kill", "stop"],
                    help="kill: the victim SIGKILLs itself; stop: it SIGSTOPs itself (sockets stay open)")
    ap.add_argument("--peer-timeout-ms", type=int, default=None,
                    help="PCCL_PEER_TIMEOUT_MS of the master (default: the environment's, else 10 s)")
    ap.add_argument("--post-ops", type=int, default=5, help="ops after the topology re-solve")
    ap.add_argument("--probe-ms", type=int, default=300, help="bandwidth probe per peer pair (PCCL_BENCHMARK_MILLIS)")
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--log-dir", default=None, help="keep every peer's stderr here")
    ap.add_argument("--no-reserve", action="store_true",
                    help="no staging reserve next to connect() (the first op allocates it)")
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--master", default=None)
    ap.add_argument("--joiner", action="store_true")
    ap.add_argument("--deadline", type=float, default=0)
    a = ap.parse_args()
    if a.rank is not None:
        return peer(a)
    if a.log_dir:
        os.makedirs(a.log_dir, exist_ok=True)
    print(json.dumps(run(a)), flush=True)


if __name__ == "__main__":
    main()
