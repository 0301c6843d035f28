"""Flagship benchmark — BASELINE.json config 2: ring all-reduce (SUM) of a 1 GiB bf16 HIP device buffer per peer,
8 peers, over the loopback-TCP device ring.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--peers 8] [--mib 1024] [--quick]

Layout: the job always has ``--peers`` peers (default 8, the config's peer count), spread evenly over the N GPUs:
  N == 1 : all 8 peers are threads of this process on cuda:0 (as literally as one GPU allows).
  N  > 1 : launched by torch.distributed.run, one process per GPU (LOCAL_RANK), 8/N peer threads per process;
           rank 0 also hosts the CCoIP master.
Every process binds to its GPU's NUMA node before it starts peer threads (extra.numa_bind). torch.distributed (gloo) only carries the bench's own barriers,
           the master port and the max-over-ranks of the timings.
The total work (8 x 1 GiB) is fixed as N grows, so ``scaling`` is "strong".

Headline (``value``): the TCP device ring (PCCL_DISABLE_IPC=1 — peers do not short-circuit to xGMI): every ring step
stages HBM -> pinned host (hipMemcpyAsync), sends over loopback TCP and reduces the received bytes into HBM with the
HIP reduce kernel. ``value`` is the per-peer nccl-tests bus bandwidth, busBW = (bytes / t) * 2 (n - 1) / n, of the
first timed window; ``extra.aggregate_bus_bw_GBps`` is its sum over the peers, ``extra.windows_ms`` the ms per op of
``--windows`` timed windows (min / median next to it), ``extra.op_ms_rank0`` the per-op spread, and
``extra.ref_metric_rx_plus_tx_per_peer_GBps`` the reference's own metric ((rx + tx) / t per peer,
reference tests/basic_reduce_test/main.cpp:141-143).

``extra`` also carries, measured in the same run: the xGMI/IPC path at the same peers (the library's default for
same-host peers), 2 peers over IPC (N == 1), a busBW-vs-size sweep for both paths, the 1 GiB busBW at 2 / 4 / 8
peers for both paths (``extra.peer_curve``, N == 1), small-message latencies (2-peer 4-element CPU all-reduce =
BASELINE config 1; 1 MiB over IPC from the C API, from Python with one process per peer, and from Python threads of
one process) and, N == 1, BASELINE configs 5 and 4 in their own processes (``extra.baseline_configs``): kill + rejoin
1 of 8 peer processes mid-all-reduce with the ATSP re-solve, on the TCP device ring and on the xGMI path, and the 1B
fp32 late joiner over TCP and IPC; ``extra.peer_rejoin_latency_ms`` (the metric's second half) is config 5's rejoin on
the TCP device ring. The measurements with one process per peer (configs 5 / 4, the per-process Python latency) run
before this process creates its GPU context (pre_gpu_measurements); ``extra.per_rank`` holds each rank's PCIe
staging bytes, socket bytes, a host DRAM traffic estimate and CPU by thread for the headline window.

vs_baseline is null: the reference publishes only WAN throughputs (25 / 45 Gbit/s), which are not
comparable with a single-host loopback/HBM measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "all-reduce bus BW (GB/s) vs tensor bytes, 2/4/8 peers; peer-rejoin latency"


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--peers", type=int, default=8, help="total peers of the job (config: 8)")
    ap.add_argument("--mib", type=int, default=1024, help="buffer per peer in MiB (config: 1024)")
    ap.add_argument("--pool", type=int, default=0,
                    help="P2P connections per ring neighbour (ring stripes); 0 = per phase, CPUs available / peers in "
                         "this process, in [1, 8]: on the 16-CPU MI355X box 8 peers x 2, 4 peers x 4 and 2 peers x 8 "
                         "stripes measured fastest with the send-ahead ring (profiles/r3/ring_ab/)")
    ap.add_argument("--windows", type=int, default=3,
                    help="timed windows of --steps ops for the headline (the first is the reported one; all of them "
                         "give extra.windows_ms min / median)")
    ap.add_argument("--quick", action="store_true", help="headline only (no IPC / sweep / latency extras)")
    ap.add_argument("--no-ipc-extra", action="store_true", help="skip the xGMI/IPC measurements in extra")
    ap.add_argument("--no-peer-curve", action="store_true", help="skip the 2 / 4 peer points of the 1 GiB curve")
    ap.add_argument("--no-quant-extra", action="store_true", help="skip the uint8-quantized device ring in extra")
    ap.add_argument("--no-config-extra", action="store_true",
                    help="skip BASELINE configs 4 / 5 (late joiner, kill + rejoin) in extra")
    ap.add_argument("--extras-child", default="", help=argparse.SUPPRESS)  # internal: run only the extras, write JSON
    return ap.parse_args()


class Job:
    """This process's share of the job: `local` peer threads on `dev`, `first` = global index of the first one."""

    def __init__(self, a):
        import torch
        self.torch = torch
        self.a = a
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.phase_log = []  # per-rank record of every measured phase (measure -> _phase_ranks)
        self.dist = None
        local_rank = int(os.environ.get("LOCAL_RANK", self.rank))
        same_gpu = os.environ.get("PCCL_BENCH_SAME_GPU") == "1"  # rehearsal of the N>1 path on a 1-GPU box
        if self.world > 1:
            import datetime

            import torch.distributed as dist
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
            self.dist = dist
        ndev = max(1, torch.cuda.device_count())
        # one GPU per rank; with fewer GPUs than ranks the ranks share them round-robin (labelled by distinct devices)
        self.gpu = 0 if same_gpu else local_rank % ndev
        torch.cuda.set_device(self.gpu)
        self.dev = torch.device("cuda", self.gpu)
        self.total = max(a.peers, self.world)
        self.total += (-self.total) % self.world  # equal peers per process
        self.local = self.total // self.world
        self.first = self.rank * self.local
        self.n_gpus = 1 if same_gpu else min(self.world, ndev)
        self.bar = threading.Barrier(self.local)
        self.auto_pool = a.pool <= 0

    def pool_for(self, local_peers: int) -> int:
        """Connections per ring neighbour for a phase with `local_peers` peer threads in each of the job's processes:
        the CPUs this process may use, shared by every peer of the node (torchrun's ranks run in one container, so the
        cgroup quota is node-wide), in [1, 8]. One GPU, 16 CPUs: 8 peers x 2, 4 x 4, 2 x 8 stripes (measured fastest,
        profiles/r3/ring_ab/); with one peer per GPU each peer owns its GPU's PCIe link, and its ring steps are bound
        by the socket copies of its stripes."""
        if not self.auto_pool:
            return self.a.pool
        share = int(_cpu_quota()) // max(1, local_peers * self.world)
        return max(1, min(8, share))

    # -- cross-peer helpers (called from peer threads) --------------------------------------------------------------
    def sync(self, i: int):
        self.bar.wait()
        if self.dist is not None and i == 0:
            self.dist.barrier()
        self.bar.wait()

    def max_over_job(self, vals):
        v = max(vals)
        if self.dist is not None:
            t = self.torch.tensor([v], dtype=self.torch.float64)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            v = float(t.item())
        return v

    def gather(self, obj):
        """[obj of every rank] on every rank (rank order)."""
        if self.dist is None:
            return [obj]
        box = [None] * self.world
        self.dist.all_gather_object(box, obj)
        return box

    def broadcast(self, obj):
        if self.dist is None:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    # -- one phase: fresh master + communicators, `fn(i, comm)` on every local peer thread ------------------------
    def phase(self, fn, *, ipc: bool, peers: int = 0, timeout: float = 900.0):
        import pccl_amd as pccl
        from pccl_amd.utils import free_port, peer_ports, wait_for_world
        total = peers or self.total
        local = total // self.world
        if ipc:
            os.environ.pop("PCCL_DISABLE_IPC", None)
        else:
            os.environ["PCCL_DISABLE_IPC"] = "1"
        master = None
        port = free_port() if self.rank == 0 else 0
        if self.rank == 0:
            master = pccl.MasterNode(f"127.0.0.1:{port}")
            master.run()
        port = self.broadcast(port)
        addr = f"127.0.0.1:{port}"
        self.addr = addr
        ports = peer_ports(local)
        out = [None] * local
        errs = [None] * local
        comms = [None] * local
        bar = threading.Barrier(local)
        self.bar = bar
        # the xGMI path moves no data over the TCP pool: keep it small there (8 connections per neighbour measured
        # 0.88 -> 1.25 ms for 2 peers x 1 GiB over IPC, setup and vote traffic only)
        pool = min(2, self.pool_for(local)) if ipc else self.pool_for(local)
        self.phase_pool = pool

        groups = _peer_cpu_groups(local) if not ipc else None

        def body(i):
            try:
                if groups:  # this peer's library threads (created from here on) inherit the mask
                    os.sched_setaffinity(0, groups[i])
                self.torch.cuda.set_device(self.dev)
                c = pccl.Communicator(addr, 0, p2p_connection_pool_size=pool, **ports[i])
                comms[i] = c
                c.connect(n_attempts=30)
                wait_for_world(c, total, timeout=300)
                out[i] = fn(i, c)
            except BaseException as e:  # noqa: BLE001 - re-raised below
                errs[i] = e
                try:
                    bar.abort()
                except Exception:  # noqa: BLE001
                    pass

        ths = [threading.Thread(target=body, args=(i,), daemon=True) for i in range(local)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=timeout)
        if any(t.is_alive() for t in ths):
            raise TimeoutError("bench phase did not finish")
        for e in errs:
            if e is not None:
                raise e
        for c in comms:
            if c is not None:
                c.destroy()
        if self.dist is not None:
            self.dist.barrier()
        if master is not None:
            master.interrupt()
            master.await_termination()
        return out


def _timed(job, i, comm, x, y, steps, warmup, tag0=0, ops=None, qopt=None):
    """warmup + `steps` timed all-reduces between job-wide barriers; returns (seconds, tx, rx, path, cpu seconds).
    `ops` (optional list) receives the wall time of every timed op as seen by this peer."""
    import pccl_amd as pccl
    torch = job.torch
    for s in range(warmup):
        for attempt in range(3):  # an aborted warmup op (e.g. xGMI vote fell back) is retried by all peers
            try:
                comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag0 + s, quantization_options=qopt)
                break
            except pccl.PCCLError:
                if attempt == 2:
                    raise
    torch.cuda.synchronize()
    job.sync(i)
    tc0 = _task_cpu() if i == 0 and tag0 == 0 else None  # the phase's main window only
    pc0 = pccl.memory.pcie_stats() if i == 0 and tag0 == 0 else None
    t0 = time.perf_counter()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    tx = rx = 0
    for s in range(steps):
        ta = time.perf_counter()
        info = comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag0 + warmup + s, quantization_options=qopt)
        if ops is not None:
            ops.append(time.perf_counter() - ta)
        tx += info.tx_bytes
        rx += info.rx_bytes
    torch.cuda.synchronize()
    job.sync(i)
    dt = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    # CPU seconds of the whole process (every peer thread of this rank) over the timed ops: the loopback-TCP ring is
    # CPU work (kernel socket copies), so cpu_s / dt shows how many cores it kept busy
    cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    sys_s = ru1.ru_stime - ru0.ru_stime  # kernel time: on the TCP rings mostly socket copies
    if tc0 is not None:
        job.cpu_by_thread = _cpu_by_thread(tc0, _task_cpu(), cpu, dt)
        pc1 = pccl.memory.pcie_stats()
        job.pcie = {k: (pc1[k] - pc0[k]) / steps for k in pc1}  # this process's (= GPU's) staging bytes per op
    return dt, tx, rx, comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH), cpu, sys_s


def _task_cpu():
    """{tid: (thread name, user s, sys s)} of this process's live threads (Linux /proc)."""
    out = {}
    tick = os.sysconf("SC_CLK_TCK")
    try:
        tids = os.listdir("/proc/self/task")
    except OSError:
        return out
    for t in tids:
        try:
            with open(f"/proc/self/task/{t}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        f = st[st.rindex(")") + 2:].split()
        out[t] = (name, int(f[11]) / tick, int(f[12]) / tick)
    return out


def _cpu_by_thread(before, after, total_cpu, wall):
    """Cores kept busy per thread name over a window: live threads' deltas grouped by name (pccl threads are named by
    libpccl: pccl-mux-rx = socket receives, pccl-stripe-tx = ring sends, pccl-op = op threads, ...); threads that
    exited inside the window (per-op sender threads) only show in the remainder ``exited_or_unnamed``."""
    agg = {}
    for tid, (name, u, s) in after.items():
        u0, s0 = before.get(tid, (name, 0.0, 0.0))[1:]
        key = name if name.startswith("pccl") else "other"
        a = agg.setdefault(key, [0.0, 0.0])
        a[0] += u - u0
        a[1] += s - s0
    seen = sum(u + s for u, s in agg.values())
    res = {k: {"user_cores": round(u / wall, 2), "sys_cores": round(s / wall, 2)} for k, (u, s) in sorted(agg.items())}
    res["exited_threads_cores"] = round(max(0.0, total_cpu - seen) / wall, 2)
    return res


def _check(job, i, comm, x, y, peers):
    """Exactness: every peer contributes (global index + 1); the bf16 sum of small integers is exact."""
    import pccl_amd as pccl
    x.fill_(float(job.first + i + 1))
    comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=999_999)
    job.torch.cuda.synchronize()
    want = peers * (peers + 1) / 2
    lo, hi = float(y.min()), float(y.max())
    return lo == hi == want


def _log(msg):
    """Progress on stderr (the JSON result line is the only stdout output)."""
    print(f"[bench {time.strftime('%H:%M:%S')} rank {os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def _cpu_quota():
    """CPUs this process may use: the cgroup v2 quota (cpu.max) if set, else the affinity mask."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
        if q != "max":
            return round(min(n, int(q) / int(period)), 2)
    except (OSError, ValueError):
        pass
    return n


def _bw(nbytes, t, n):
    alg = nbytes / t / 1e9
    return alg, alg * 2 * (n - 1) / n


def _curve_point(nbytes, t, n):
    return {"ms": round(t * 1e3, 4), "bus_bw_per_peer_GBps": round(_bw(nbytes, t, n)[1], 3)}


def measure(job, *, ipc, nbytes, steps, warmup, sweep=(), peers=0, check=False, windows=1, quant=False, label=None):
    """Runs one phase; returns {"t": s/op (max over the job), "tx", "rx", "path", "sweep": {bytes: s/op}, "ok",
    "windows": [s/op of each timed window (the first is "t")], "op_ms": per-op wall times of peer 0 in window 1}.
    Every phase also appends its per-rank record to ``job.phase_log`` (``_phase_ranks``)."""
    import pccl_amd as pccl
    torch = job.torch
    total = peers or job.total
    ipc0 = pccl.memory.ipc_buffer_stats()

    def fn(i, comm):
        import contextlib

        import pccl_amd as pccl
        g = torch.Generator(device=job.dev).manual_seed(job.first + i)
        n = nbytes // 2
        # xGMI path: buffers in fd-shareable memory (pccl_amd.memory), the documented way to get zero-copy fault-safe
        # ops between processes; the TCP ring does not care where the buffers live
        with pccl.memory.maybe_shareable(job.dev) if ipc else contextlib.nullcontext():
            x = torch.randn(n, device=job.dev, dtype=torch.bfloat16, generator=g)
            y = torch.empty_like(x)
        ops = []
        qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if quant else None
        r = {"main": _timed(job, i, comm, x, y, steps, warmup, ops=ops, qopt=qopt), "ops": ops, "win": []}
        tag = 5_000
        for _w in range(1, windows):  # further windows of the same ops (the first one is the reported value)
            r["win"].append(_timed(job, i, comm, x, y, steps, 0, tag0=tag)[0])
            tag += steps + 10
        tag = 10_000
        for b in sweep:
            m = b // 2
            reps = max(3, min(50, int(2e9 // max(b, 1) // 8)))
            r[b] = _timed(job, i, comm, x[:m], y[:m], reps, 2, tag0=tag)[0] / reps
            tag += reps + 10
        if check:
            r["ok"] = _check(job, i, comm, x, y, total)
        return r

    _log(f"phase {'xGMI/IPC' if ipc else 'TCP device ring'}: {total} peers x {nbytes >> 20} MiB, {steps} steps")
    res = job.phase(fn, ipc=ipc, peers=peers)
    dt = job.max_over_job([r["main"][0] for r in res])
    _log(f"  done: {dt / steps * 1e3:.3f} ms/op")
    out = {"t": dt / steps, "tx": res[0]["main"][1] / steps, "rx": res[0]["main"][2] / steps,
           "path": res[0]["main"][3], "sweep": {}, "cpu_cores": res[0]["main"][4] / max(dt, 1e-9),
           "op_ms": [round(v * 1e3, 2) for v in res[0]["ops"]], "pool": job.phase_pool}
    out["windows"] = [out["t"]] + [job.max_over_job([r["win"][w] for r in res]) / steps for w in range(windows - 1)]
    # per rank (= per GPU): socket bytes of its peers, PCIe staging bytes and CPU by thread over the main window
    local_tx = sum(r["main"][1] for r in res) / steps
    local_rx = sum(r["main"][2] for r in res) / steps
    out["per_rank"] = job.gather({"rank": job.rank, "gpu": job.gpu, "peers": len(res), "tx": local_tx, "rx": local_rx,
                                  "pcie": getattr(job, "pcie", None), "cpu_cores": res[0]["main"][4] / max(dt, 1e-9),
                                  "cpu_by_thread": getattr(job, "cpu_by_thread", None)})
    for b in sweep:
        out["sweep"][b] = job.max_over_job([r[b] for r in res])
    job.phase_log.append(_phase_ranks(job, label or ("ipc" if ipc else "device_ring"), res, dt / steps, ipc0))
    if check:
        ok = all(r["ok"] for r in res)
        if job.dist is not None:
            t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64)
            job.dist.all_reduce(t, op=job.dist.ReduceOp.MAX)
            ok = t.item() == 0.0
        out["ok"] = ok
    return out


def _phase_ranks(job, label, res, t, ipc0):
    """One phase, per rank (= per GPU at N > 1): the reduce path its peers' ops took, the cross-GPU pre-flight probes
    that ran in it (passed / failed: the xGMI path's first op of an arena spanning GPUs writes a probe into every
    peer's buffer; a failure moves the ring to TCP), and the kernel CPU time per socket throughput - what the TCP
    ring's host-bound scaling model (docs/PERFORMANCE.md) depends on, measured on every rank."""
    import pccl_amd as pccl
    ipc1 = pccl.memory.ipc_buffer_stats()
    main = res[0]["main"]
    tx = sum(r["main"][1] for r in res)  # this rank's peers, over the main window
    rx = sum(r["main"][2] for r in res)
    wall = max(main[0], 1e-9)
    sys_cores = main[5] / wall
    paths = sorted({pccl.ReducePath(r["main"][3]).name for r in res})
    # (the op counters count an xGMI op's bytes too: socket rates only where a TCP ring ran)
    tcp = any(p in ("HOST_RING", "DEVICE_RING", "HIERARCHICAL") for p in paths)
    tx_gbps = tx / wall / 1e9 if tcp else 0.0
    rec = {"rank": job.rank, "gpu": job.gpu, "peers": len(res), "paths": paths,
           "preflight_passed": ipc1.get("preflight_passed", 0) - ipc0.get("preflight_passed", 0),
           "preflight_failed": ipc1.get("preflight_failed", 0) - ipc0.get("preflight_failed", 0),
           "socket_tx_GBps": round(tx_gbps, 3) if tcp else None,
           "socket_rx_GBps": round(rx / wall / 1e9, 3) if tcp else None,
           "sys_cores": round(sys_cores, 2),
           "sys_cores_per_socket_GBps": round(sys_cores / tx_gbps, 3) if tx_gbps > 0.01 else None}
    return {"phase": label, "ms_per_op": round(t * 1e3, 3), "per_rank": job.gather(rec)}


def _per_rank_diag(ring, nbytes, P):
    """Per rank (one GPU each at N > 1) over the headline window, per op: the PCIe staging bytes the library queued
    (``pcie_*_GB``, pcclxPcieStats) next to the ring's model (per peer D2H = S, H2D = 1.75 S at 8 peers: the step-0
    payload and every reduced piece leave the GPU once, every received piece enters it once, 2(W-1)/W S each way on
    the wire), the peers' loopback-TCP bytes and an estimate of the host DRAM traffic they cause: every socket byte is
    read and written once by the receiver's copy (same-host data sockets send MSG_ZEROCOPY: the kernel reads the
    sender's pinned pages in place; 2 x tx), and every PCIe byte is one DMA access of pinned memory. What the N >= 4 host-memory-bound prediction
    (docs/PERFORMANCE.md) hinges on, measured rather than assumed."""
    rows = []
    t = ring["t"]
    for r in ring.get("per_rank") or []:
        peers = r["peers"]
        wire = 2 * (P - 1) / P * nbytes
        row = {"rank": r["rank"], "gpu": r["gpu"], "peers": peers,
               "socket_tx_GB": round(r["tx"] / 1e9, 3), "socket_rx_GB": round(r["rx"] / 1e9, 3),
               "model_pcie_d2h_GB": round(peers * nbytes / 1e9, 3) if P > 1 else 0.0,
               "model_pcie_h2d_GB": round(peers * wire / 1e9, 3),
               "cpu_cores_busy": round(r["cpu_cores"], 2), "cpu_by_thread": r["cpu_by_thread"]}
        if r.get("pcie"):
            h2d, d2h = r["pcie"]["h2d"], r["pcie"]["d2h"]
            dram = 2 * r["tx"] + h2d + d2h
            row.update({"pcie_h2d_GB": round(h2d / 1e9, 3), "pcie_d2h_GB": round(d2h / 1e9, 3),
                        "pcie_GBps": round((h2d + d2h) / t / 1e9, 2),
                        "host_dram_est_GB": round(dram / 1e9, 2), "host_dram_est_GBps": round(dram / t / 1e9, 1)})
        rows.append(row)
    return rows


def latency_cpu(job, n_ops=300):
    """BASELINE config 1: 2 peers, 4 fp32 elements, host memory; median / p99 microseconds per all-reduce."""
    import numpy as np

    import pccl_amd as pccl

    def fn(i, comm):
        x = np.arange(4, dtype=np.float32) + i
        y = np.empty_like(x)
        ts = []
        for s in range(n_ops):
            job.bar.wait()
            t0 = time.perf_counter()
            comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=s)
            ts.append(time.perf_counter() - t0)
        return ts

    res = job.phase(fn, ipc=False, peers=2)
    ts = sorted(max(r[k] for r in res) for k in range(n_ops))[10:]
    return {"median_us": round(statistics.median(ts) * 1e6, 1), "p99_us": round(ts[int(0.99 * (len(ts) - 1))] * 1e6, 1)}


class _full_cpu_mask:
    """Runs a block with the calling thread's CPU mask from before the bench's per-CCD spread (_cpu_spread), if any;
    threads and processes started inside inherit it. For the latency measurements: the spread suits the
    socket-copy-bound TCP ring, but it scatters a phase's threads over 16 L3 domains of both sockets, where every
    wake-up of a waiting peer lands on a sleeping core of another CCD. ccd=True narrows the mask further to the L3
    domain (CCD) of its first CPU: BASELINE config 1 (2 threaded peers, 4 elements) measured 32-37 us median there in
    3 / 3 runs vs 41-94 us (bimodal) with the full mask on the same box (profiles/r3/latency_futex/cfg1_masks.jsonl)."""

    def __init__(self, ccd: bool = False):
        self.ccd = ccd

    def __enter__(self):
        full = os.environ.get("PCCL_BENCH_FULL_CPUS")
        self.own = os.sched_getaffinity(0)
        mask = {int(c) for c in full.split(",")} if full else set(self.own)
        if self.ccd:
            try:
                with open(f"/sys/devices/system/cpu/cpu{min(mask)}/cache/index3/shared_cpu_list") as f:
                    ccd = set()
                    for part in f.read().strip().split(","):
                        lo, _, hi = part.partition("-")
                        ccd.update(range(int(lo), int(hi or lo) + 1))
                if len(ccd & mask) >= 4:
                    mask &= ccd
            except (OSError, ValueError):
                pass
        if mask != self.own:
            os.sched_setaffinity(0, mask)
        return self

    def __exit__(self, *exc):
        os.sched_setaffinity(0, self.own)
        return False


class _cpu_mask:
    """Runs a block with the given CPU mask; threads and processes started inside inherit it."""

    def __init__(self, mask):
        self.mask = set(mask)

    def __enter__(self):
        self.own = os.sched_getaffinity(0)
        if self.mask != self.own:
            os.sched_setaffinity(0, self.mask)
        return self

    def __exit__(self, *exc):
        os.sched_setaffinity(0, self.own)
        return False


def _gpu_numa_node_child(local_rank: int = 0) -> int:
    """_gpu_numa_node(local_rank) read by a child process, so this process's GPU runtime stays uninitialised (its
    threads would keep the CPU mask from before a later sched_setaffinity); -1 if unknown."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, "-c", f"import bench; print(bench._gpu_numa_node({int(local_rank)}))"],
                           cwd=ROOT, capture_output=True, text=True, timeout=180)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else -1
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
        return -1


# baseline_configs runs that take _config_tcp_mask's mask. Interleaved over two passes (profiles/r5/b23/): config 5 over
# TCP 372 / 367 ms per op on the node vs 383 / 414 with the full mask (kill -> survivors' failed op 193 / 187 vs
# 220 / 219 ms), config 3 uint8 1.09 / 1.11 vs 1.21 / 1.17 s; the collocated run (its relay moves 10 Gbit/s flows)
# is faster with the full mask: 62.3 / 66.1 vs 60.3 / 57.3 Gbit/s.
_NODE_MASKED = ("config5_kill_rejoin_tcp", "config5_stop_rejoin_tcp", "config3_wan_50ms")


def _config_tcp_mask():
    """CPU mask for the one-process-per-peer runs over loopback TCP named in _NODE_MASKED. PCCL_BENCH_CONFIG_MASK:
    full (the mask from before the per-CCD spread), spread (the bench's per-CCD spread), numa (default: the spread
    restricted to the GPU's NUMA node, as the headline runs). None = the full mask."""
    mode = os.environ.get("PCCL_BENCH_CONFIG_MASK", "numa")
    if mode == "full" or not os.environ.get("PCCL_BENCH_FULL_CPUS"):
        return None  # (no spread applied: the harnesses keep this process's mask)
    own = os.sched_getaffinity(0)
    if mode == "spread":
        return own
    node = _gpu_numa_node_child()
    if node < 0:
        return own
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _parse_cpulist(f.read()) & own
    except (OSError, ValueError):
        return own
    return cpus if len(cpus) >= 8 else own


def latency_native(peers):
    """Small-op latency of the xGMI/IPC path without Python in the loop: pccl_amd/lib/pccl_latency (the C API with
    hipMalloc'd buffers, threaded peers on cuda:0, csrc/tools/latency_native.hip), 1 MiB bf16 at `peers` and 2 peers;
    median / p90 of the per-op max over the peers. The Python sweep point (extra.latency_1MiB_ipc_us) adds the
    interpreter: 8 peer threads serialise on the GIL around every op."""
    import subprocess

    from pccl_amd.utils import free_port
    exe = os.path.join(ROOT, "pccl_amd", "lib", "pccl_latency")
    if not os.path.exists(exe):
        return {"error": "pccl_latency not built"}
    # the harness runs with the process's CPU mask from before the bench's per-CCD spread (_cpu_spread): the spread
    # suits the socket-copy-bound TCP ring, but it scatters the peers' op threads over 16 L3 domains and both sockets,
    # where every shared-memory barrier word bounces between CCDs - 8 peers x 1 MiB measured 445 us median with the
    # 3-per-CCD mask vs 153-167 us with the full mask on the same box (profiles/r3/latency_futex/affinity.jsonl)
    out = {"cpu_mask": "full" if os.environ.get("PCCL_BENCH_FULL_CPUS") else "inherited"}
    for p in sorted({peers, 2}):
        try:
            env = dict(os.environ)
            env.pop("PCCL_DISABLE_IPC", None)  # set by the TCP-ring phases of this process; this is the xGMI path
            with _full_cpu_mask():  # the child inherits this thread's mask
                r = subprocess.run([exe, str(free_port()), str(p), str(1 << 20), "400", "50"], capture_output=True,
                                   text=True, timeout=120, env=env)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            out[f"{p}_peers_1MiB"] = json.loads(line[-1]) if r.returncode == 0 and line else \
                {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
        except subprocess.TimeoutExpired:
            out[f"{p}_peers_1MiB"] = {"error": "timeout"}
    return out


def latency_python_processes(peers):
    """The Python API's small-op latency in the deployment shape: one process per peer (benchmarks/py_latency.py),
    `peers` processes on cuda:0 over the xGMI/IPC path, 1 MiB bf16; the blocking call and the async call awaited at
    once. Unlike extra.latency_1MiB_ipc_python_threads_us no GIL is shared between the peers."""
    import subprocess
    env = dict(os.environ)
    env.pop("PCCL_DISABLE_IPC", None)
    # 8 peer processes next to this one on the same GPU: 2 hardware queues each (README: several processes on one
    # GPU). The blocking latency of this layout is bimodal on the shared boxes either way (docs/ROUND4_RESPONSE.md)
    env.setdefault("GPU_MAX_HW_QUEUES", "2")
    try:
        with _full_cpu_mask():
            r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "py_latency.py"), "--peers",
                                str(peers), "--iters", "200", "--sizes", str(1 << 20)], capture_output=True, text=True,
                               timeout=180, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not line:
        return {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
    row = json.loads(line[-1])["sizes"]["1024KiB"]
    # every call variant of the run (interleaved op by op on the same buffers), median / p90 us
    variants = {k: {"median_us": v["median_us"], "p90_us": v["p90_us"]} for k, v in row.items()
                if isinstance(v, dict) and "median_us" in v}
    return {"peers": peers, "path": row["path"], "blocking_median_us": row["all_reduce"]["median_us"],
            "blocking_p90_us": row["all_reduce"]["p90_us"],
            "async_median_us": row["async"]["median_us"] if "async" in row else None,
            "ready_median_us": row["ready"]["median_us"] if "ready" in row else None,
            "variants": variants}


def baseline_configs(a, peers):
    """BASELINE configs 5 and 4 as the reference defines them, each in its own processes (one per peer) and under its
    own time limit, so a failure is reported here instead of losing the headline:
      * config 5 (benchmarks/fault_tolerance.py): `peers` peer processes on cuda:0, in-place SUM of `--mib` MiB bf16;
        the last peer SIGKILLs itself mid-op (PCCL_FAULT_INJECT; TCP device ring: reduce-scatter step 1 with its first
        received piece in flight; xGMI path: right after launching its push kernel); the survivors abort, re-form the
        ring and continue; a replacement process joins; every peer re-solves the ring (bandwidth probes + ATSP). On the
        TCP device ring (PCCL_DISABLE_IPC=1, the reference's data path) and on the xGMI path.
      * config 4 (benchmarks/shared_state_sync.py): a 1B-parameter fp32 shared state (8 tensors, 4 GB in HBM); a late
        joiner at revision 0 catches up from a trainer at revision 3, over loopback TCP (pinned staging) and over the
        same-host IPC hand-off; content and simplehash digests compared with the trainer's.
      * config 5 with SIGSTOP instead of SIGKILL (--signal stop): the victim stops without closing a socket, so only
        the liveness protocol (heartbeats, PCCL_PEER_TIMEOUT_MS = 2 s here) detects it; the stopped victim is then
        SIGKILLed and a replacement joins as above (config5_stop_rejoin_tcp).
      * config 3 (benchmarks/wan_quantized.py, EMULATED WAN: pccl_wan_relay, a separate process delaying and pacing
        every byte; tc-netem needs root; each format cold + warm, the warm repeat reported): `peers` peer processes on cuda:0, 2 GiB fp32 AVG per peer, 50 ms one way,
        1 Gbit/s flows, 25 Gbit/s links, 16 connections per neighbour; fp32 (8 ops in flight) and uint8 / int8
        zero-point-scale / fp8 (32 ops in flight, 512 KiB stripes: groups of 4 connections shared by 8 ops measured
        fastest, profiles/r5/b12/); seconds and the reference's metric (rx + tx Gbit/s per peer, its
        published 25 / 45 Gbit/s). Plus the collocated-sites emulation: 5 ms one way, 10 Gbit/s flows, 50 Gbit/s
        links, fp32, 4 peers (8 peers plus the relay exceed the box's CPU share)."""
    import subprocess
    runs = [("config5_kill_rejoin_tcp", ["fault_tolerance.py", "--transport", "tcp", "--peers", str(peers), "--mib",
                                         str(a.mib)], 240),
            # the same with a peer that stops without closing a socket (SIGSTOP): only the liveness protocol detects it
            ("config5_stop_rejoin_tcp", ["fault_tolerance.py", "--transport", "tcp", "--peers", str(peers), "--mib",
                                         str(a.mib), "--signal", "stop", "--peer-timeout-ms", "2000"], 240),
            ("config5_kill_rejoin_ipc", ["fault_tolerance.py", "--transport", "ipc", "--peers", str(peers), "--mib",
                                         str(a.mib)], 180),
            ("config4_late_joiner_tcp", ["shared_state_sync.py", "--transport", "tcp", "--params", "1e9"], 180),
            ("config4_late_joiner_ipc", ["shared_state_sync.py", "--transport", "ipc", "--params", "1e9"], 120),
            ("config3_wan_50ms", ["wan_quantized.py", "--peers", str(peers), "--mib", "2048", "--latency-ms", "50",
                                  "--flow-mbit", "1000", "--link-mbit", "25000", "--pool", "16", "--concurrent", "8",
                                  "--concurrent-quant", "32", "--stripe-min-kib", "512", "--repeat", "2",
                                  "--formats", "fp32,uint8,int8_zps,fp8"], 180),
            ("collocated_5ms_4peers", ["wan_quantized.py", "--peers", "4", "--mib", "2048", "--latency-ms", "5",
                                       "--flow-mbit", "10000", "--link-mbit", "50000", "--pool", "16",
                                       "--concurrent", "8", "--repeat", "2", "--formats", "fp32"], 120)]
    only = os.environ.get("PCCL_BENCH_CONFIGS")
    if only:
        runs = [r for r in runs if r[0] in only.split(",")]
    out = {}
    env = dict(os.environ)
    env.pop("PCCL_DISABLE_IPC", None)  # set by this process's TCP-ring phases; the harnesses choose per run
    tcp_mask = _config_tcp_mask()
    for name, args, limit in runs:
        _log(f"{name}: {' '.join(args)}")
        t0 = time.time()
        try:
            # the process's CPU mask from before the bench's per-CCD spread (as for the latency measurements): one
            # process per peer, whose spinning op threads and shared-memory barriers suffer when spread over CCDs;
            # config 5 over TCP and config 3 run on the GPU's NUMA node instead (_config_tcp_mask)
            with (_cpu_mask(tcp_mask) if tcp_mask and name in _NODE_MASKED else _full_cpu_mask()):
                r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", args[0]), *args[1:],
                                    *(["--timeout", str(limit - 40)] if args[0] == "fault_tolerance.py" else [])],
                                   capture_output=True, text=True, timeout=limit, env=env)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            out[name] = json.loads(line[-1]) if r.returncode == 0 and line else \
                {"error": f"rc {r.returncode}: {r.stderr[-400:]}"}
        except subprocess.TimeoutExpired:
            out[name] = {"error": f"timeout after {limit} s"}
        out[name]["wall_s"] = round(time.time() - t0, 1)
        _log(f"  done in {out[name]['wall_s']} s")
    return out


def pre_gpu_measurements(a):
    """N == 1, before this process touches the GPU: the per-process Python latency (8 peer processes over the xGMI
    path) and BASELINE configs 5 and 4 (one process per peer), each failure-isolated in its own children."""
    out = {}
    if not a.no_ipc_extra:
        _log("latency_1MiB_ipc_python_processes: py_latency.py")
        out["latency_1MiB_ipc_python_processes"] = latency_python_processes(a.peers)
    if not a.no_config_extra:
        out["baseline_configs"] = baseline_configs(a, a.peers)
    return out


def rejoin_latency(job):
    """A new peer connects mid-run; seconds from its connect() until its first all-reduce completed (admission vote +
    P2P establishment + IPC rendezvous + first op). N == 1 only."""
    import pccl_amd as pccl
    torch = job.torch
    out = {}

    def fn(i, comm):
        small = torch.ones(1 << 16, device=job.dev, dtype=torch.bfloat16)
        y = torch.empty_like(small)
        comm.all_reduce(small, y, op=pccl.ReduceOp.SUM, tag=1)
        joiner = None
        if i == 0:
            def join():
                c = pccl.Communicator(job.addr, 0, p2p_connection_pool_size=job.phase_pool)
                t0 = time.perf_counter()
                c.connect(n_attempts=30)
                yy = torch.empty_like(small)
                c.all_reduce(small, yy, op=pccl.ReduceOp.SUM, tag=77)
                torch.cuda.synchronize()
                out["s"] = time.perf_counter() - t0
                out["c"] = c
            joiner = threading.Thread(target=join, daemon=True)
            joiner.start()
        deadline = time.time() + 120
        while time.time() < deadline:
            if comm.are_peers_pending():
                comm.update_topology()
                comm.all_reduce(small, y, op=pccl.ReduceOp.SUM, tag=77)
                break
            time.sleep(0.001)
        if joiner is not None:
            joiner.join(timeout=120)
            if "c" in out:
                out["c"].destroy()

    job.phase(fn, ipc=True, peers=2)
    return out.get("s")


def run_extras(job, a, nbytes):
    """The measurements that go into ``extra`` besides the headline: the xGMI/IPC path at the same peers, its size
    sweep, 2 peers over IPC (N == 1), small-message latencies and the peer-rejoin latency."""
    import pccl_amd as pccl
    P = job.total
    extra, sweep, curve = {}, {}, {}
    if not a.no_ipc_extra:
        ipc = measure(job, ipc=True, nbytes=nbytes, steps=a.steps, warmup=a.warmup, check=True,
                      sweep=(1 << 20, 16 << 20, 256 << 20), label="ipc_same_peers")
        ialg, ibus = _bw(nbytes, ipc["t"], P)
        extra["ipc_same_peers"] = {"ms_per_op": round(ipc["t"] * 1e3, 4), "bus_bw_per_peer_GBps": round(ibus, 3),
                                   "aggregate_bus_bw_GBps": round(ibus * P, 3),
                                   "reduce_path": pccl.ReducePath(ipc["path"]).name, "result_exact": ipc.get("ok")}
        sweep["DEVICE_IPC"] = {str(b >> 20) + "MiB": {"ms": round(t * 1e3, 4),
                                                      "bus_bw_per_peer_GBps": round(_bw(b, t, P)[1], 3)}
                               for b, t in ipc["sweep"].items()}
        sweep["DEVICE_IPC"][f"{a.mib}MiB"] = {"ms": round(ipc["t"] * 1e3, 4), "bus_bw_per_peer_GBps": round(ibus, 3)}
        # through this harness: 8 peer threads of one Python interpreter, serialised on the GIL around every op
        extra["latency_1MiB_ipc_python_threads_us"] = round(ipc["sweep"][1 << 20] * 1e6, 1)
        # how this rank's IPC ops handed buffers over, incl. the cross-GPU pre-flight result (pccl_amd.memory)
        extra["ipc_buffer_stats_rank0"] = pccl.memory.ipc_buffer_stats()
        if job.world == 1:
            two = measure(job, ipc=True, nbytes=nbytes, steps=a.steps, warmup=a.warmup, peers=2, label="ipc_2_peers")
            talg, tbus = _bw(nbytes, two["t"], 2)
            extra["ipc_2_peers_1gpu"] = {"ms_per_op": round(two["t"] * 1e3, 4), "bus_bw_per_peer_GBps": round(tbus, 3),
                                         "reduce_path": pccl.ReducePath(two["path"]).name}
            curve.setdefault("DEVICE_IPC", {})["2"] = _curve_point(nbytes, two["t"], 2)
            curve["DEVICE_IPC"][str(P)] = _curve_point(nbytes, ipc["t"], P)
    if not a.no_quant_extra:
        # the quantized wire format on the same device ring (uint8 min-max: bf16 -> u8 on the GPU, 2x fewer bytes on
        # the wire; BASELINE config 3's format without the WAN)
        qr = measure(job, ipc=False, nbytes=nbytes, steps=max(3, a.steps // 2), warmup=2, quant=True,
                     label="ring_quant_u8")
        extra["ring_quant_u8_same_peers"] = {"ms_per_op": round(qr["t"] * 1e3, 3),
                                             "bus_bw_per_peer_GBps": round(_bw(nbytes, qr["t"], P)[1], 3),
                                             "wire_tx_bytes_per_op_rank0": qr["tx"],
                                             "reduce_path": pccl.ReducePath(qr["path"]).name}
    if job.world == 1 and not a.no_peer_curve:
        # the metric's "2/4/8 peers": the same 1 GiB all-reduce at fewer peers (8 is the headline / ipc_same_peers)
        for p in (2, 4):
            if p >= P:
                continue
            r = measure(job, ipc=False, nbytes=nbytes, steps=a.steps, warmup=a.warmup, peers=p, label=f"device_ring_{p}")
            curve.setdefault("DEVICE_RING", {})[str(p)] = _curve_point(nbytes, r["t"], p)
            if not a.no_ipc_extra and p != 2:
                r = measure(job, ipc=True, nbytes=nbytes, steps=a.steps, warmup=a.warmup, peers=p, label=f"ipc_{p}")
                curve.setdefault("DEVICE_IPC", {})[str(p)] = _curve_point(nbytes, r["t"], p)
    if curve:
        extra["peer_curve"] = curve
    if job.world == 1:
        extra["latency_native"] = latency_native(P)
        nat = extra["latency_native"].get(f"{P}_peers_1MiB", {})
        if "median_us" in nat:  # the library's latency: C API, threaded peers, no interpreter in the loop
            extra["latency_1MiB_ipc_us"] = nat["median_us"]
        with _full_cpu_mask(ccd=True):
            extra["latency_cpu_4elem_2peers"] = latency_cpu(job)
        if a.no_config_extra:  # (else: BASELINE config 5 in main(), outside this child's time limit)
            with _full_cpu_mask():
                r = rejoin_latency(job)
            extra["peer_rejoin_latency_ms"] = round(r * 1e3, 1) if r else None
            extra["peer_rejoin_latency_source"] = "2 threaded peers, xGMI path, connect -> first op (no kill)"
    else:
        extra["multi_gpu_table"] = multi_gpu_table(job, a, nbytes)
    extra["per_rank_phases"] = job.phase_log
    return extra, sweep


SIZES_MIB = (1, 16, 256, 1024)


def _size_row(job, P, ts):
    return {f"{m}MiB": {"ms": round(t * 1e3, 4), "bus_bw_per_peer_GBps": round(_bw(m << 20, t, P)[1], 3)}
            for m, t in ts.items()}


def multi_gpu_table(job, a, nbytes):
    """N > 1: the same sizes (1 / 16 / 256 / 1024 MiB) through RCCL (one rank per GPU, the vendor yardstick) and
    through the xGMI path in each of its variants: one-shot push (default), two-shot (PCCL_IPC_ALGO=two_shot) and push
    with a larger remote-aware workgroup budget (PCCL_IPC_REMOTE_GRID=1024), so the first cross-GPU run decides the
    algorithm and the budget from data. Every variant is failure-isolated (an error is reported in its entry)."""
    import pccl_amd as pccl
    P = job.total
    table = {"sizes_MiB": list(SIZES_MIB), "peers": P, "gpus": job.n_gpus}
    if job.n_gpus > 1 and os.environ.get("PCCL_BENCH_RCCL", "1") == "1":
        table["rccl"] = rccl_reference(job, a, nbytes)
    else:
        table["rccl"] = {"skipped": "peers share one GPU (RCCL needs one rank per GPU)"}
    variants = [("ipc_push", {}), ("ipc_two_shot", {"PCCL_IPC_ALGO": "two_shot"}),
                ("ipc_push_remote_grid_1024", {"PCCL_IPC_REMOTE_GRID": "1024"})]
    for name, env in variants:
        saved = {k: os.environ.get(k) for k in env}
        try:
            os.environ.update(env)  # read per op by the library; every rank switches at the same phase boundary
            r = measure(job, ipc=True, nbytes=nbytes, steps=a.steps, warmup=a.warmup, check=True,
                        sweep=tuple(m << 20 for m in SIZES_MIB if (m << 20) < nbytes), label=name)
            ts = {m: r["sweep"][m << 20] for m in SIZES_MIB if (m << 20) < nbytes}
            ts[nbytes >> 20] = r["t"]
            table[name] = {"sizes": _size_row(job, P, ts), "result_exact": r.get("ok"),
                           "reduce_path": pccl.ReducePath(r["path"]).name}
        except Exception as e:  # noqa: BLE001 - one variant's failure must not hide the others
            table[name] = {"error": repr(e)[:300]}
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    return table


def rccl_reference(job, a, nbytes):
    """RCCL (torch.distributed "nccl" backend) all-reduce of bf16 buffers of SIZES_MIB, one rank per GPU: the MI355X
    vendor collective as a yardstick for the xGMI path (RCCL has no elastic membership, so it is not an alternative for
    PCCL's use case). N > 1 distinct GPUs only."""
    torch = job.torch
    dist = job.dist
    try:
        g = dist.new_group(backend="nccl")
        x = torch.randn(nbytes // 2, device=job.dev, dtype=torch.bfloat16)
        n = job.world
        out = {"ranks": n}
        for m in SIZES_MIB:
            v = x[:min(x.numel(), (m << 20) // 2)]
            reps = max(a.steps, min(200, int(4e9 // max(v.numel() * 2, 1))))
            for _ in range(max(2, a.warmup)):
                dist.all_reduce(v, group=g)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                dist.all_reduce(v, group=g)
            torch.cuda.synchronize()
            dt = job.max_over_job([time.perf_counter() - t0]) / reps
            out[f"{m}MiB"] = {"ms": round(dt * 1e3, 4), "bus_bw_per_rank_GBps": round(_bw(v.numel() * 2, dt, n)[1], 3)}
        dist.destroy_process_group(g)
        return out
    except Exception as e:  # noqa: BLE001 - a yardstick: report, never fail the bench
        return {"error": repr(e)[:300]}


def extras_in_child(job, a):
    """Runs run_extras() in a child process per rank (its own gloo group on MASTER_PORT + 11): a failure there (e.g.
    a GPU fault on an xGMI path never exercised on this node) is reported in ``extra`` instead of losing the
    headline. Returns (extra, sweep) on rank 0, ({}, {}) elsewhere."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"pccl_bench_extras_{os.getpid()}_{job.rank}.json")
    args = [sys.executable, os.path.abspath(__file__), "--gpus", str(a.gpus), "--steps", str(a.steps), "--warmup",
            str(a.warmup), "--peers", str(a.peers), "--mib", str(a.mib), "--pool", str(0 if job.auto_pool else a.pool),
            "--extras-child", out]
    if a.no_ipc_extra:
        args.append("--no-ipc-extra")
    if a.no_peer_curve:
        args.append("--no-peer-curve")
    if a.no_quant_extra:
        args.append("--no-quant-extra")
    if a.no_config_extra:
        args.append("--no-config-extra")
    env = dict(os.environ)
    if job.world > 1:
        env["MASTER_PORT"] = str(int(os.environ.get("MASTER_PORT", "29500")) + 11)
        # under torchrun the process group joins the elastic agent's store as a client; the child's group needs its
        # own store (hosted by rank 0's child on the new port)
        env["TORCHELASTIC_USE_AGENT_STORE"] = "False"
    try:
        rc = subprocess.run(args, env=env, timeout=float(os.environ.get("PCCL_BENCH_EXTRAS_TIMEOUT", "300"))).returncode
    except subprocess.TimeoutExpired:
        rc = "timeout"
    res = {}
    if job.rank == 0:
        try:
            with open(out) as f:
                res = json.load(f)
            os.unlink(out)
        except (OSError, ValueError):
            res = {}
        if rc != 0:
            res.setdefault("extra", {})["extras_error"] = f"extras child exited with {rc}"
    return res.get("extra", {}), res.get("sweep", {})


def _gpu_numa_node(local_rank: int) -> int:
    """NUMA node of the GPU this rank drives (cuda:LOCAL_RANK), from its PCI address (torch device properties) and
    sysfs; -1 if unknown. Initialises the GPU runtime of this process."""
    import torch
    props = torch.cuda.get_device_properties(local_rank % max(1, torch.cuda.device_count()))
    addr = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    with open(f"/sys/bus/pci/devices/{addr}/numa_node") as f:
        return int(f.read().strip())


def _numa_bind():
    """PCCL_BENCH_NUMA_BIND (default 1; 0 = off): restricts the process to the CPUs of its GPU's NUMA node before it
    starts any thread of its own, so the pinned staging memory the library allocates (first touch by these threads)
    and the socket copies stay on the socket the GPU's PCIe link is attached to. The GPU is identified by its PCI
    address, not by the order of /sys/class/drm. N == 1, on top of the per-CCD spread: 330.3 / 328.3 vs 332.9 /
    331.1 ms per op, interleaved (profiles/r5/b18/). Returns a description for extra, or None."""
    if os.environ.get("PCCL_BENCH_NUMA_BIND", "1") != "1":
        return None
    try:
        # looked up in a child: this process must not initialise the GPU runtime (and start its threads) before the
        # binding, or those threads keep the old mask (sched_setaffinity changes the calling thread only)
        node = _gpu_numa_node_child(int(os.environ.get("LOCAL_RANK", "0")))
        if node < 0:
            return {"numa_bind": "no node"}
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _parse_cpulist(f.read())
        cpus &= os.sched_getaffinity(0)
        if not cpus:
            return {"numa_bind": "node outside the CPU mask", "numa_node": node}
        os.sched_setaffinity(0, cpus)
        return {"numa_node": node, "cpus": len(cpus)}
    except (OSError, ValueError, RuntimeError, AttributeError) as e:
        return {"numa_bind_error": repr(e)[:200]}


def _parse_cpulist(spec: str) -> set:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}"""
    cpus = set()
    for part in spec.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def _peer_cpu_groups(local: int):
    """PCCL_BENCH_PEER_CCD=1 (TCP-ring phases, several peers in this process): peer thread i gets its own share of the
    L3 domains (CCDs) of the process's CPU mask, so the threads the library starts for that peer (op thread, receive
    and sender threads) stay on a few CCDs instead of migrating over all of them. Returns one CPU set per peer, or
    None when off or when there are fewer L3 domains than peers."""
    if local < 2 or os.environ.get("PCCL_BENCH_PEER_CCD", "0") != "1":
        return None
    domains = {}
    for c in sorted(os.sched_getaffinity(0)):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                domains.setdefault(f.read().strip(), []).append(c)
        except OSError:
            return None
    doms = [d for _, d in sorted(domains.items(), key=lambda kv: kv[1][0])]
    if len(doms) < local:
        return None
    return [set(c for d in doms[i * len(doms) // local:(i + 1) * len(doms) // local] for c in d) for i in range(local)]


def _cpu_spread():
    """PCCL_BENCH_CPU_SPREAD=k (default 4 on one GPU, 0 = off; off by default with several ranks): restrict the
    process to the first k CPUs of every L3 domain (CCD) in its affinity mask, before any thread exists. The
    loopback-TCP ring moves ~15 GB through socket copies per op on a 16-CPU quota; with all 256 CPUs of the host in the
    mask its ~40 threads migrate over every CCD and both sockets and burst past the quota (the cgroup then throttles
    the whole process, GPU feeding included), while k cores per CCD keep the memory bandwidth of every CCD at hand.
    Measured, 8 peers x 1 GiB, 3 runs each (profiles/r3/cpu_spread/): all 256 CPUs 374 / 355 / 389 ms, 2 per CCD
    337 / 349 / 342, 3 per CCD 330 / 344 / 328, 4 per CCD 329 / 331 / 359. Round 5, with the NUMA binding on top
    (the GPU's node keeps k x 8 CPUs), interleaved over two passes (profiles/r5/b19/): 2 per CCD 362 / 425, 3 per CCD
    324.6 / 327.0, 4 per CCD 322.7 / 324.4, 8 per CCD 322.2 / 326.0 ms. Returns a description for extra."""
    default = "4" if int(os.environ.get("WORLD_SIZE", "1")) == 1 else "0"
    k = int(os.environ.get("PCCL_BENCH_CPU_SPREAD", default))
    if k <= 0:
        return None
    try:
        allowed = os.sched_getaffinity(0)
        domains = {}
        for c in sorted(allowed):
            try:
                with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                    key = f.read().strip()
            except OSError:
                key = "?"
            domains.setdefault(key, []).append(c)
        pick = set()
        for cpus in domains.values():
            pick.update(cpus[:k])
        if len(pick) < min(16, len(allowed)):  # unknown topology: leave the mask alone
            return {"cpu_spread": "skipped", "l3_domains": len(domains)}
        # the mask before the spread, for measurements that are not the loopback-TCP ring (latency_native)
        os.environ.setdefault("PCCL_BENCH_FULL_CPUS", ",".join(map(str, sorted(allowed))))
        os.sched_setaffinity(0, pick)
        return {"cpus": len(pick), "per_l3": k, "l3_domains": len(domains)}
    except (OSError, ValueError) as e:
        return {"cpu_spread_error": repr(e)[:200]}


def main():
    spread = _cpu_spread()
    several = int(os.environ.get("WORLD_SIZE", "1")) > 1
    numa = _numa_bind() if several else None  # (N == 1: after the multi-process measurements, see below)
    a = _args()
    # stdout carries exactly one line, the result JSON: everything else any library, child process or the gloo
    # rendezvous writes to fd 1 goes to stderr
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    if os.environ.get("PCCL_BENCH_WATCHDOG"):  # periodic Python stacks of every thread (hang diagnosis)
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["PCCL_BENCH_WATCHDOG"]), repeat=True)
    # N == 1: the measurements with one process per peer (BASELINE configs 5 / 4, the per-process Python latency) run
    # first, before this process creates its own GPU context: 8-9 peer processes on one GPU next to a process holding
    # its queues (the headline's 8 peers, copy queues, stream pools) oversubscribe the GPU's hardware queues, and the
    # time-sliced queues made config 5 on the xGMI path run into its deadline (55.9 vs 8.9 ms per op standalone,
    # profiles/r5/b2 vs b4) and the small-op latency bimodal
    pre = {}
    if not a.extras_child and not a.quick and not several:
        pre = pre_gpu_measurements(a)
    if not several:  # (bound after the multi-process measurements, which keep the full mask)
        numa = _numa_bind()
    job = Job(a)
    nbytes = a.mib << 20
    P = job.total
    if a.extras_child:
        extra, sweep = run_extras(job, a, nbytes)
        if job.rank == 0:
            with open(a.extras_child, "w") as f:
                json.dump({"extra": extra, "sweep": sweep}, f)
        if job.dist is not None:
            job.dist.barrier()
            job.dist.destroy_process_group()
        return
    extra = {}

    # ---- headline: TCP device ring, P peers x 1 GiB bf16
    ring = measure(job, ipc=False, nbytes=nbytes, steps=a.steps, warmup=a.warmup, check=not a.quick,
                   sweep=() if a.quick else (1 << 20, 16 << 20, 256 << 20), windows=max(1, a.windows),
                   label="headline_device_ring")
    import pccl_amd as pccl
    alg, bus = _bw(nbytes, ring["t"], P)
    path_name = pccl.ReducePath(ring["path"]).name
    wins = sorted(ring["windows"])
    ops = sorted(ring["op_ms"])
    extra.update({"bus_bw_per_peer_GBps": round(bus, 3), "aggregate_bus_bw_GBps": round(bus * P, 3),
                  "alg_bw_GBps": round(alg, 3),
                  "windows_ms": [round(w * 1e3, 2) for w in ring["windows"]],
                  "windows_ms_min": round(wins[0] * 1e3, 2), "windows_ms_median": round(statistics.median(wins) * 1e3, 2),
                  "op_ms_rank0": {"min": ops[0], "median": round(statistics.median(ops), 2), "max": ops[-1]},
                  "ref_metric_rx_plus_tx_per_peer_GBps": round((ring["tx"] + ring["rx"]) / ring["t"] / 1e9, 3),
                  "reduce_path": path_name, "peers_per_gpu": job.local, "p2p_connections_per_neighbour": ring["pool"],
                  "cpu_cores_busy_rank0": round(ring["cpu_cores"], 2), "cpus_available": _cpu_quota(),
                  "cpu_by_thread_rank0": getattr(job, "cpu_by_thread", None),
                  "result_exact": ring.get("ok")})
    extra["per_rank"] = _per_rank_diag(ring, nbytes, P)
    extra["per_rank_phases"] = list(job.phase_log)
    sweep = {"DEVICE_RING": {str(b >> 20) + "MiB": {"ms": round(t * 1e3, 3),
                                                    "bus_bw_per_peer_GBps": round(_bw(b, t, P)[1], 3)}
                             for b, t in ring["sweep"].items()}}
    sweep["DEVICE_RING"][f"{a.mib}MiB"] = {"ms": round(ring["t"] * 1e3, 3), "bus_bw_per_peer_GBps": round(bus, 3)}
    if not a.quick:
        # PCCL_BENCH_EXTRAS_INPROC=1: the extras in this process (rehearsals with many ranks on one GPU, where a child
        # per rank would double the processes holding the GPU)
        if os.environ.get("PCCL_BENCH_EXTRAS_INPROC") == "1":
            x_extra, x_sweep = run_extras(job, a, nbytes)
        else:
            x_extra, x_sweep = extras_in_child(job, a)
        headline_phases = job.phase_log[:1] if os.environ.get("PCCL_BENCH_EXTRAS_INPROC") != "1" else []
        extra.update(x_extra)
        extra["per_rank_phases"] = headline_phases + x_extra.get("per_rank_phases", [])
        sweep.update(x_sweep)
        if "latency_1MiB_ipc_python_processes" in pre:
            extra["latency_1MiB_ipc_python_processes"] = pre["latency_1MiB_ipc_python_processes"]
        if "baseline_configs" in pre:
            cfg = pre["baseline_configs"]
            extra["baseline_configs"] = cfg
            c5 = cfg.get("config5_kill_rejoin_tcp", {})
            # the metric's "peer-rejoin latency": BASELINE config 5 on the TCP device ring, the replacement process's
            # connect() -> its first exact all-reduce with the full world (admission vote + P2P establishment + op)
            extra["peer_rejoin_latency_ms"] = c5.get("joiner_connect_to_first_exact_op_ms")
            extra["peer_rejoin_latency_source"] = ("BASELINE config 5, TCP device ring: replacement process's connect() "
                                                   "-> its first exact 1 GiB all-reduce at full world, after a peer was "
                                                   "SIGKILLed mid-op")
            c5s = cfg.get("config5_stop_rejoin_tcp", {})
            # a peer that stops without closing its sockets (SIGSTOP): detection by the liveness protocol alone
            extra["stopped_peer_detection_ms"] = {
                "peer_timeout_ms": c5s.get("peer_timeout_ms"),
                "stop_to_survivors_failed_op_ms": c5s.get("stop_to_survivors_failed_op_ms"),
                "stop_to_survivors_first_exact_op_ms": c5s.get("stop_to_survivors_first_exact_op_ms")}
        if "peer_curve" in extra:
            extra["peer_curve"].setdefault("DEVICE_RING", {})[str(P)] = _curve_point(nbytes, ring["t"], P)
    extra["sweep"] = sweep
    if numa is not None:
        extra["numa_bind"] = numa
    extra["cpu_affinity"] = spread or {"cpus": len(os.sched_getaffinity(0)), "per_l3": "all"}

    cfg_model = (f"{P}-peer ring all-reduce (SUM), {a.mib} MiB bf16 HIP device buffer per peer, "
                 f"{'loopback TCP device ring' if path_name == 'DEVICE_RING' else path_name}")
    line = {
        "metric": METRIC, "value": round(bus, 3),
        "unit": "GB/s (per-peer nccl-tests busBW of the 1 GiB all-reduce; job aggregate in extra)",
        "n_gpus": job.n_gpus, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ring["t"] * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (torch.randn bf16 on device)",
        "config": {"model": cfg_model, "global_batch": P, "seq_len": nbytes // 2,
                   "parallelism": f"{P} peers on {job.n_gpus} GPU{'s' if job.n_gpus > 1 else ''} "
                                  f"({job.local} per GPU), reduce path {path_name}",
                   "tensor_bytes": nbytes, "n_peers": P, "reduce_path": path_name},
        "extra": extra,
    }
    if job.rank == 0:
        print(json.dumps(line), file=result_out, flush=True)
    if job.dist is not None:
        job.dist.barrier()
        job.dist.destroy_process_group()


if __name__ == "__main__":
    main()
