"""BASELINE config 3: int8/uint8-quantized all-reduce over a simulated 50 ms WAN, 8 peers.

    python benchmarks/wan_quantized.py [--peers 8] [--mib 2048] [--latency-ms 50] [--flow-mbit 1000]
                                        [--link-mbit 25000] [--device cuda:0|cpu] [--pool 16] [--concurrent 8]
                                        [--concurrent-quant 32] [--stripes 4]

Defaults model a transatlantic long fat pipe: 50 ms one way, ~1 Gbit/s per TCP flow (window-limited at 100 ms RTT),
a 25 Gbit/s NIC per peer (the reference's transatlantic figure), 16 pooled connections per neighbour.

Peer processes on one host behind a WAN emulator -- tc-netem needs root, which the benchmark boxes do not grant:
  * --emulator relay (default): pccl_wan_relay, a separate process outside the library (csrc/tools/wan_relay.cpp);
    every peer advertises a relay port as its P2P address and the relay delays each byte by the one-way latency and
    paces it per TCP connection and per link (token buckets). The library cannot influence this link.
  * --emulator builtin: the in-library pacing model (PCCL_SIM_WAN, csrc/net/mux.hpp), for comparison.
The xGMI IPC path is disabled (PCCL_DISABLE_IPC=1) so every byte crosses the emulated WAN through the TCP ring:
device tensors are staged through pinned memory and (de)quantized by the HIP kernels.
For each wire format (fp32 / uint8 min-max / int8 zero-point-scale / fp8 e4m3 min-max) an AVG all-reduce of --mib MiB
of fp32 per peer, split into --concurrent slices in flight at once, is timed after a warm-up. Reported per format:
  * seconds, effective algorithm bandwidth (fp32 bytes / time) and bus bandwidth (x 2(n-1)/n),
  * the reference's metric: (rx + tx wire bytes) / time per peer, in Gbit/s -- comparable to its published
    25 / 45 Gbit/s WAN figures (docs/md/01_Introduction.md:8), which were link-limited as the emulated link is here,
  * the max abs error vs the exact fp32 average.
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FORMATS = ["fp32", "uint8", "int8_zps", "fp8"]


def peer(a):
    import torch

    import pccl_amd as pccl
    from pccl_amd.utils import wait_for_world
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    ports = json.loads(a.ports) if a.ports else {}
    comm = pccl.Communicator(a.master, 0, p2p_connection_pool_size=a.pool, **ports)
    comm.connect(n_attempts=60)
    wait_for_world(comm, a.peers, timeout=300)
    D, Q = pccl.DataType, pccl.QuantizationAlgorithm
    qopts = {"fp32": None, "uint8": pccl.QuantizationOptions(D.UINT8, Q.MIN_MAX),
             "int8_zps": pccl.QuantizationOptions(D.INT8, Q.ZERO_POINT_SCALE),
             "fp8": pccl.QuantizationOptions(D.FLOAT8_E4M3, Q.MIN_MAX)}
    n = (a.mib << 20) // 4

    def inputs(r, k=None, device="cpu"):  # deterministic, size-independent synthetic data (no RNG stream to replay)
        i = torch.arange(n if k is None else k, dtype=torch.float32, device=device)
        return torch.sin(0.37 * i + r) * (1.0 + 0.1 * r) + 0.05 * torch.cos(0.011 * i * (r + 1))

    check = min(n, 1 << 20)
    # the exact average of the first `check` elements, from every peer's inputs computed on this peer's device
    exact = torch.stack([inputs(r, check, dev) for r in range(a.peers)]).double().mean(0).float().cpu()
    x = inputs(a.rank, device=dev)
    out = {}
    tag = 0
    for f in a.formats.split(","):
        y = torch.empty_like(x)
        comm.all_reduce(x[:65536], y[:65536], op=pccl.ReduceOp.AVG, tag=tag, quantization_options=qopts[f])
        tag += 1
        # --concurrent all-reduces of equal slices in flight at once over the connection pool (the reference's
        # recipe for long fat pipes: pcclAllReduceMultipleWithRetry, docs/md/01_Introduction.md:8). A quantized
        # op moves 4x fewer bytes per ring step while every step still pays the link latency (and a reduce-scatter
        # step cannot start before the previous one's min / max exist): --concurrent-quant slices keep the link busy
        conc = a.concurrent if qopts[f] is None else (a.concurrent_quant or a.concurrent)
        q = qopts[f] or pccl.QuantizationOptions(D.FLOAT, Q.NONE)
        per = (n + conc - 1) // conc
        descs = []
        for k in range(conc):
            lo, hi = k * per, min(n, (k + 1) * per)
            rd = pccl.ReduceDescriptor(hi - lo, pccl.ReduceOp.AVG, tag, pccl.ReduceOperandDescriptor(D.FLOAT), q)
            descs.append(pccl.ReduceOpDescriptor.from_torch(x[lo:hi], y[lo:hi], rd))
            tag += 1
        reps = []
        for rep in range(a.repeat):
            if rep:  # the same ops again under fresh tags (every peer derives the same tag sequence)
                for d in descs:
                    d.reduce_descriptor.tag = tag
                    tag += 1
            if dev.type == "cuda":
                torch.cuda.synchronize()
            pstats0 = pccl.memory.staging_pool_stats(reset_peak=True)
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            t0 = time.perf_counter()
            info = run_multi(comm, descs, conc, a.cohorts, a.cohort_delay_ms)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            pstats = pccl.memory.staging_pool_stats()
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
            reps.append({"seconds": dt, "tx": info.tx_bytes, "rx": info.rx_bytes, "cpu_cores": cpu / max(dt, 1e-9),
                         "pinned_peak": pstats["pinned"]["peak"], "pinned_allocs": pstats["pinned"].get("allocs", 0)
                         - pstats0["pinned"].get("allocs", 0),
                         "alloc_ms": sum(pstats[k].get("alloc_us", 0) - pstats0[k].get("alloc_us", 0)
                                         for k in ("pinned", "device")) / 1e3})
        err = float((y[:check].cpu() - exact).abs().max())
        out[f] = dict(reps[-1], max_abs_err=err, reps=reps)
    print(json.dumps({"rank": a.rank, "res": out}), flush=True)
    comm.destroy()


def run_multi(comm, descs, conc, cohorts=1, delay_ms=0.0):
    """all_reduce_multiple_with_retry over `descs` with `conc` in flight; with --cohorts K > 1 (experiment) the ops are
    split into K interleaved cohorts, each its own multi-op call on its own thread, cohort k starting k x delay_ms
    later, so the cohorts' ring steps are out of phase (one cohort transfers while another waits out the latency)."""
    if cohorts <= 1:
        return comm.all_reduce_multiple_with_retry(descs, max_in_flight=conc)
    import threading
    groups = [descs[k::cohorts] for k in range(cohorts)]
    infos = [None] * cohorts
    errs = []

    def body(k):
        try:
            time.sleep(k * delay_ms / 1e3)
            infos[k] = comm.all_reduce_multiple_with_retry(groups[k], max_in_flight=max(1, conc // cohorts))
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    ths = [threading.Thread(target=body, args=(k,)) for k in range(cohorts)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    tx = sum(i.tx_bytes for i in infos)
    rx = sum(i.rx_bytes for i in infos)
    return type(infos[0])(infos[0].local_world_size, tx, rx)


def _proc_cpu_s(pid):
    """user + sys CPU seconds of a process (the relay: its CPU use next to the bytes it moved)."""
    with open(f"/proc/{pid}/stat") as f:
        st = f.read()
    fields = st[st.rindex(")") + 2:].split()
    return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--mib", type=int, default=2048)
    ap.add_argument("--latency-ms", type=float, default=50)
    ap.add_argument("--flow-mbit", type=float, default=1000)
    ap.add_argument("--link-mbit", type=float, default=25000)
    ap.add_argument("--pool", type=int, default=16)
    ap.add_argument("--concurrent", type=int, default=8, help="all-reduces in flight (slices of the tensor)")
    ap.add_argument("--concurrent-quant", type=int, default=32, help="the same for the quantized formats (0: --concurrent)")
    ap.add_argument("--stripe-min-kib", type=int, default=1024,
                    help="PCCL_STRIPE_MIN_BYTES / 1024: smallest stripe of a ring step (>= 256)")
    ap.add_argument("--stripes", type=int, default=0, help="PCCL_RING_STRIPES (connections per ring step; 0 = default)")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--repeat", type=int, default=2,
                    help="run each format's multi-op this many times: the summary is the last (warm) one, the first "
                         "(cold: staging pools and connections' first use) is reported alongside")
    ap.add_argument("--formats", default=",".join(FORMATS))
    ap.add_argument("--emulator", default="relay", choices=["relay", "builtin"])
    ap.add_argument("--log-dir", default=None, help="keep every peer's stderr here")
    ap.add_argument("--cohorts", type=int, default=1, help=argparse.SUPPRESS)  # experiment: out-of-phase op cohorts
    ap.add_argument("--cohort-delay-ms", type=float, default=0.0, help=argparse.SUPPRESS)
    ap.add_argument("--ports", default="", help=argparse.SUPPRESS)  # internal: Communicator port kwargs (JSON)
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--master", default=None)
    a = ap.parse_args()
    if a.rank is not None:
        return peer(a)
    from pccl_amd.utils import free_ports, local_master, spawn_python
    env = {"PCCL_DISABLE_IPC": "1", "OMP_NUM_THREADS": "2", "PCCL_STRIPE_MIN_BYTES": str(a.stripe_min_kib << 10),
           "PCCL_MAX_CONCURRENT_COLLECTIVE_OPS": str(max(16, a.concurrent, a.concurrent_quant))}
    if a.stripes:
        env["PCCL_RING_STRIPES"] = str(a.stripes)
    args = ["--peers", str(a.peers), "--mib", str(a.mib), "--pool", str(a.pool), "--device", a.device,
            "--concurrent", str(a.concurrent), "--concurrent-quant", str(a.concurrent_quant),
            "--formats", a.formats, "--repeat", str(a.repeat), "--cohorts", str(a.cohorts),
            "--cohort-delay-ms", str(a.cohort_delay_ms)]
    relay = None
    peer_ports = [{} for _ in range(a.peers)]
    if a.emulator == "builtin":
        env["PCCL_SIM_WAN"] = f"{a.latency_ms}:{a.flow_mbit}:{a.link_mbit}"
    else:
        fp = free_ports(4 * a.peers)
        maps = []
        for r in range(a.peers):
            listen, adv, ss, bm = fp[4 * r:4 * r + 4]
            peer_ports[r] = {"p2p_listen_port": listen, "advertised_p2p_port": adv, "shared_state_listen_port": ss,
                             "benchmark_listen_port": bm}
            maps += ["--map", f"{adv}:{listen}"]
        exe = os.path.join(ROOT, "pccl_amd", "lib", "pccl_wan_relay")
        relay = subprocess.Popen([exe, "--delay-ms", str(a.latency_ms), "--flow-mbit", str(a.flow_mbit),
                                  "--link-mbit", str(a.link_mbit), *maps], stdout=subprocess.PIPE,
                                 stderr=subprocess.DEVNULL, text=True)
        relay.stdout.readline()  # {"relay": "ready"}
    t_run0 = time.perf_counter()
    relay_cpu0 = _proc_cpu_s(relay.pid) if relay is not None else None
    relay_cpu = None
    try:
        with local_master() as addr:
            ps = [spawn_python([os.path.abspath(__file__), "--rank", str(r), "--master", addr, "--ports",
                                json.dumps(peer_ports[r]), *args], env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(a.peers)]
            outs = [p.communicate(timeout=1500) for p in ps]
            if a.log_dir:  # every peer's stderr (e.g. PCCL_TRACE_OPS=1 phase lines)
                os.makedirs(a.log_dir, exist_ok=True)
                for r, (_, e) in enumerate(outs):
                    with open(os.path.join(a.log_dir, f"peer{r}.err"), "w") as f:
                        f.write(e)
    finally:
        relayed = None
        if relay is not None and relay.poll() is None:
            relay_cpu = _proc_cpu_s(relay.pid) - relay_cpu0
        if relay is not None:
            relay.terminate()
            try:
                line = relay.stdout.readline()
                relayed = json.loads(line).get("relayed_bytes") if line.startswith("{") else None
                relay.wait(timeout=10)
            except (subprocess.TimeoutExpired, ValueError):
                relay.kill()
                relay.wait()
    res = []
    for p, (o, e) in zip(ps, outs):
        if p.returncode != 0:
            raise RuntimeError(e[-3000:])
        res.append(json.loads([x for x in o.splitlines() if x.startswith("{")][-1])["res"])
    nbytes = (a.mib << 20)
    summary = {}
    for f in a.formats.split(","):
        t = max(r[f]["seconds"] for r in res)
        wire = max((r[f]["tx"] + r[f]["rx"]) / r[f]["seconds"] for r in res)
        alg = nbytes / t
        cold = max(r[f]["reps"][0]["seconds"] for r in res)
        summary[f] = {"seconds": round(t, 4), "repeat_reported": "warm (last of %d)" % a.repeat if a.repeat > 1
                      else "cold (single run)", "seconds_cold": round(cold, 4), "alg_GBps": round(alg / 1e9, 3),
                      "bus_GBps": round(alg * 2 * (a.peers - 1) / a.peers / 1e9, 3),
                      "ref_metric_rx_plus_tx_Gbit_per_peer": round(wire * 8 / 1e9, 2),
                      "effective_fp32_Gbit_per_peer": round(2 * nbytes * (a.peers - 1) / a.peers * 2 / t * 8 / 1e9, 2),
                      "max_abs_err": max(r[f]["max_abs_err"] for r in res),
                      "seconds_per_repeat": [round(max(r[f]["reps"][k]["seconds"] for r in res), 4)
                                             for k in range(a.repeat)],
                      "pinned_peak_MiB_max_peer": round(max(r[f]["pinned_peak"] for r in res) / 2**20, 1),
                      "pinned_allocs_per_repeat_max_peer": [max(r[f]["reps"][k]["pinned_allocs"] for r in res)
                                                            for k in range(a.repeat)],
                      "alloc_ms_per_repeat_max_peer": [round(max(r[f]["reps"][k]["alloc_ms"] for r in res), 1)
                                                       for k in range(a.repeat)],
                      # CPU cores the peer processes kept busy (sum over peers) while the multi-op ran
                      "peer_cpu_cores_per_repeat": [round(sum(r[f]["reps"][k]["cpu_cores"] for r in res), 2)
                                                    for k in range(a.repeat)]}
    emulator = ("userspace relay (pccl_wan_relay, a separate process)" if a.emulator == "relay"
                else "in-library pacing (PCCL_SIM_WAN)")
    quant = [f for f in a.formats.split(",") if f != "fp32"]
    cq = a.concurrent_quant or a.concurrent
    if not quant:
        ops = f"{a.concurrent} ops in flight"
    elif "fp32" not in a.formats.split(","):
        ops = f"{cq} ops in flight"
    else:
        ops = f"{a.concurrent} ops in flight (fp32), {cq} (quantized)"
    config = (f"{'/'.join(a.formats.split(','))} AVG all-reduce of {a.mib} MiB fp32 per peer, {a.peers} peers "
              f"({a.device}, one process each, TCP ring), {ops}, {a.pool} connections per neighbour, emulated WAN: "
              f"{emulator}, {a.latency_ms:g} ms one way, {a.flow_mbit:g} Mbit/s per flow, {a.link_mbit:g} Mbit/s "
              f"per link; warm repeat of {a.repeat}")
    print(json.dumps({"metric": "all-reduce over emulated WAN" + (" (quantized formats)" if quant else ""),
                      "config": config,
                      "peers": a.peers, "mib_per_peer": a.mib, "device": a.device,
                      "wan": {"emulator": "pccl_wan_relay (separate process)" if a.emulator == "relay"
                              else "PCCL_SIM_WAN (inside the library)",
                              "one_way_latency_ms": a.latency_ms, "flow_mbit": a.flow_mbit, "link_mbit": a.link_mbit,
                              "pool": a.pool, "concurrent_ops": a.concurrent,
                              "concurrent_ops_quantized": a.concurrent_quant or a.concurrent, "stripes": a.stripes or 4,
                              "relayed_GB": round(relayed / 1e9, 3) if relayed is not None else None,
                              "relay_cpu_s": round(relay_cpu, 2) if relay_cpu is not None else None,
                              "run_s": round(time.perf_counter() - t_run0, 2)},
                      "reference_published_Gbit": {"transatlantic": 25, "collocated_eu": 45},
                      "formats": summary}), flush=True)


if __name__ == "__main__":
    main()
