"""Interleaved A/B of device-ring knobs inside ONE bench process (8 threaded peers on cuda:0, TCP device ring):
windows of K ops alternate between variants (env settings applied while every peer waits at a barrier; the library
reads these knobs per op), so slow drifts of a noisy box hit every variant alike. Prints one JSON line per variant
with the median / min ms per op over its windows.

    python scripts/ring_ab_interleaved.py --variants "s2:PCCL_RING_STRIPES=2;s4:PCCL_RING_STRIPES=4" [--windows 6]
                                          [--ops 4] [--peers 8] [--mib 1024] [--pool 0]
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--ops", type=int, default=4)
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--pool", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--quant", action="store_true", help="uint8 min-max quantized ring instead of plain bf16")
    a = ap.parse_args()
    variants = []
    for v in a.variants.split(";"):
        name, _, envs = v.partition(":")
        kv = dict(e.split("=", 1) for e in envs.split(",") if e)
        variants.append((name, kv))
    import torch

    import bench
    import pccl_amd as pccl
    ba = argparse.Namespace(gpus=1, steps=a.ops, warmup=a.warmup, peers=a.peers, mib=a.mib, pool=a.pool, windows=1,
                            quick=True, no_ipc_extra=True, no_peer_curve=True, no_quant_extra=True, extras_child="")
    job = bench.Job(ba)
    n = (a.mib << 20) // 2
    times = {name: [] for name, _ in variants}
    extra = {name: [] for name, _ in variants}  # per window: (cgroup throttled ms, process CPU cores busy)

    def throttled_us():
        try:
            with open("/sys/fs/cgroup/cpu.stat") as f:
                for ln in f:
                    if ln.startswith("throttled_usec"):
                        return int(ln.split()[1])
        except OSError:
            pass
        return 0
    lock = threading.Lock()

    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if a.quant else None

    def fn(i, comm):
        x = torch.randn(n, device=job.dev, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        tag = 0
        for _ in range(a.warmup):
            comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag, quantization_options=qopt)
            tag += 1
        for w in range(a.windows):
            for name, kv in (variants if w % 2 == 0 else variants[::-1]):
                job.sync(i)
                if i == 0:
                    for k, v in kv.items():
                        os.environ[k] = v
                job.sync(i)
                # a first op under the new settings (pooled buffers of the new shape), untimed
                comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag, quantization_options=qopt)
                tag += 1
                torch.cuda.synchronize()
                job.sync(i)
                th0, c0 = throttled_us(), time.process_time()
                t0 = time.perf_counter()
                for _ in range(a.ops):
                    comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag, quantization_options=qopt)
                    tag += 1
                torch.cuda.synchronize()
                job.sync(i)
                wall = time.perf_counter() - t0
                dt = wall / a.ops
                if i == 0:
                    with lock:
                        times[name].append(dt * 1e3)
                        extra[name].append((round((throttled_us() - th0) / 1e3, 1),
                                            round((time.process_time() - c0) / wall, 2)))
        return True

    job.phase(fn, ipc=False)
    for name, _ in variants:
        t = times[name]
        print(json.dumps({"variant": name, "env": dict(variants)[name], "median_ms": round(statistics.median(t), 2),
                          "min_ms": round(min(t), 2), "windows_ms": [round(v, 1) for v in t],
                          "throttled_ms_and_cores": extra[name]}), flush=True)


if __name__ == "__main__":
    main()
