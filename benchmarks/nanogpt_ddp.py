"""Application benchmark: nanoGPT (GPT-2 124M) data-parallel training over PCCL on one MI355X.

    python benchmarks/nanogpt_ddp.py [--peers 2] [--iters 30] [--batch-size 12] [--overlap]

Spawns an in-process master and `peers` training processes of examples/nanogpt/train_pccl.py on cuda:0 (synthetic
tokens, bf16 autocast, AdamW). Gradients are all-reduced as device buckets in fd-shareable memory over the xGMI path
(peers are separate processes on one host). Reports the median iteration time, tokens/s over all peers, and the
median forward+backward and gradient all-reduce phase times (reference workload:
python/examples/nanogptddp/train_pccl.py; the reference publishes no number for it).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=2)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--batch-size", type=int, default=12)
    ap.add_argument("--preset", default="gpt2-124m")
    ap.add_argument("--overlap", action="store_true")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from pccl_amd.utils import local_master, spawn_python
    script = os.path.join(ROOT, "examples", "nanogpt", "train_pccl.py")
    args = ["--preset", a.preset, "--device", a.device, "--batch-size", str(a.batch_size), "--max-iters",
            str(a.iters), "--dtype", "bfloat16"] + (["--overlap"] if a.overlap else [])
    with local_master() as addr:
        ps = [spawn_python([script, "--master", addr, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True) for _ in range(a.peers)]
        outs = [p.communicate(timeout=1200) for p in ps]
    for p, (_, e) in zip(ps, outs):
        if p.returncode != 0:
            raise RuntimeError(e[-3000:])
    recs = [[json.loads(x) for x in o.splitlines() if x.startswith("{") and '"iter"' in x and '"ms"' in x]
            for o, _ in outs]
    done = [json.loads([x for x in o.splitlines() if x.startswith("{")][-1]) for o, _ in outs]
    skip = max(3, a.iters // 5)  # warm-up iterations (allocator, first shared-state sync, IPC mappings)
    ms = [r["ms"] for rr in recs for r in rr[skip:]]
    fb = [r["phase_ms"].get("forward_backward", 0.0) for rr in recs for r in rr[skip:]]
    ar = [r["phase_ms"].get("all_reduce", 0.0) for rr in recs for r in rr[skip:]]
    tok = [r["tok_s"] for rr in recs for r in rr[skip:]]
    print(json.dumps({
        "metric": "nanoGPT DDP over PCCL", "preset": a.preset, "peers": a.peers, "device": a.device,
        "batch_size": a.batch_size, "overlap": a.overlap, "iters": a.iters,
        "median_iter_ms": round(statistics.median(ms), 2),
        "tokens_per_s_all_peers": round(statistics.median(tok) * a.peers, 1),
        "median_forward_backward_ms": round(statistics.median(fb), 2),
        "median_grad_all_reduce_ms": round(statistics.median(ar), 2),
        "peers_identical": len({d.get("param_sum") for d in done}) == 1}), flush=True)


if __name__ == "__main__":
    main()
