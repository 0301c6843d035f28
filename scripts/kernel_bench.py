"""Throughput of the pccl-amd HIP kernels on one MI355X (effective HBM GB/s = bytes read + written / time), with the
equivalent PyTorch ops as reference points.

    python scripts/kernel_bench.py [--mib 512] [--iters 20] > profiles/kernels.md
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pccl_amd.ops import kernels as K  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = (a.mib << 20) // 2  # bf16 elements
    bf = lambda: torch.randn(n, device=dev).to(torch.bfloat16)  # noqa: E731
    x, y = bf(), bf()
    rows = []

    def row(name, sec, nbytes, note=""):
        rows.append((name, sec * 1e6, nbytes / sec / 1e9, note))

    row("reduce_ bf16 sum (pccl)", timeit(lambda: K.reduce_(x, y, "sum"), a.iters), 3 * n * 2)
    row("torch add_ bf16", timeit(lambda: x.add_(y), a.iters), 3 * n * 2, "reference point")
    q, meta = K.quantize(y, torch.uint8, "min_max")
    row("quantize bf16->u8 min-max (pccl, 2 passes)", timeit(lambda: K.quantize(y, torch.uint8, "min_max"), a.iters),
        n * 2 * 2 + n)
    row("dequant_reduce u8->bf16 sum (pccl)", timeit(lambda: K.dequant_reduce(x, q, meta, "min_max", "sum"), a.iters),
        n + 2 * n * 2)
    ys = y.clone()
    row("quantize_setback bf16->u8 + D(Q(x)) back (pccl, min/max pass + fused pass)",
        timeit(lambda: K.quantize_setback(ys, torch.uint8, "min_max"), a.iters), n * 2 * 2 + n + n * 2)
    row("dequant_reduce_minmax u8->bf16 sum + min/max partials (pccl)",
        timeit(lambda: K.dequant_reduce_minmax(x, q, meta, "min_max", "sum"), a.iters), n + 2 * n * 2)
    qz, mz = K.quantize(y, torch.uint8, "zero_point_scale")
    row("quantize bf16->u8 zero-point-scale (pccl)",
        timeit(lambda: K.quantize(y, torch.uint8, "zero_point_scale"), a.iters), n * 2 * 2 + n)
    row("dequant_reduce u8 zps->bf16 sum (pccl)",
        timeit(lambda: K.dequant_reduce(x, qz, mz, "zero_point_scale", "sum"), a.iters), n + 2 * n * 2)
    if hasattr(torch, "float8_e4m3fn"):
        q8, m8 = K.quantize(y, torch.float8_e4m3fn, "min_max")
        row("quantize bf16->fp8 e4m3 (pccl)", timeit(lambda: K.quantize(y, torch.float8_e4m3fn, "min_max"), a.iters),
            n * 2 * 2 + n)
        row("dequant_reduce fp8->bf16 sum (pccl)",
            timeit(lambda: K.dequant_reduce(x, q8, m8, "min_max", "sum"), a.iters), n + 2 * n * 2)
    u8 = y.view(torch.uint8)
    dst2 = [torch.empty_like(x), torch.empty_like(x)]
    row("simplehash (pccl)", timeit(lambda: K.simplehash(u8), a.iters), n * 2)
    row("crc32c (pccl, tiled kernel + host fold)", timeit(lambda: K.crc32c(u8), a.iters), n * 2)
    row("multi_reduce 2 srcs -> 2 dsts bf16 (pccl push kernel)",
        timeit(lambda: K.multi_reduce([x, y], "sum", out=dst2[0], outs=[dst2[1]]), a.iters), 4 * n * 2)
    srcs = [bf() for _ in range(8)]
    m = n // 8
    shards = [s[:m] for s in srcs]
    out = torch.empty(m, device=dev, dtype=torch.bfloat16)
    row("multi_reduce 8 srcs bf16 (pccl)", timeit(lambda: K.multi_reduce(shards, "sum", out=out), a.iters), 9 * m * 2)
    dst = torch.empty(n, device=dev, dtype=torch.bfloat16)
    parts = [s[i * m:(i + 1) * m] for i, s in enumerate(srcs)]
    row("multi_gather 8 segments (pccl)",
        timeit(lambda: K.multi_gather(dst, parts, [i * m for i in range(8)], skip=-1), a.iters), 2 * 8 * m * 2)
    nf = n // 2
    outer = torch.randn(nf, device=dev)
    mom = torch.zeros_like(outer)
    pg = torch.empty_like(outer)
    local = outer.to(torch.bfloat16)
    row("pseudo_grad fp32/bf16 (pccl)", timeit(lambda: K.pseudo_grad(pg, outer, local), a.iters), nf * (4 + 2 + 4))
    row("outer_sgd nesterov fused (pccl)",
        timeit(lambda: K.outer_sgd(outer, mom, pg, local, lr=0.7, momentum=0.9, nesterov=True), a.iters),
        nf * (12 + 8 + 2))
    p = torch.nn.Parameter(outer.clone())
    p.grad = pg.clone()
    opt = torch.optim.SGD([p], lr=0.7, momentum=0.9, nesterov=True, foreach=True)

    def torch_outer():
        opt.step()
        local.copy_(p.detach())

    row("torch SGD nesterov + copy (reference point)", timeit(torch_outer, a.iters), nf * (12 + 8 + 2),
        "same logical traffic")
    print(f"# pccl-amd kernel throughput, {a.mib} MiB bf16 operands, MI355X\n")
    print("| kernel | us / call | effective GB/s | note |")
    print("|---|---:|---:|---|")
    for name, us, gbs, note in rows:
        print(f"| {name} | {us:.1f} | {gbs:.0f} | {note} |")


if __name__ == "__main__":
    main()
