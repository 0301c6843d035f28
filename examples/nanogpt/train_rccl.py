"""Baseline: plain PyTorch DDP over RCCL (torch.distributed backend "nccl" = RCCL on ROCm), no PCCL — the
comparison point of the reference's python/examples/nanogptddp/train_nccl.py.

    torchrun --nproc-per-node 8 train_rccl.py --preset gpt2-124m
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from common import Timer, build, device_of, get_lr, parser  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: E402


def main():
    a = parser(__doc__).parse_args()
    device = device_of(a)
    distributed = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if distributed:
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo")
    cfg, model, opt, data, ctx = build(a, device)
    ddp = DDP(model, device_ids=[device.index] if device.type == "cuda" else None,
              bucket_cap_mb=256, gradient_as_bucket_view=True) if distributed else model
    world = dist.get_world_size() if distributed else 1
    tokens_per_iter = a.batch_size * cfg.block_size * a.grad_accum * world
    timer = Timer()
    for it in range(a.max_iters):
        for g in opt.param_groups:
            g["lr"] = get_lr(it, a)
        opt.zero_grad(set_to_none=True)
        for micro in range(a.grad_accum):
            x, y = data.batch(a.batch_size, cfg.block_size, device)
            if distributed:
                ddp.require_backward_grad_sync = micro == a.grad_accum - 1
            with ctx:
                _, loss = ddp(x, y)
            (loss / a.grad_accum).backward()
        if a.grad_clip:
            torch.nn.utils.clip_grad_norm_(model.parameters(), a.grad_clip)
        opt.step()
        dt = timer.lap()
        if not distributed or dist.get_rank() == 0:
            print(json.dumps({"iter": it, "loss": round(loss.item(), 4), "ms": round(dt * 1e3, 1),
                              "tok_s": round(tokens_per_iter / dt, 1),
                              "mfu": round(model.estimate_mfu(tokens_per_iter // world, dt), 4)}), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
