"""Shared pieces of the nanoGPT examples: config, model/data construction, LR schedule, eval, checkpoints.

Reference: python/examples/nanogptddp/train_pccl.py and nanogpt_diloco/*.py (config dicts, get_lr cosine schedule,
estimate_loss, ckpt.pt). Checkpoints are written with torch.save and read back with weights_only=True.
"""
import argparse
import math
import os
import sys
import time
from contextlib import nullcontext

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from pccl_amd.models import GPT, GPTConfig  # noqa: E402
from pccl_amd.models.data import TokenStream  # noqa: E402

PRESETS = {
    "gpt2-124m": dict(n_layer=12, n_head=12, n_embd=768, block_size=1024),
    "tiny": dict(n_layer=2, n_head=2, n_embd=64, block_size=64, vocab_size=512),
}


def parser(desc: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("--master", default=os.environ.get("PCCL_MASTER", "127.0.0.1:48148"))
    ap.add_argument("--preset", default="gpt2-124m", choices=sorted(PRESETS))
    ap.add_argument("--data", default=None, help="uint16 token memmap (nanoGPT train.bin); synthetic if absent")
    ap.add_argument("--batch-size", type=int, default=12)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--max-iters", type=int, default=100)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--min-lr", type=float, default=6e-5)
    ap.add_argument("--warmup-iters", type=int, default=10)
    ap.add_argument("--weight-decay", type=float, default=0.1)
    ap.add_argument("--grad-clip", type=float, default=1.0)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--dtype", default="bfloat16", choices=["float32", "bfloat16"])
    ap.add_argument("--out-dir", default=None, help="checkpoint directory (ckpt.pt); resume if present")
    ap.add_argument("--eval-interval", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1337)
    ap.add_argument("--min-world", type=int, default=2, help="peers required before training starts")
    return ap


def device_of(a) -> torch.device:
    if a.device == "cuda":
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    return torch.device(a.device)


def build(a, device: torch.device):
    torch.manual_seed(a.seed)
    cfg = GPTConfig(**PRESETS[a.preset])
    model = GPT(cfg).to(device)
    opt = model.configure_optimizers(a.weight_decay, a.lr, (0.9, 0.95), device.type)
    data = TokenStream(a.data, vocab_size=cfg.vocab_size, seed=a.seed + int(os.environ.get("RANK", "0")) + os.getpid())
    ctx = torch.autocast(device_type=device.type, dtype=torch.bfloat16) if a.dtype == "bfloat16" else nullcontext()
    return cfg, model, opt, data, ctx


def get_lr(it: int, a) -> float:
    if it < a.warmup_iters:
        return a.lr * (it + 1) / (a.warmup_iters + 1)
    if it > a.max_iters:
        return a.min_lr
    ratio = (it - a.warmup_iters) / max(1, a.max_iters - a.warmup_iters)
    return a.min_lr + 0.5 * (1.0 + math.cos(math.pi * ratio)) * (a.lr - a.min_lr)


@torch.no_grad()
def estimate_loss(model, data, cfg, a, device, ctx, iters: int = 5) -> float:
    model.eval()
    tot = 0.0
    for _ in range(iters):
        x, y = data.batch(a.batch_size, cfg.block_size, device)
        with ctx:
            _, loss = model(x, y)
        tot += float(loss)
    model.train()
    return tot / iters


def save_checkpoint(a, model, opt, it: int) -> None:
    if not a.out_dir:
        return
    os.makedirs(a.out_dir, exist_ok=True)
    torch.save({"model": model.state_dict(), "optimizer": opt.state_dict(), "iter_num": it},
               os.path.join(a.out_dir, "ckpt.pt"))


def load_checkpoint(a, model, opt) -> int:
    path = os.path.join(a.out_dir, "ckpt.pt") if a.out_dir else None
    if not path or not os.path.exists(path):
        return 0
    ck = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(ck["model"])
    opt.load_state_dict(ck["optimizer"])
    return int(ck["iter_num"])


class Timer:
    def __init__(self):
        self.t = time.perf_counter()

    def lap(self) -> float:
        now = time.perf_counter()
        dt, self.t = now - self.t, now
        return dt
