"""GPT-2-style decoder (nanoGPT, the workload of the reference's DDP / DiLoCo examples).

Behavioural parity with /root/reference/python/examples/nanogptddp/model.py (GPTConfig defaults = GPT-2 124M,
pre-LN blocks, fused QKV projection, causal SDPA, GELU MLP, tied input/output embeddings, scaled init of residual
projections, AdamW param groups with/without weight decay, 6N+12LHQT FLOP estimate). Written for MI355X:

* attention is ``scaled_dot_product_attention`` (PyTorch-ROCm dispatches it to its CK/AOTriton flash kernels);
* training runs in bf16 autocast (MFU priced against the 2.5 PFLOP/s dense bf16 peak of one MI355X);
* AdamW uses the fused multi-tensor implementation when parameters live on the GPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

MI355X_BF16_DENSE_FLOPS = 2.5e15


@dataclass
class GPTConfig:
    block_size: int = 1024
    vocab_size: int = 50304  # 50257 padded to a multiple of 64
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    dropout: float = 0.0
    bias: bool = True


class Block(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.n_head = cfg.n_head
        self.dropout = cfg.dropout
        self.ln_1 = nn.LayerNorm(cfg.n_embd, bias=cfg.bias)
        self.c_attn = nn.Linear(cfg.n_embd, 3 * cfg.n_embd, bias=cfg.bias)
        self.c_proj = nn.Linear(cfg.n_embd, cfg.n_embd, bias=cfg.bias)
        self.ln_2 = nn.LayerNorm(cfg.n_embd, bias=cfg.bias)
        self.c_fc = nn.Linear(cfg.n_embd, 4 * cfg.n_embd, bias=cfg.bias)
        self.mlp_proj = nn.Linear(4 * cfg.n_embd, cfg.n_embd, bias=cfg.bias)
        self.drop = nn.Dropout(cfg.dropout)

    def attention(self, x: torch.Tensor) -> torch.Tensor:
        b, t, c = x.shape
        qkv = self.c_attn(x).view(b, t, 3, self.n_head, c // self.n_head)
        q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)  # each (B, nh, T, hs)
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=self.dropout if self.training else 0.0,
                                           is_causal=True)
        return self.drop(self.c_proj(y.transpose(1, 2).reshape(b, t, c)))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x + self.attention(self.ln_1(x))
        return x + self.drop(self.mlp_proj(F.gelu(self.c_fc(self.ln_2(x)))))


class GPT(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.config = cfg
        self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.block_size, cfg.n_embd)
        self.drop = nn.Dropout(cfg.dropout)
        self.h = nn.ModuleList(Block(cfg) for _ in range(cfg.n_layer))
        self.ln_f = nn.LayerNorm(cfg.n_embd, bias=cfg.bias)
        self.apply(self._init_weights)
        # GPT-2 scaled init of the residual projections
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight") or name.endswith("mlp_proj.weight"):
                nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * cfg.n_layer))

    @staticmethod
    def _init_weights(m: nn.Module) -> None:
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)

    def num_params(self, non_embedding: bool = True) -> int:
        n = sum(p.numel() for p in self.parameters())
        return n - self.wpe.weight.numel() if non_embedding else n

    def forward(self, idx: torch.Tensor, targets: Optional[torch.Tensor] = None
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        b, t = idx.shape
        assert t <= self.config.block_size, f"sequence {t} > block size {self.config.block_size}"
        pos = torch.arange(t, device=idx.device)
        x = self.drop(self.wte(idx) + self.wpe(pos))
        for blk in self.h:
            x = blk(x)
        x = self.ln_f(x)
        logits = F.linear(x, self.wte.weight)  # tied lm head
        if targets is None:
            return logits[:, -1:, :], None
        loss = F.cross_entropy(logits.float().view(-1, logits.size(-1)), targets.view(-1), ignore_index=-1)
        return logits, loss

    def crop_block_size(self, block_size: int) -> None:
        assert block_size <= self.config.block_size
        self.config.block_size = block_size
        self.wpe.weight = nn.Parameter(self.wpe.weight[:block_size].detach().clone())

    def configure_optimizers(self, weight_decay: float, learning_rate: float, betas=(0.9, 0.95),
                             device_type: str = "cuda") -> torch.optim.AdamW:
        params = [p for p in self.parameters() if p.requires_grad]
        decay = [p for p in params if p.dim() >= 2]
        no_decay = [p for p in params if p.dim() < 2]
        groups = [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]
        return torch.optim.AdamW(groups, lr=learning_rate, betas=betas, fused=device_type == "cuda")

    def flops_per_token(self) -> float:
        c = self.config
        return 6 * self.num_params() + 12 * c.n_layer * c.n_head * (c.n_embd // c.n_head) * c.block_size

    def estimate_mfu(self, tokens_per_iter: int, dt: float, peak: float = MI355X_BF16_DENSE_FLOPS) -> float:
        return self.flops_per_token() * tokens_per_iter / dt / peak

    @torch.no_grad()
    def generate(self, idx: torch.Tensor, max_new_tokens: int, temperature: float = 1.0,
                 top_k: Optional[int] = None) -> torch.Tensor:
        for _ in range(max_new_tokens):
            ctx = idx if idx.size(1) <= self.config.block_size else idx[:, -self.config.block_size:]
            logits, _ = self(ctx)
            logits = logits[:, -1, :] / temperature
            if top_k is not None:
                v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
                logits[logits < v[:, [-1]]] = -float("inf")
            idx = torch.cat((idx, torch.multinomial(F.softmax(logits, dim=-1), num_samples=1)), dim=1)
        return idx
