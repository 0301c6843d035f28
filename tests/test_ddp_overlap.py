"""DataParallel(overlap=True): bucket all-reduces start from post-accumulate-grad hooks during backward.

Checks against the synchronous path (same AVG gradients), unused parameters (buckets launched at sync time),
no_sync() accumulation, zero_grad(set_to_none=True) re-binding, and several steps in a row. CPU peers are threads in
one process; the GPU variant runs the same model on cuda:0 (xGMI IPC path between the two peers).
"""
import copy

import pytest
import torch

from pccl_amd.parallel import DataParallel
from pccl_amd.utils import local_master, run_threaded_peers


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(64, 256)
        self.b = torch.nn.Linear(256, 256)
        self.c = torch.nn.Linear(256, 8)
        self.unused = torch.nn.Linear(8, 8)  # never receives a gradient

    def forward(self, x):
        return self.c(torch.relu(self.b(torch.relu(self.a(x)))))


def _grads(model):
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


def _run(device, overlap, steps=3, accumulate=1, set_to_none=False):
    torch.manual_seed(0)
    base = Net()  # built once: the peer threads share torch's global RNG

    def fn(rank, comm):
        if device.startswith("cuda"):
            torch.cuda.set_device(device)
        model = copy.deepcopy(base).to(device)
        # ~70 KiB buckets: the 256x256 layer spans two of them, so hooks of one parameter complete two buckets
        dp = DataParallel(model, comm, bucket_bytes=70_000, overlap=overlap)
        g = torch.Generator().manual_seed(100 + rank)
        out = []
        for step in range(steps):
            if set_to_none:
                for p in model.parameters():
                    p.grad = None
            else:
                dp.zero_grad()
            for micro in range(accumulate):
                x = torch.randn(16, 64, generator=g).to(device)
                if micro < accumulate - 1:
                    with dp.no_sync():
                        model(x).square().mean().backward()
                else:
                    model(x).square().mean().backward()
            res = dp.sync_gradients()
            assert res.ok and res.world_size == 2
            out.append(_grads(model))
            with torch.no_grad():
                for p in model.parameters():
                    if p.grad is not None:
                        p -= 0.01 * p.grad
        if overlap:
            dp.close()
        return out

    with local_master() as addr:
        return run_threaded_peers(2, fn, address=addr, timeout=120)


def _check(device, **kw):
    ref = _run(device, overlap=False, **kw)
    got = _run(device, overlap=True, **kw)
    for r in range(2):
        for step, (gr, gg) in enumerate(zip(ref[r], got[r])):
            assert gr.keys() == gg.keys()
            for k in gr:
                torch.testing.assert_close(gg[k], gr[k], rtol=0, atol=0, msg=f"rank {r} step {step} {k}")
    # both peers hold the same averaged gradients
    for k in ref[0][0]:
        assert torch.equal(got[0][-1][k], got[1][-1][k])


def test_overlap_matches_sync_path():
    _check("cpu")


def test_overlap_no_sync_accumulation():
    _check("cpu", accumulate=3)


def test_overlap_grad_set_to_none():
    _check("cpu", set_to_none=True, steps=2)


def test_overlap_bucket_plan_covers_every_gradient():
    torch.manual_seed(0)
    model = Net()

    class _Comm:  # bucket planning only
        pass

    dp = DataParallel(model, _Comm(), bucket_bytes=70_000, overlap=True)
    try:
        total = sum(v.numel() for v in dp._bucket_views)
        assert total == sum(p.numel() for p in model.parameters())
        # buckets are cut from the end: the first bucket holds the last layer (first gradients of backward)
        assert any(p is model.c.weight for p in dp._bucket_of if 0 in dp._bucket_of[p])
        assert len(dp._bucket_of[model.b.weight]) >= 2  # spans buckets
    finally:
        dp.close()


@pytest.mark.gpu
def test_overlap_matches_sync_path_gpu():
    _check("cuda:0")
