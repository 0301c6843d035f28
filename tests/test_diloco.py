"""DiLoCo: fused outer-step kernels (host twin vs torch.optim.SGD) and sync/async DiLoCo over threaded peers."""
import pytest
import torch

import pccl_amd as pccl
from pccl_amd.models.mlp import MLP
from pccl_amd.ops import kernels as K
from pccl_amd.parallel.diloco import AsyncDiLoCo, DiLoCo
from pccl_amd.utils import local_master, run_threaded_peers


def _torch_sgd_reference(outer, grads, lr, momentum, nesterov, wd):
    p = torch.nn.Parameter(outer.clone())
    opt = torch.optim.SGD([p], lr=lr, momentum=momentum, nesterov=nesterov, weight_decay=wd)
    for g in grads:
        p.grad = g.clone()
        opt.step()
    return p.detach()


@pytest.mark.parametrize("local_dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("momentum,nesterov,wd", [(0.0, False, 0.0), (0.9, True, 0.0), (0.9, False, 0.01)])
def test_outer_sgd_matches_torch(local_dtype, momentum, nesterov, wd):
    n = 10_001
    g = torch.Generator().manual_seed(0)
    outer = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * 0.1 for _ in range(3)]
    o, m = outer.clone(), torch.zeros(n)
    local = torch.empty(n, dtype=local_dtype)
    for k, gr in enumerate(grads):
        K.outer_sgd(o, m, gr, local, lr=0.7, momentum=momentum, nesterov=nesterov, weight_decay=wd, first=k == 0)
    ref = _torch_sgd_reference(outer, grads, 0.7, momentum, nesterov, wd)
    torch.testing.assert_close(o, ref, rtol=1e-5, atol=1e-6)
    assert torch.equal(local, o.to(local_dtype))


@pytest.mark.parametrize("local_dtype", [torch.float32, torch.bfloat16])
def test_pseudo_grad(local_dtype):
    outer = torch.randn(4097)
    local = torch.randn(4097).to(local_dtype)
    pg = K.pseudo_grad(torch.empty(4097), outer, local)
    assert torch.equal(pg, outer - local.float())


_BASE = {}


def _make_model(seed, device="cpu"):
    """Identical init on every (threaded) peer: the global RNG is shared between threads, so copy a base state."""
    if seed not in _BASE:
        torch.manual_seed(seed)
        _BASE[seed] = MLP(hidden_sizes=(32,)).state_dict()
    m = MLP(hidden_sizes=(32,))
    m.load_state_dict(_BASE[seed])
    return m.to(device)


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_sync_diloco_two_peers(momentum):
    """After an outer step every peer holds outer = outer0 - lr * avg(outer0 - local_r) (momentum: first step)."""
    world = 2
    outer0 = torch.cat([p.detach().reshape(-1) for p in _make_model(0).parameters()])

    def fn(rank, comm):
        model = _make_model(0)
        d = DiLoCo(model, comm, outer_lr=0.7, outer_momentum=momentum, nesterov=momentum > 0)
        with torch.no_grad():  # "inner steps": a rank-dependent shift
            for p in model.parameters():
                p.add_(0.01 * (rank + 1))
        local = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        res = d.outer_step()
        assert res.ok and res.world_size == 2
        after = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        return local, after, d.outer[0].clone()

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    avg_pg = sum(outer0 - r[0] for r in res) / world
    step = avg_pg + (0.9 * avg_pg if momentum else 0)  # nesterov with m = g on the first step
    expect = outer0 - 0.7 * step
    for local, after, outer in res:
        assert torch.equal(after, res[0][1])
        torch.testing.assert_close(after, expect, rtol=1e-5, atol=1e-6)
        assert torch.equal(outer, after)


def test_async_diloco_two_peers():
    _make_model(0)
    world, rounds = 2, 4

    def fn(rank, comm):
        model = _make_model(0)
        d = AsyncDiLoCo(model, comm, outer_lr=0.5)
        history = []
        for r in range(rounds):
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(0.01 * (rank + 1) * (r + 1))
            d.outer_step()
            history.append(d.outer[0].clone())
        d.close()
        return history

    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr)
    for h0, h1 in zip(res[0], res[1]):
        assert torch.equal(h0, h1)  # outer params identical on both peers after every round
    assert not torch.equal(res[0][1], res[0][0])  # round 0's reduce was applied at the end of round 1


@pytest.mark.gpu
@pytest.mark.parametrize("local_dtype", [torch.float32, torch.bfloat16])
def test_outer_kernels_gpu_match_host(hip, local_dtype):
    n = (1 << 22) + 3
    outer = torch.randn(n)
    mom = torch.randn(n)
    pg = torch.randn(n)
    local = torch.randn(n).to(local_dtype)
    host = [outer.clone(), mom.clone(), pg.clone(), local.clone()]
    dev = [t.to(hip) for t in host]
    K.outer_sgd(*host, lr=0.7, momentum=0.9, nesterov=True, weight_decay=0.01)
    K.outer_sgd(*dev, lr=0.7, momentum=0.9, nesterov=True, weight_decay=0.01)
    for a, b in zip(host, dev):
        assert torch.equal(a, b.cpu())
    K.pseudo_grad(host[2], host[0], host[3])
    K.pseudo_grad(dev[2], dev[0], dev[3])
    assert torch.equal(host[2], dev[2].cpu())


@pytest.mark.gpu
def test_sync_diloco_gpu(hip):
    _make_model(0)  # build the shared init in the main thread

    def fn(rank, comm):
        model = _make_model(0, hip)
        d = DiLoCo(model, comm, outer_lr=0.7, outer_momentum=0.9, nesterov=True)
        for _ in range(3):
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(0.01 * (rank + 1))
            assert d.outer_step().ok
        torch.cuda.synchronize()
        return torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])

    with local_master() as addr:
        res = run_threaded_peers(2, fn, address=addr)
    assert torch.equal(res[0], res[1])
