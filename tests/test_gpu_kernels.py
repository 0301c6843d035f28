"""HIP/CDNA4 kernels on an MI355X vs plain PyTorch fp32 references and vs the host twins (bit-exact).

Reference parity: simplehash CUDA == CPU goldens (ccoip/tests/unit_tests/simple_hash/simplehash_cuda_test.cpp),
random_init_kernel golden 1054399963 (simplehash_cpu_test.cu:106).
"""
import numpy as np
import pytest
import torch

from pccl_amd.ops import kernels as K
from tests._util import lcg_bytes
from tests.test_hash import reference_test_pattern
from tests.test_host_kernels import FLOATS, INTS, _rand, _ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,golden", [(154533888, 3391090508), (1, 344386053), (4, 3765247898), (25, 3651434421)])
def test_device_simplehash_goldens(hip, n, golden):
    x = torch.from_numpy(lcg_bytes(n)).to(hip)
    assert K.simplehash(x) == golden


def test_device_test_pattern_golden(hip):
    n = 154533888
    x = torch.empty(n, dtype=torch.uint8, device=hip)
    K.fill_test_pattern(x)
    torch.cuda.synchronize()
    assert torch.equal(x.cpu(), torch.from_numpy(reference_test_pattern(n)))
    assert K.simplehash(x) == 1054399963


@pytest.mark.parametrize("n", [16, 17, 1000, 4096 + 5, (1 << 22) + 9, 960 * 256 * 16 * 3 + 48])
def test_device_hash_equals_host(hip, n):
    x = torch.from_numpy(lcg_bytes(n, seed=n))
    assert K.simplehash(x.to(hip)) == K.simplehash(x)


@pytest.mark.parametrize("n", [1, 15, 16, 16384, 16384 * 5 + 3, (1 << 22) + 77, 154533888])
@pytest.mark.parametrize("offset", [0, 5])
def test_device_crc32c_equals_host(hip, n, offset):
    """HIP CRC-32C (tiled kernel + host fold) == the host SSE4.2 / table implementation, any length and alignment."""
    x = torch.from_numpy(lcg_bytes(n + offset, seed=n % 1000))
    expect = K.crc32c(x[offset:].clone())
    assert K.crc32c(x.to(hip)[offset:]) == expect


@pytest.mark.parametrize("dtype", FLOATS + INTS)
@pytest.mark.parametrize("op", ["sum", "prod", "max", "min", "set"])
@pytest.mark.parametrize("n", [1, 4099, (1 << 20) + 3])
def test_device_reduce_matches_torch(hip, dtype, op, n):
    a, b = _rand(n, dtype, 11), _rand(n, dtype, 12)
    expect = _ref(a, b, op)
    got = K.reduce_(a.to(hip), b.to(hip), op)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), expect)


@pytest.mark.parametrize("dtype", FLOATS + [torch.int32, torch.int64])
def test_device_finalize_avg(hip, dtype):
    x = _rand(100_003, dtype, 13)
    assert torch.equal(K.finalize_avg(x.to(hip), 3).cpu(), K.finalize_avg(x.clone(), 3))


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("qdtype", [torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64,
                                    getattr(torch, "uint16", None), getattr(torch, "uint32", None),
                                    getattr(torch, "uint64", None), getattr(torch, "float8_e4m3fn", None),
                                    getattr(torch, "float8_e5m2", None)])
@pytest.mark.parametrize("algo", ["min_max", "zero_point_scale"])
def test_device_quant_bit_exact_with_host(hip, vdtype, qdtype, algo):
    """HIP quantize / de-quantize-reduce vs the host kernels, bit for bit, for every wire type of both algorithms
    (zero-point-scale: 8- to 64-bit integers, like the reference's piquant map)."""
    if qdtype is None:
        pytest.skip("dtype not in this torch build")
    if algo == "zero_point_scale" and qdtype.is_floating_point:
        pytest.skip("zero-point-scale needs an integer wire type")
    x = _rand((1 << 20) + 7, vdtype, 14)
    qh, mh = K.quantize(x, qdtype, algo)
    qd, md = K.quantize(x.to(hip), qdtype, algo)
    torch.cuda.synchronize()
    assert mh == md
    assert torch.equal(qd.cpu().view(torch.uint8), qh.view(torch.uint8))
    acc = _rand(x.numel(), vdtype, 15)
    rh = K.dequant_reduce(acc.clone(), qh, mh, algo, "sum")
    rd = K.dequant_reduce(acc.to(hip), qd, md, algo, "sum")
    torch.cuda.synchronize()
    assert torch.equal(rd.cpu(), rh)


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("qdtype,algo", [(torch.uint8, "min_max"), (torch.int8, "zero_point_scale"),
                                         (torch.int16, "min_max"), (torch.int64, "zero_point_scale"),
                                         (getattr(torch, "float8_e4m3fn", None), "min_max"),
                                         (getattr(torch, "float8_e5m2", None), "min_max")])
@pytest.mark.parametrize("n", [1, 1000, (1 << 21) + 7])
def test_device_quantize_setback_matches_two_pass(hip, vdtype, qdtype, algo, n):
    """The fused owner-parity kernel (quantize and overwrite the source with D(Q(x)) in one pass, used by the
    quantized ring's all-gather payload) equals quantize followed by a de-quantize (Set) kernel, bit for bit, and its
    quantized bytes equal the plain quantize's."""
    if qdtype is None:
        pytest.skip("no fp8 dtype")
    x = _rand(n, vdtype, 41).to(hip)
    q1, m1 = K.quantize(x, qdtype, algo)
    two = K.dequant_reduce(torch.zeros_like(x), q1, m1, algo, "set")
    y = x.clone()
    q2, m2 = K.quantize_setback(y, qdtype, algo)
    torch.cuda.synchronize()
    assert m1 == m2
    assert torch.equal(q2.cpu().view(torch.uint8), q1.cpu().view(torch.uint8))
    assert torch.equal(y.cpu(), two.cpu())


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("qdtype,algo", [(torch.uint8, "min_max"), (torch.int8, "zero_point_scale"),
                                         (getattr(torch, "float8_e4m3fn", None), "min_max")])
@pytest.mark.parametrize("op", ["sum", "max"])
@pytest.mark.parametrize("n,pieces", [(1, 1), (5000, 3), ((1 << 22) + 7, 7), (3_000_011, 1), ((1 << 25) + 5, 3)])
def test_device_dequant_reduce_fused_minmax(hip, vdtype, qdtype, algo, op, n, pieces):
    """The quantized device ring's de-quantize-reduce kernels also emit per-workgroup (min, max) partials of the
    values they store (several launches per chunk, like the ring's receive ranges), folded by k_minmax_final: the
    stored result equals the plain kernel's bit for bit, and the fold equals torch's min / max of that result."""
    if qdtype is None:
        pytest.skip("no fp8 dtype")
    x = _rand(n, vdtype, 31)
    q, meta = K.quantize(x.to(hip), qdtype, algo)
    acc = _rand(n, vdtype, 32) * 3 - 1
    plain = K.dequant_reduce(acc.to(hip), q, meta, algo, op)
    fused, mm = K.dequant_reduce_minmax(acc.to(hip), q, meta, algo, op, pieces=pieces)
    torch.cuda.synchronize()
    assert torch.equal(fused.cpu(), plain.cpu())
    ref = plain.float()
    assert mm == [float(ref.min()), float(ref.max())]


@pytest.mark.parametrize("n", [1, 1000, (1 << 22) + 3, 300_000_001])
def test_device_minmax_repeated(hip, n):
    """min/max is two launches (k_minmax_partial writes one partial per workgroup, k_minmax_final folds them,
    csrc/hip/kernels.hpp): repeated calls on the same stream (all-negative data, then shifted data, tails, > 1024
    workgroups of tiles) must equal the host."""
    for shift in (-50.0, 3.0, 0.0):
        if n < (1 << 23):
            xd = (_rand(n, torch.float32, 7 + int(shift)) * 4 - 10.0 + shift).bfloat16().to(hip)
        else:
            xd = (torch.arange(n, device=hip, dtype=torch.float32).remainder_(977.0) - 500.0 + shift).bfloat16()
        _, md = K.quantize(xd, torch.uint8, "min_max")
        torch.cuda.synchronize()
        xf = xd.float()
        assert md[0] == float(xf.min()) and md[1] == float(xf.max()), (md, shift)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int32])
@pytest.mark.parametrize("nsrc", [2, 3, 5, 8, 16])
@pytest.mark.parametrize("op", ["sum", "avg", "max"])
def test_multi_reduce(hip, dtype, nsrc, op):
    n = (1 << 18) + 13
    srcs = [_rand(n, dtype, 20 + k) for k in range(nsrc)]
    # the kernel accumulates in the compute type (fp32 for 16-bit floats) in fixed source order, rounds once
    ct = {torch.bfloat16: torch.float32, torch.float16: torch.float32}.get(dtype, dtype)
    acc = srcs[0].to(ct)
    for s in srcs[1:]:
        acc = torch.maximum(acc, s.to(ct)) if op == "max" else acc + s.to(ct)
    if op == "avg":
        acc = acc / nsrc if dtype.is_floating_point else torch.div(acc, nsrc, rounding_mode="trunc")
    ref = acc.to(dtype)
    out2 = torch.empty(n, dtype=dtype, device=hip)
    got = K.multi_reduce([s.to(hip) for s in srcs], op, out2=out2)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), ref)
    assert torch.equal(out2.cpu(), ref)


def test_multi_reduce_more_tiles_than_workgroups(hip):
    """Large shard: more vector tiles than the 512-workgroup budget, so each workgroup walks several tiles (plus a
    partial last tile and a scalar tail)."""
    n = 5_000_000 + 3
    srcs = [_rand(n, torch.bfloat16, 60 + k) for k in range(3)]
    ref = (srcs[0].float() + srcs[1].float() + srcs[2].float()).bfloat16()
    outs = [torch.empty(n, dtype=torch.bfloat16, device=hip)]
    got = K.multi_reduce([s.to(hip) for s in srcs], "sum", outs=outs)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), ref)
    assert torch.equal(outs[0].cpu(), ref)


@pytest.mark.parametrize("ndst", [1, 2, 8, 16])
@pytest.mark.parametrize("misalign", [0, 3])
def test_multi_reduce_broadcast(hip, ndst, misalign):
    """One-shot push kernel: the reduced shard lands in every destination (scalar path when misaligned)."""
    n = (1 << 17) + 5
    srcs = [_rand(n + misalign, torch.bfloat16, 40 + k).to(hip)[misalign:] for k in range(4)]
    acc = srcs[0].cpu().float()
    for s in srcs[1:]:
        acc = acc + s.cpu().float()
    ref = acc.bfloat16()
    outs = [torch.full((n,), 7.0, dtype=torch.bfloat16, device=hip) for _ in range(ndst - 1)]
    got = K.multi_reduce(srcs, "sum", outs=outs)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), ref)
    for o in outs:
        assert torch.equal(o.cpu(), ref)


def test_multi_gather(hip):
    parts = [torch.randn(n, device=hip) for n in (1000, 0, 4099, 17)]
    offs = [0, 1000, 1000, 5099]
    dst = torch.zeros(5116, device=hip)
    K.multi_gather(dst, parts, offs, skip=2)
    torch.cuda.synchronize()
    expect = torch.cat([parts[0], parts[1], torch.zeros(4099, device=hip), parts[3]])
    assert torch.equal(dst, expect)
