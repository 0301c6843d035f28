"""Host (CPU) reduction / quantization kernels against plain PyTorch fp32 references.

Parity targets: reference reduce table `ccoip/src/cpp/reduce_kernels.cpp`, min-max quantization
`ccoip/src/cpp/quantize.cpp` (our integer min-max rounds to nearest instead of truncating — documented divergence).
"""
import pytest
import torch

from pccl_amd.ops import kernels as K

FLOATS = [torch.float32, torch.float64, torch.bfloat16, torch.float16]
INTS = [torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64]


def _rand(n, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    if dtype.is_floating_point:
        return (torch.randn(n, generator=g) * 4).to(dtype)
    info = torch.iinfo(dtype)
    lo, hi = max(info.min, -1000), min(info.max, 1000)
    return torch.randint(lo, hi, (n,), generator=g, dtype=torch.int64).to(dtype)


def _ref(a, b, op):
    if a.dtype.is_floating_point:
        x, y = a.double() if a.dtype == torch.float64 else a.float(), b.double() if b.dtype == torch.float64 else b.float()
    else:
        x, y = a, b
    r = {"sum": lambda: x + y, "prod": lambda: x * y, "max": lambda: torch.maximum(x, y),
         "min": lambda: torch.minimum(x, y), "set": lambda: y}[op]()
    return r.to(a.dtype)


@pytest.mark.parametrize("dtype", FLOATS + INTS)
@pytest.mark.parametrize("op", ["sum", "prod", "max", "min", "set"])
@pytest.mark.parametrize("n", [1, 17, 4099])
def test_reduce_matches_torch(dtype, op, n):
    a, b = _rand(n, dtype, 1), _rand(n, dtype, 2)
    expect = _ref(a, b, op)
    got = K.reduce_(a.clone(), b, op)
    assert torch.equal(got, expect), (dtype, op)


@pytest.mark.parametrize("dtype", FLOATS + [torch.int32, torch.int64, torch.int16])
@pytest.mark.parametrize("ws", [1, 2, 3, 8])
def test_finalize_avg(dtype, ws):
    x = _rand(1000, dtype, 3)
    got = K.finalize_avg(x.clone(), ws)
    if dtype.is_floating_point:
        acc = x.double() if dtype == torch.float64 else x.float()
        expect = (acc / ws).to(dtype)
    else:
        expect = torch.div(x, ws, rounding_mode="trunc")
    assert torch.equal(got, expect)


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("qdtype,levels", [(torch.uint8, 255), (torch.int8, 255), (torch.uint16, 65535),
                                           (torch.int16, 65535)])
def test_minmax_quant_roundtrip(vdtype, qdtype, levels):
    if not hasattr(torch, "uint16") and qdtype == getattr(torch, "uint16", None):
        pytest.skip("no torch.uint16")
    x = _rand(5000, vdtype, 4)
    q, meta = K.quantize(x, qdtype, "min_max")
    mn, mx = x.double().min().item(), x.double().max().item()
    assert meta[0] == pytest.approx(mn) and meta[1] == pytest.approx(mx)
    out = K.dequant_reduce(torch.zeros_like(x), q, meta, "min_max", "set")
    step = (mx - mn) / levels
    err = (out.double() - x.double()).abs().max().item()
    tol = step / 2 * 1.001 + (x.double().abs().max().item() * 2 ** -7 if vdtype == torch.bfloat16 else 0) + \
        (x.double().abs().max().item() * 2 ** -10 if vdtype == torch.float16 else 0)
    assert err <= tol, (err, step)


def test_minmax_quant_constant_tensor():
    x = torch.full((100,), 3.25)
    q, meta = K.quantize(x, torch.uint8, "min_max")
    out = K.dequant_reduce(torch.zeros_like(x), q, meta, "min_max", "set")
    assert torch.equal(out, x)


@pytest.mark.parametrize("op", ["sum", "max", "min"])
def test_dequant_reduce_accumulates(op):
    x = _rand(3000, torch.float32, 5)
    acc = _rand(3000, torch.float32, 6)
    q, meta = K.quantize(x, torch.uint8, "min_max")
    dq = K.dequant_reduce(torch.zeros_like(x), q, meta, "min_max", "set")
    got = K.dequant_reduce(acc.clone(), q, meta, "min_max", op)
    assert torch.equal(got, _ref(acc, dq, op))


@pytest.mark.parametrize("qdtype", [getattr(torch, "float8_e4m3fn", None), getattr(torch, "float8_e5m2", None)])
def test_fp8_quant_roundtrip(qdtype):
    if qdtype is None:
        pytest.skip("torch has no fp8 dtype")
    x = _rand(4096, torch.float32, 7)
    q, meta = K.quantize(x, qdtype, "min_max")
    out = K.dequant_reduce(torch.zeros_like(x), q, meta, "min_max", "set")
    rel = 2 ** -3 if qdtype == torch.float8_e4m3fn else 2 ** -2
    amax = x.abs().max().item()
    assert ((out - x).abs() <= x.abs() * rel + amax * 2 ** -9).all()


@pytest.mark.parametrize("qdtype", ["uint8", "int8", "uint16", "int16", "uint32", "int32", "uint64", "int64"])
@pytest.mark.parametrize("shift", [0.0, -5.0, 5.0])
def test_zero_point_scale_roundtrip(qdtype, shift):
    """Zero-point-scale to every integer wire type the reference's piquant map accepts (int8 .. uint64,
    /root/reference/ccoip/internal/piquant_utils.hpp:13-38); mostly-negative / mostly-positive data moves the zero
    point to the ends of the range. Wide types are limited by the float math of the formula (scale in float), not by
    the wire range."""
    qt = getattr(torch, qdtype, None)
    if qt is None:
        pytest.skip(f"no torch.{qdtype}")
    x = _rand(4096, torch.float32, 8) + shift
    q, meta = K.quantize(x, qt, "zero_point_scale")
    assert q.dtype == qt
    out = K.dequant_reduce(torch.zeros_like(x), q, meta, "zero_point_scale", "set")
    bits = torch.iinfo(qt).bits
    step = (x.max() - x.min()).item() / (2 ** bits - 1)
    amax = x.abs().max().item()
    assert (out - x).abs().max().item() <= step * 0.51 + amax * 2 ** -22 + 1e-6
