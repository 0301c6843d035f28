"""Thin wrappers over the ``pcclx*`` kernel entry points of libpccl.so.

Each op runs either the HIP kernel (tensor on a GPU) or the host SIMD twin (CPU tensor); both produce identical bytes.
On a GPU box these calls fail loudly if the HIP plugin is missing instead of silently falling back to the host path.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch

from .._native import C

# torch dtype -> CCoIP wire dtype code (pccl::DType)
WIRE_DTYPE = {torch.uint8: 0, torch.int8: 1, torch.int16: 4, torch.int32: 5, torch.int64: 7, torch.float16: 8,
              torch.bfloat16: 9, torch.float32: 10, torch.float64: 11}
for _name, _code in (("uint16", 2), ("uint32", 3), ("uint64", 6), ("float8_e4m3fn", 12), ("float8_e5m2", 13)):
    if hasattr(torch, _name):
        WIRE_DTYPE[getattr(torch, _name)] = _code

OPS = {"set": 0, "sum": 1, "avg": 2, "prod": 3, "max": 4, "min": 5}
ALGOS = {"none": 0, "min_max": 1, "zero_point_scale": 2}


def hip_device_count() -> int:
    return int(C.pcclxHipDeviceCount())


def _on_device(t: torch.Tensor) -> int:
    if t.device.type == "cuda":
        if hip_device_count() == 0:
            raise RuntimeError("pccl-amd HIP backend (libpccl_hip.so) is not loaded but a GPU tensor was passed")
        torch.cuda.current_stream(t.device).synchronize()
        return 1
    return 0


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def simplehash(t: torch.Tensor) -> int:
    assert t.is_contiguous()
    return int(C.pcclxSimpleHash(t.data_ptr(), t.numel() * t.element_size(), _on_device(t)))


def crc32c(t: torch.Tensor, force_software: bool = False, single_chain: bool = False) -> int:
    """CRC-32C (Castagnoli) of a contiguous tensor: host SSE4.2 (3 interleaved chains; ``single_chain`` selects the
    one-chain variant) or table path (``force_software``), or the HIP kernel for GPU tensors."""
    assert t.is_contiguous()
    if t.device.type != "cpu":
        _on_device(t)
    mode = 1 if force_software else (2 if single_chain else 0)
    return int(C.pcclxCrc32c(t.data_ptr(), t.numel() * t.element_size(), mode))


def crc32c_has_hw() -> bool:
    return bool(C.pcclxCrc32cHasHw())


def fill_test_pattern(t: torch.Tensor):
    """Reference test pattern (random_init_kernel<<<8,256>>>) on a GPU uint8/uint64 buffer."""
    assert t.device.type == "cuda"
    _check(C.pcclxFillTestPattern(t.data_ptr(), t.numel() * t.element_size() // 8), "fill_test_pattern")


def reduce_(dst: torch.Tensor, src: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """dst = dst (op) src in place, with the library's exact accumulation/rounding rules."""
    assert dst.dtype == src.dtype and dst.numel() == src.numel() and dst.device == src.device
    _check(C.pcclxReduce(dst.data_ptr(), src.data_ptr(), dst.numel(), WIRE_DTYPE[dst.dtype], OPS[op], _on_device(dst)),
           "reduce")
    return dst


def finalize_avg(dst: torch.Tensor, world_size: int) -> torch.Tensor:
    _check(C.pcclxFinalizeAvg(dst.data_ptr(), dst.numel(), WIRE_DTYPE[dst.dtype], world_size, _on_device(dst)),
           "finalize_avg")
    return dst


def quantize(src: torch.Tensor, qdtype: torch.dtype, algo: str = "min_max") -> Tuple[torch.Tensor, List[float]]:
    """Quantizes src -> (q, meta) where meta = [min, max, zero_point, scale]."""
    out = torch.empty(src.shape, dtype=qdtype, device=src.device)
    meta = (ctypes.c_double * 4)()
    _check(C.pcclxQuantize(out.data_ptr(), src.data_ptr(), src.numel(), WIRE_DTYPE[src.dtype], WIRE_DTYPE[qdtype],
                           ALGOS[algo], _on_device(src), meta), "quantize")
    return out, list(meta)


def quantize_setback(src: torch.Tensor, qdtype: torch.dtype, algo: str = "min_max") -> Tuple[torch.Tensor, List[float]]:
    """GPU only: quantizes ``src`` and overwrites it with its de-quantized value D(Q(src)) in one kernel pass (the
    quantized ring's owner parity step); returns (q, meta) like ``quantize``."""
    out = torch.empty(src.shape, dtype=qdtype, device=src.device)
    meta = (ctypes.c_double * 4)()
    _check(C.pcclxQuantizeSetback(out.data_ptr(), src.data_ptr(), src.numel(), WIRE_DTYPE[src.dtype],
                                  WIRE_DTYPE[qdtype], ALGOS[algo], meta), "quantize_setback")
    return out, list(meta)


def dequant_reduce(dst: torch.Tensor, q: torch.Tensor, meta: Sequence[float], algo: str = "min_max",
                   op: str = "sum") -> torch.Tensor:
    m = (ctypes.c_double * 4)(*meta)
    _check(C.pcclxDequantReduce(dst.data_ptr(), q.data_ptr(), dst.numel(), WIRE_DTYPE[dst.dtype], WIRE_DTYPE[q.dtype],
                                ALGOS[algo], OPS[op], m, _on_device(dst)), "dequant_reduce")
    return dst


def dequant_reduce_minmax(dst: torch.Tensor, q: torch.Tensor, meta: Sequence[float], algo: str = "min_max",
                          op: str = "sum", pieces: int = 1) -> Tuple[torch.Tensor, List[float]]:
    """``dequant_reduce`` on the GPU in ``pieces`` launches whose kernels also emit per-workgroup (min, max) partials
    of the values they store, folded into [min, max] of the result (the quantized device ring's next-step min / max
    without a second pass; GPU only)."""
    m = (ctypes.c_double * 4)(*meta)
    out = (ctypes.c_double * 2)()
    _check(C.pcclxDequantReduceMinmax(dst.data_ptr(), q.data_ptr(), dst.numel(), WIRE_DTYPE[dst.dtype],
                                      WIRE_DTYPE[q.dtype], ALGOS[algo], OPS[op], m, pieces, out),
           "dequant_reduce_minmax")
    return dst, [out[0], out[1]]


def quant_minmax_stats() -> dict:
    """Quantized device ring, this process since start: payloads whose min / max was folded from the previous step's
    fused de-quantize partials (``folds``) vs separate min / max passes over the payload (``passes``)."""
    out = (ctypes.c_uint64 * 2)()
    C.pcclxQuantStats(out)
    return {"folds": int(out[0]), "passes": int(out[1])}


def multi_reduce(srcs: Sequence[torch.Tensor], op: str = "sum", out: Optional[torch.Tensor] = None,
                 out2: Optional[torch.Tensor] = None, outs: Sequence[torch.Tensor] = ()) -> torch.Tensor:
    """out = op(srcs[0], ..., srcs[n-1]) in fixed order, also stored to out2 and every tensor of ``outs`` (the xGMI
    one-shot reduce + broadcast kernel; GPU only)."""
    s0 = srcs[0]
    out = torch.empty_like(s0) if out is None else out
    _on_device(s0)
    dsts = [out] + ([out2] if out2 is not None else []) + list(outs)
    for d in dsts:
        if d.numel() != s0.numel() or d.dtype != s0.dtype:
            raise ValueError("multi_reduce: every output must match the sources' shape and dtype")
    arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    darr = (ctypes.c_void_p * len(dsts))(*[d.data_ptr() for d in dsts])
    _check(C.pcclxMultiReduce(darr, len(dsts), arr, len(srcs), s0.numel(), WIRE_DTYPE[s0.dtype], OPS[op]),
           "multi_reduce")
    return out


def multi_gather(dst: torch.Tensor, srcs: Sequence[torch.Tensor], offsets: Sequence[int], skip: int = -1):
    """dst[offsets[k] : offsets[k] + srcs[k].numel()] = srcs[k] for k != skip (the xGMI all-gather kernel)."""
    _on_device(dst)
    arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    offs = (ctypes.c_size_t * len(srcs))(*offsets)
    cnts = (ctypes.c_size_t * len(srcs))(*[s.numel() for s in srcs])
    _check(C.pcclxMultiGather(dst.data_ptr(), arr, offs, cnts, len(srcs), skip, WIRE_DTYPE[dst.dtype]),
           "multi_gather")
    return dst


def bench_kernel(which: str, dst: torch.Tensor, src: torch.Tensor, n: int = 1, iters: int = 20) -> float:
    """Average microseconds per launch of a device kernel ('reduce', 'hash', 'multi_reduce', 'quantize', 'crc32c')."""
    w = {"reduce": 0, "hash": 1, "multi_reduce": 2, "quantize": 3, "crc32c": 4}[which]
    _on_device(src)
    return float(C.pcclxBenchKernel(w, dst.data_ptr(), src.data_ptr(), src.numel(), WIRE_DTYPE[src.dtype], n, iters))


def _local_code(t: torch.Tensor) -> int:
    if t.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        raise TypeError(f"DiLoCo local parameters must be fp32/bf16/fp16, got {t.dtype}")
    return WIRE_DTYPE[t.dtype]


def pseudo_grad(pg: torch.Tensor, outer: torch.Tensor, local: torch.Tensor) -> torch.Tensor:
    """pg = outer - local (fp32 outer/pg; local fp32/bf16/fp16), fused HIP kernel on GPU tensors."""
    assert pg.dtype == outer.dtype == torch.float32 and pg.numel() == outer.numel() == local.numel()
    assert pg.is_contiguous() and outer.is_contiguous() and local.is_contiguous()
    _check(C.pcclxPseudoGrad(pg.data_ptr(), outer.data_ptr(), local.data_ptr(), pg.numel(), _local_code(local),
                             _on_device(pg)), "pseudo_grad")
    return pg


def outer_sgd(outer: torch.Tensor, momentum_buf: torch.Tensor, pg: torch.Tensor, local: torch.Tensor, *, lr: float,
              momentum: float = 0.0, dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
              first: bool = False) -> None:
    """One fused pass: SGD(+momentum/nesterov) update of ``outer`` with gradient ``pg``, then local = cast(outer)."""
    for t in (outer, momentum_buf, pg):
        assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == local.numel()
    assert local.is_contiguous()
    _check(C.pcclxOuterSgd(outer.data_ptr(), momentum_buf.data_ptr(), pg.data_ptr(), local.data_ptr(), outer.numel(),
                           _local_code(local), lr, momentum, dampening, weight_decay, int(nesterov), int(first),
                           _on_device(outer)), "outer_sgd")
