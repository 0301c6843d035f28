"""Direct access to the HIP/CDNA4 kernels (and their bit-exact host twins) of pccl-amd."""
from .kernels import (WIRE_DTYPE, bench_kernel, crc32c, crc32c_has_hw, dequant_reduce, fill_test_pattern,
                      finalize_avg, hip_device_count, multi_gather, multi_reduce, outer_sgd, pseudo_grad, quantize, reduce_,
                      simplehash)

__all__ = ["WIRE_DTYPE", "bench_kernel", "crc32c", "crc32c_has_hw", "dequant_reduce", "fill_test_pattern",
           "finalize_avg", "hip_device_count", "multi_gather", "multi_reduce", "outer_sgd", "pseudo_grad", "quantize",
           "reduce_", "simplehash"]
