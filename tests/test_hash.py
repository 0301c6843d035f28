"""simplehash + CRC32C goldens (reference: ccoip/tests/unit_tests/simple_hash/simplehash_cpu_test_no_cuda.cpp:52,90,127,165;
ccoip/tests/unit_tests/crc32/crc32_cpu_test.cpp)."""
import zlib

import numpy as np
import pytest
import torch

from pccl_amd.ops import kernels as K
from tests._util import lcg_bytes


@pytest.mark.parametrize("n,golden", [(154533888, 3391090508), (1, 344386053), (4, 3765247898), (25, 3651434421)])
def test_simplehash_cpu_goldens(n, golden):
    buf = torch.from_numpy(lcg_bytes(n))
    assert K.simplehash(buf) == golden


def test_simplehash_empty_and_deterministic():
    assert K.simplehash(torch.empty(0, dtype=torch.uint8)) == 0
    x = torch.from_numpy(lcg_bytes(1 << 20, seed=7))
    assert K.simplehash(x) == K.simplehash(x.clone())


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 4095, 4096, 1 << 20, (1 << 20) + 3])
def test_simplehash_sensitivity(n):
    x = torch.from_numpy(lcg_bytes(max(n, 1), seed=n + 1))[:n].clone()
    h = K.simplehash(x)
    if n:
        y = x.clone()
        y[n // 2] ^= 1
        assert K.simplehash(y) != h


def _crc32c_bytewise(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def test_crc32c_check_value():
    t = torch.frombuffer(bytearray(b"123456789"), dtype=torch.uint8)
    assert K.crc32c(t) == 0xE3069283
    assert K.crc32c(t, force_software=True) == 0xE3069283


@pytest.mark.parametrize("n", [1, 7, 8, 63, 64, 65, 1000, 4097, 100003, 3 * 8192, 3 * 8192 + 5, 1000003])
def test_crc32c_hw_vs_sw_vs_bytewise(n):
    data = lcg_bytes(n, seed=n)
    t = torch.from_numpy(data)
    sw = K.crc32c(t, force_software=True)
    assert sw == K.crc32c(t)
    assert sw == K.crc32c(t, single_chain=True)
    if n <= 4097:
        assert sw == _crc32c_bytewise(data.tobytes())
    assert sw != zlib.crc32(data.tobytes()) or n == 0  # Castagnoli, not IEEE


def reference_test_pattern(n_bytes: int) -> np.ndarray:
    """Host model of the reference's random_init_kernel<<<8,256>>> (simplehash_cpu_test.cu:17-23)."""
    n = n_bytes // 8
    nt = 2048
    i = np.arange(n, dtype=np.uint64)
    a = (((i % np.uint64(nt)) * np.uint64(nt)) & np.uint64(0xFFFFFFFF)) ^ (i & np.uint64(n))
    return (a * np.uint64(0xAABAABABAB1)).view(np.uint8)


def test_simplehash_test_pattern_golden():
    assert K.simplehash(torch.from_numpy(reference_test_pattern(154533888))) == 1054399963
