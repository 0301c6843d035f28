"""Test helpers shared by CPU and GPU tests."""
import numpy as np


def lcg_bytes(n: int, seed: int = 42) -> np.ndarray:
    """Byte stream of the reference's hash-test LCG (seed = 1664525*seed + 1013904223; byte = seed % 256),
    `/root/reference/ccoip/tests/unit_tests/simple_hash/simplehash_cpu_test_no_cuda.cpp:10-15`, vectorised in
    blocks of 2^16 steps with the composed affine map."""
    a, c, blk = 1664525, 1013904223, 1 << 16
    first = np.empty(blk, dtype=np.uint64)
    s = seed
    for i in range(blk):
        s = (a * s + c) & 0xFFFFFFFF
        first[i] = s
    big_a, big_c = 1, 0
    for _ in range(blk):
        big_a, big_c = (a * big_a) & 0xFFFFFFFF, (a * big_c + c) & 0xFFFFFFFF
    nblk = (n + blk - 1) // blk
    out = np.empty(nblk * blk, dtype=np.uint8)
    cur = first
    for b in range(nblk):
        out[b * blk:(b + 1) * blk] = (cur & 0xFF).astype(np.uint8)
        cur = (np.uint64(big_a) * cur + np.uint64(big_c)) & np.uint64(0xFFFFFFFF)
    return out[:n].copy()
