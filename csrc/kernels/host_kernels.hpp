// Host (CPU) reduce / quantize / hash kernels. These serve host-memory collectives and are the bit-exact reference
// for the HIP kernels (csrc/hip/*.hip), which must produce identical bytes.
#pragma once

#include <cstddef>
#include <cstdint>

#include "../common/types.hpp"
#include "../proto/packets.hpp"
#include "optim_common.hpp"
#include "quant_common.hpp"

namespace pccl::kernels {

// dst[i] = dst[i] (op) src[i] for `count` elements of `t`. op Set copies. Avg accumulates like Sum.
bool host_reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op);
// out = op(a, b), element-wise (out may be a, not b); bit-identical to the scalar definition and to the HIP kernels
// (fp32 math for 16-bit floats, round to nearest even). AVX-512 path for bf16 / fp32 sums (host_reduce uses it).
bool host_reduce3(void *out, const void *a, const void *b, size_t count, DType t, ReduceOp op);

// dst[i] = dst[i] (op) dequant(src_q[i]) — fused de-quantization + accumulation (op Set = plain dequant).
bool host_dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                         const proto::QuantMeta &meta);

// The same with given parameters (make_params of a metadata packet): what the device kernels compute.
bool host_dequant_reduce_params(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                                const QuantParams &p);
bool host_quantize_params(void *dst_q, const void *src, size_t count, DType vtype, DType qtype, const QuantParams &p);

// Computes metadata over src and quantizes into dst_q.
proto::QuantMeta host_quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype, QuantAlgo algo);

// min / max of a chunk as double.
void host_minmax(const void *src, size_t count, DType vtype, double &mn, double &mx);

// AVG finalization: dst[i] /= world_size (integer division for integer types).
bool host_finalize_avg(void *dst, size_t count, DType t, size_t world_size);

// "simplehash": non-associative 32-bit hash whose reduction tree emulates a 960x256 GPU launch with a 32-lane
// shuffle tree (definition: reference ccoip/src/cuda/simplehash_cuda.cu). Requires 16-byte aligned data.
uint32_t simplehash_host(const void *data, size_t n_bytes);

// DiLoCo outer step (optim_common.hpp): pg = outer - local; outer/mom SGD update and local = cast(outer).
// outer, mom, pg are fp32; local is F32 / BF16 / F16.

bool host_pseudo_grad(float *pg, const float *outer, const void *local, size_t count, DType local_t);
bool host_outer_sgd(float *outer, float *mom, const float *pg, void *local, size_t count, DType local_t,
                    const OuterSgdParams &p);

// CRC-32C (Castagnoli). Uses SSE4.2 when available (and not spoofed off), otherwise slicing-by-8 tables.
uint32_t crc32c(const void *data, size_t n_bytes);
uint32_t crc32c_sw(const void *data, size_t n_bytes);
uint32_t crc32c_hw(const void *data, size_t n_bytes);  // one crc32q chain
uint32_t crc32c_hw3(const void *data, size_t n_bytes); // three interleaved chains + table-driven combine (default)
uint32_t crc32c_hw3_clmul(const void *data, size_t n_bytes); // three chains + PCLMUL combine (default on EPYC)
bool crc32c_clmul_ready(); // PCLMUL tier usable (CPU features + fold constants solved and verified)
void crc32c_spoof_no_hw(bool no_hw); // test hook: force the software path
// implementation tier picked by crc32c(): 0 table (slicing-by-8), 1 SSE4.2 (3 chains, table combine),
// 2 SSE4.2 + PCLMUL; crc32c_spoof_tier(t) caps it for tests (-1 restores), like the reference's spoofed features
int crc32c_tier();
void crc32c_spoof_tier(int max_tier);
bool crc32c_has_hw();

// CRC-32C algebra for split computation (HIP kernel partials, hip_hash.hip). A "raw" CRC has no initial value and no
// final inversion; it is linear: raw(A || B) = shift(raw(A), |B|) ^ raw(B), and crc(M) = ~(shift(~0, |M|) ^ raw(M)).
// Polynomials are in the reflected representation (x^0 is the most significant bit).
uint32_t crc32c_raw_update(uint32_t state, const void *data, size_t n_bytes); // continues from `state`
uint32_t crc32c_gf_mul(uint32_t a, uint32_t b);                                // a * b mod P
uint32_t crc32c_x8n(uint64_t n_bytes);                                         // x^(8 n) mod P
inline uint32_t crc32c_shift(uint32_t raw, uint64_t n_bytes) { return crc32c_gf_mul(crc32c_x8n(n_bytes), raw); }
inline uint32_t crc32c_finish(uint32_t raw, uint64_t n_bytes) { return ~(crc32c_shift(0xffffffffu, n_bytes) ^ raw); }
// slicing-by-8 tables: T[k][b] = raw CRC of byte b followed by k zero bytes
const uint32_t (*crc32c_tables())[256];

} // namespace pccl::kernels
