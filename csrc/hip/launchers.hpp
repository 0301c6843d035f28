// Host-side launch functions of the HIP kernels, one translation unit per kernel family so that the (heavily
// templated) device code compiles in parallel.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../common/types.hpp"
#include "../kernels/optim_common.hpp"
#include "../kernels/quant_common.hpp"

namespace pccl::hipk {

// hip_reduce.hip
bool launch_reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op, hipStream_t s);
bool launch_reduce_copy(void *dst, const void *src, void *out, size_t count, DType t, ReduceOp op, hipStream_t s);
bool launch_finalize_avg(void *dst, size_t count, DType t, size_t ws, hipStream_t s);
bool launch_copy_bytes(void *dst, const void *src, size_t n, int max_grid, hipStream_t s);

// hip_quant.hip
bool launch_dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                           const kernels::QuantParams &p, hipStream_t s, double *mm = nullptr, int mm_max_blocks = 0,
                           int *mm_blocks = nullptr);
// set_back: also overwrite src with D(Q(src)) (src is written: the caller passes a mutable buffer)
bool launch_quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype,
                     const kernels::QuantParams &p, hipStream_t s, bool set_back = false);
bool launch_minmax(const void *src, size_t count, DType vtype, double *partial, double *out2, hipStream_t st);
bool launch_minmax_fold(const double *partial, int nblocks, size_t count, double *out2, hipStream_t st);

// hip_ipc.hip
bool launch_multi_reduce(void *const *dsts, int ndst, const void *const *srcs, int n, size_t count, DType t,
                         ReduceOp op, hipStream_t s, int max_grid = 0, bool release = false);
bool launch_multi_gather(void *dst, const void *const *srcs, const size_t *offsets, const size_t *counts, int n,
                         int skip, DType t, hipStream_t s, bool release = false);

// hip_optim.hip
bool launch_pseudo_grad(float *pg, const float *outer, const void *local, size_t count, DType lt, hipStream_t s);
bool launch_outer_sgd(float *outer, float *mom, const float *pg, void *local, size_t count, DType lt,
                      const kernels::OuterSgdParams &p, hipStream_t s);

// hip_hash.hip
bool launch_simplehash(const void *dev_ptr, size_t n_bytes, uint32_t *partial_scratch, uint32_t *out, hipStream_t s);
bool launch_test_pattern(void *dev_ptr, size_t n_u64, hipStream_t s);
// tables: 12 x 256 words in device memory (CrcTables layout); returns the grid size / tiles per workgroup used
bool launch_crc32c(const void *dev_ptr, size_t n_tiles, const void *tables_dev, const uint32_t *levels,
                   uint32_t *partial_dev, size_t max_partials, size_t &grid, size_t &tiles_per_wg, hipStream_t s);

} // namespace pccl::hipk
