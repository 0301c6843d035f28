// simplehash (wave64 emulation of the reference's 32-lane tree) + reference test pattern launchers.
#include <algorithm>

#include "dispatch.hpp"
#include "launchers.hpp"

namespace pccl::hipk {

bool launch_simplehash(const void *dev_ptr, size_t n_bytes, uint32_t *partial, uint32_t *out, hipStream_t st) {
    const size_t n_words = n_bytes / 4;
    const size_t n_vec = n_words / 4;
    size_t grid = (n_vec + 255) / 256;
    if (grid > 960) grid = 960;
    return launch_ok([&] {
        if (grid > 0) {
            const size_t vpb = (n_vec + grid - 1) / grid;
            k_hash_big<><<<static_cast<int>(grid), kBlock, 0, st>>>(static_cast<const uint4 *>(dev_ptr), partial, n_vec, vpb);
        }
        k_hash_final<><<<1, kBlock, 0, st>>>(partial, static_cast<int>(grid), static_cast<const uint8_t *>(dev_ptr), n_bytes, out);
    });
}

bool launch_crc32c(const void *dev_ptr, size_t n_tiles, const void *tables_dev, const uint32_t *levels,
                   uint32_t *partial_dev, size_t max_partials, size_t &grid, size_t &tiles_per_wg, hipStream_t st) {
    if (n_tiles == 0 || max_partials == 0) return false;
    // >= 4 workgroups per CU when there is enough data, at least 4 tiles (64 KiB) per workgroup
    grid = std::min<size_t>(max_partials, std::max<size_t>(1, n_tiles / 4));
    tiles_per_wg = (n_tiles + grid - 1) / grid;
    grid = (n_tiles + tiles_per_wg - 1) / tiles_per_wg;
    CrcLevels lv{};
    for (int k = 0; k < 8; ++k) lv.m[k] = levels[k];
    return launch_ok([&] {
        k_crc32c<><<<static_cast<int>(grid), kBlock, 0, st>>>(static_cast<const uint8_t *>(dev_ptr), n_tiles, tiles_per_wg,
                                                               static_cast<const CrcTables *>(tables_dev), lv, partial_dev);
    });
}

bool launch_test_pattern(void *dev_ptr, size_t n_u64, hipStream_t st) {
    return launch_ok([&] { k_test_pattern<><<<8, 256, 0, st>>>(static_cast<uint64_t *>(dev_ptr), n_u64); });
}

} // namespace pccl::hipk
