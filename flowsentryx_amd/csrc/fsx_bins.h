// fsx_bins.h — launcher of the bin sort (fsx_bins.hip, DESIGN.md §3 "Bin sort").
#pragma once
#include "fsx_internal.h"

namespace fsx {

// Tables of 2^17..2^23 slots (the heavy-source sort): sort passes 0 and 1 take slot bits
// [8, 15) and [15, id bits), so the light entries leave pass 1 ordered by slot >> 8 — bins
// of 256 consecutive slots, sorted locally by the low 8 bits.
constexpr uint32_t kBinSlotBits = 8;
constexpr uint32_t kBinMinIdBits = 17, kBinMaxIdBits = 23;

// The third sort pass as a per-bin LDS sort (fsx_bins.hip "bin sort"): S / pay (sort pass
// 1's output, [0, n_light)) -> out / pout grouped by source, in arrival order per source.
struct BinSort {
    const uint64_t *S;
    const uint64_t *pay;
    uint64_t *out;
    uint64_t *pout;
    const BatchState *bs;
    uint32_t *bin_start;      // nbins + 1
    uint32_t *bin_order;      // nbins
    uint64_t table_mask;
    // segment heads (else null): flag per output position, heads per kTile tile (and per
    // 1024-position flow sub-tile), zeroed by the caller
    uint8_t *headf;
    uint32_t *tile_cnt;
    uint32_t *sub_cnt;
};
hipError_t launch_bin_sort(const BinSort &A, uint32_t n, hipStream_t st);

}  // namespace fsx
