// fsx_bins.h — launcher of the light-bin tail (fsx_bins.hip, DESIGN.md §3 "Light bins").
#pragma once
#include "fsx_internal.h"

namespace fsx {

// Tables of 2^17..2^21 slots: the light entries leave sort pass 1 ordered by the low
// id_bits - 6 bits of their slot, 64 slots per bin.
constexpr uint32_t kBinSlotBits = 6;
constexpr uint32_t kBinMinIdBits = 17, kBinMaxIdBits = 21;

struct BinTail {
    const uint64_t *S;        // light sort words after sort pass 1, [0, n_light)
    const uint64_t *pay;      // their payload words (when bs->pay_ok)
    const uint64_t *ts;       // arrival timestamps / lengths (gathers when !pay_ok, ports)
    const uint32_t *len;
    PacketIn in;
    BatchState *bs;
    TableState *tstate;
    uint32_t *bin_start;      // nbins + 1
    uint64_t *bin_mask;       // nbins: the slots of each bin seen in the batch
    uint32_t *bin_row;        // nbins: first row of each bin
    uint32_t *bin_order;      // nbins: the bins in processing order (multi-chunk bins first)
    void *stage;              // per table slot: FlowAcc of the batch's sums (row mode)
    void *sacc;               // accumulate mode: SlotAcc per slot (else null)
    uint32_t epoch;
    uint8_t *verdict;
    Slot *table;
    Limits lim;
    uint32_t binbits;         // id bits - kBinSlotBits
};

// Light tail of one batch on st: bin bounds, per-bin walk + flow sums + verdicts, row
// numbering (bs->nseg = light sources), and with fq (row mode, fq->sacc null) the rows.
hipError_t launch_bins(const BinTail &A, uint32_t n, const FlowRequest *fq, uint32_t salt, hipStream_t st,
                       const Marker &mark);
size_t bin_stage_bytes(uint64_t slots);

}  // namespace fsx
