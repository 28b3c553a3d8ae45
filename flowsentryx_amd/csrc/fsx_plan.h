// The radix sort's digit plan (host code): which passes a batch's sort takes and the bit
// range of each pass's digit. Shared by launch_verdict_pipeline (fsx_device.hip) and the CPU
// unit test tests/csrc/sort_plan.cpp, which checks every id width and mode against the
// invariants the kernels assume (DESIGN.md §3 "Heavy-source sort", "Wider ids", "Two 9-bit
// light passes").
//
// Sort word: bucket | slot id (idbits, from bit kPlanIdShift) | arrival index (31 bits).
//  * plain: ceil(idbits / 8) LSD passes of equal digits of at most 8 bits (21 bits: 3 x 7);
//    25- / 26-bit ids: 8 + 8 + 9 / 8 + 9 + 9 (plain9), the later passes' digit bases from the
//    tile scan since k_parse counts 8-bit digits only;
//  * heavy-source sort (ids of 17..25 bits): pass 0 on the 8-bit bucket at bit 56 (a 7-bit
//    light digit, or 128 + heavy index), then the light passes over the remaining id bits in
//    equal digits: 8-bit ones, or two 9-bit ones (wide9) for the 17 / 18 bits of 24- / 25-bit
//    ids; an even pass count only with the fixed window's heavy lists.
#pragma once
#include <algorithm>
#include <cstdint>

namespace fsx {

constexpr uint32_t kPlanIdShift = 31;   // the slot id's bit in the sort word (kIdShift)

struct SortPlanIn {
    uint32_t idbits = 0;     // log2(slots); 32 for the home-ordered key hashes
    bool onesweep = false, full_digits = false, no_heavy = false, admit = false;
    bool lists_any = false;  // a limiter batch with verdicts (heavy lists possible)
    bool lists_ok = false;   // ... under the fixed window (an even pass count allowed)
    bool light6 = false;     // A/B: three 6-bit light passes instead of two 9-bit ones
    bool plain4 = false;     // A/B: four plain passes for 25- / 26-bit ids
};

struct SortPlan {
    int npass = 1;
    bool heavy_sort = false, wide9 = false, plain9 = false;
    uint32_t bshift = 0, lbits = 0, hrest = 0;
    uint32_t shift[4] = {0, 0, 0, 0}, mask[4] = {0, 0, 0, 0};
    uint32_t light_b = 0;    // heavy sort: pass-0 buckets below it are light
    uint32_t nhist = 1;      // digits k_parse counts (its counters are 256 wide)
    bool tile_bases = false; // passes >= 1 take their digit bases from the tile scan
};

inline SortPlan make_sort_plan(const SortPlanIn &q) {
    SortPlan p;
    const uint32_t idbits = q.idbits;
    p.npass = std::max(1, (int)((idbits + 7) / 8));
    const uint32_t dbits = q.full_digits ? 8u : std::max<uint32_t>(1, (idbits + p.npass - 1) / p.npass);
    const uint32_t dmask = (1u << dbits) - 1u;
    p.bshift = std::max<uint32_t>(56, kPlanIdShift + idbits);
    p.lbits = 63 - p.bshift;                                  // light digit bits of the bucket
    p.hrest = idbits > p.lbits ? idbits - p.lbits : 0;
    p.wide9 = q.lists_any && !q.light6 && p.hrest > 16 && p.hrest <= 18;
    const int hpass = 1 + (p.wide9 ? 2 : (int)((p.hrest + 7) / 8));   // pass 0 + the light passes
    p.heavy_sort = !q.admit && !q.onesweep && !q.full_digits && !q.no_heavy && idbits <= 25 && p.npass >= 3 &&
                   (hpass == 3 || (hpass == 4 && q.lists_ok));
    if (p.heavy_sort) p.npass = hpass;
    p.plain9 = !p.heavy_sort && !q.onesweep && !q.full_digits && !q.admit && !q.plain4 && p.npass == 4 &&
               idbits >= 25 && idbits <= 26;
    if (p.plain9) p.npass = 3;
    p.tile_bases = (p.heavy_sort && p.wide9) || p.plain9;
    p.nhist = p.tile_bases ? 1u : (uint32_t)p.npass;
    if (p.heavy_sort) {
        p.light_b = 1u << p.lbits;
        p.shift[0] = p.bshift;
        p.mask[0] = (1u << (64 - p.bshift)) - 1u;
        const uint32_t lp = (uint32_t)hpass - 1, w = (p.hrest + lp - 1) / lp;
        for (uint32_t k = 1; k <= lp; ++k) {
            const uint32_t lo = (k - 1) * w, wb = std::min(w, p.hrest - lo);
            p.shift[k] = kPlanIdShift + p.lbits + lo;
            p.mask[k] = (1u << wb) - 1u;
        }
    } else if (p.plain9) {
        const uint32_t w1 = idbits - 17;   // 8 (25-bit ids) or 9 (26-bit ids)
        p.shift[0] = kPlanIdShift;          p.mask[0] = 255u;
        p.shift[1] = kPlanIdShift + 8;      p.mask[1] = (1u << w1) - 1u;
        p.shift[2] = kPlanIdShift + 8 + w1; p.mask[2] = 511u;
        p.shift[3] = kPlanIdShift + 8 + w1 + 9;   // (no fourth pass)
    } else {
        for (int k = 0; k < 4; ++k) { p.shift[k] = kPlanIdShift + dbits * (uint32_t)k; p.mask[k] = dmask; }
    }
    return p;
}

}  // namespace fsx
