// fsx_search.h — one round of the 64-ary search the heavy rank view (fsx_heavy_view.h) runs
// over a heavy source's prefix row of per-tile counts: find the largest tile t in [lo, hi)
// with pre(t) <= r. Lane k of the wave probes q = lo + k * width(lo, hi) (q < hi) and the
// ballot of "pre(q) <= r" picks the sub-range. Host-compilable (tests/test_search_bounds.py
// checks it on valid and corrupted rows with g++).
//
// A valid row has pre(lo) <= r, so lane 0 is always in the ballot. A corrupted row (round 5's
// hang: a pass overwrote the rows, ff010e0) can leave the ballot empty; the unguarded step
// then moved lo below itself and the search never ended. ary64_step ends the search at lo
// instead and reports the violation, which the caller turns into a batch error (-EIO).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define FSX_HD __host__ __device__
#else
#define FSX_HD
#endif

namespace fsx {

FSX_HD inline uint32_t ary64_width(uint32_t lo, uint32_t hi) { return (hi - lo + 63u) / 64u; }

// One round from the ballot m (bit k: lane k's probe has pre(q) <= r). Returns false — and
// narrows to [lo, lo + 1), ending the search — when no lane qualified.
FSX_HD inline bool ary64_step(uint32_t &lo, uint32_t &hi, uint32_t width, uint64_t m) {
    if (m == 0) {
        hi = lo + 1u;
        return false;
    }
    const uint32_t f = 63u - (uint32_t)__builtin_clzll((unsigned long long)m);
    lo += f * width;
    hi = hi < lo + width ? hi : lo + width;
    return true;
}

}  // namespace fsx
