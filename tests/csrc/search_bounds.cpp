// Host harness for fsx_search.h (tests/test_search_bounds.py): the heavy rank view's 64-ary
// search simulated lane by lane over prefix rows — valid rows (non-decreasing, pre(0) = 0) must
// give the largest tile with pre(t) <= r in at most ceil(log64(ntiles)) + 1 rounds; corrupted
// rows must end (bounded rounds, lo inside [0, ntiles)) and report the violation when the
// ballot comes back empty. Prints "ok <cases>" or the first failure.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fsx_search.h"

using fsx::ary64_step;
using fsx::ary64_width;

struct Res { uint32_t t, rounds; bool violated; };

static Res search(const std::vector<uint32_t> &pre, uint32_t r) {
    const uint32_t ntiles = (uint32_t)pre.size();
    uint32_t lo = 0, hi = ntiles, rounds = 0;
    bool violated = false;
    while (hi - lo > 1) {
        const uint32_t step = ary64_width(lo, hi);
        uint64_t m = 0;
        for (uint32_t lane = 0; lane < 64; ++lane) {
            const uint64_t q = (uint64_t)lo + (uint64_t)lane * step;
            if (q < hi && pre[q] <= r) m |= 1ull << lane;
        }
        if (!ary64_step(lo, hi, step, m)) violated = true;
        if (++rounds > 64) break;   // (a hang in the unguarded version)
    }
    return Res{lo, rounds, violated};
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t)(rng >> 16);
}

int main() {
    uint32_t cases = 0;
    const uint32_t sizes[] = {1, 2, 63, 64, 65, 4095, 4096, 4097, 16384, 70000};
    for (uint32_t ntiles : sizes) {
        uint32_t max_rounds = 1;
        for (uint64_t s = 1; s < ntiles; s *= 64) ++max_rounds;
        for (int trial = 0; trial < 20; ++trial) {
            // valid: per-tile counts >= 0, pre(0) = 0
            std::vector<uint32_t> pre(ntiles);
            uint32_t acc = 0;
            for (uint32_t t = 0; t < ntiles; ++t) {
                pre[t] = acc;
                acc += (trial & 1) ? rnd() % 3 : rnd() % 200;
            }
            const uint32_t cnt = acc ? acc : 1;
            for (int k = 0; k < 50; ++k) {
                const uint32_t r = rnd() % cnt;
                const Res a = search(pre, r);
                uint32_t want = 0;
                for (uint32_t t = 0; t < ntiles; ++t)
                    if (pre[t] <= r) want = t;
                if (a.violated || a.t != want || a.rounds > max_rounds) {
                    printf("FAIL valid ntiles=%u r=%u got t=%u rounds=%u viol=%d want %u\n", ntiles, r, a.t,
                           a.rounds, (int)a.violated, want);
                    return 1;
                }
                ++cases;
            }
            // corrupted: garbage rows (the aliasing bug wrote other digits' offsets), and rows
            // with every entry past the count
            std::vector<uint32_t> bad(ntiles);
            for (uint32_t t = 0; t < ntiles; ++t) bad[t] = (trial & 2) ? cnt + 7 : rnd();
            for (int k = 0; k < 50; ++k) {
                const uint32_t r = rnd() % cnt;
                const Res a = search(bad, r);
                if (a.t >= ntiles || a.rounds > max_rounds) {
                    printf("FAIL corrupt ntiles=%u r=%u got t=%u rounds=%u\n", ntiles, r, a.t, a.rounds);
                    return 1;
                }
                if (ntiles > 1 && bad[0] > r && !a.violated) {
                    printf("FAIL corrupt ntiles=%u r=%u: pre(0) > r not reported\n", ntiles, r);
                    return 1;
                }
                ++cases;
            }
        }
    }
    printf("ok %u\n", cases);
    return 0;
}
