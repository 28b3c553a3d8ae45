// CPU harness for the sort's digit plan (flowsentryx_amd/csrc/fsx_plan.h, the shipped
// function): every id width 1..32 under every combination of the plan's switches, checked
// against what the kernels assume (tests/test_sort_plan.py):
//  * 1..4 passes; every digit at most 9 bits (512-digit tiles), pass 0's at most 8 (k_parse's
//    per-tile counters are 256 wide), and every digit k_parse counts (nhist) at most 8;
//  * the id digits tile the id exactly: contiguous from bit 31 (the heavy sort: its light
//    digit, bits 31..37, then the light passes from bit 38), no bit outside the id;
//  * the heavy sort's bucket sits above the id (bit 56, 8 bits: 128 light + 128 heavy buckets)
//    and an even pass count only with the fixed window's heavy lists;
//  * digit bases from the tile scan exactly for the 9-bit plans, which then count one digit in
//    k_parse.
#include <cstdio>
#include <cstdlib>

#include "fsx_plan.h"

using fsx::SortPlan;
using fsx::SortPlanIn;

static int fails = 0;
#define CHECK(c, ...)                                                                       \
    do {                                                                                    \
        if (!(c)) {                                                                         \
            if (fails < 20) {                                                               \
                std::printf("FAIL %s: ", #c);                                               \
                std::printf(__VA_ARGS__);                                                   \
                std::printf("\n");                                                          \
            }                                                                               \
            ++fails;                                                                        \
        }                                                                                   \
    } while (0)

static uint32_t width(uint32_t mask) {
    uint32_t w = 0;
    while (mask >> w) ++w;
    return w;
}

int main() {
    long plans = 0, heavy = 0, wide9 = 0, plain9 = 0;
    for (uint32_t idbits = 1; idbits <= 32; ++idbits) {
        for (uint32_t f = 0; f < 256; ++f) {
            SortPlanIn q;
            q.idbits = idbits;
            q.onesweep = f & 1;
            q.full_digits = f & 2;
            q.no_heavy = f & 4;
            q.admit = f & 8;
            q.lists_any = f & 16;
            q.lists_ok = (f & 32) && q.lists_any;   // (the fixed window's lists are lists)
            q.light6 = f & 64;
            q.plain4 = f & 128;
            const SortPlan p = fsx::make_sort_plan(q);
            ++plans;
            heavy += p.heavy_sort;
            wide9 += p.heavy_sort && p.wide9;
            plain9 += p.plain9;
            CHECK(p.npass >= 1 && p.npass <= 4, "idbits %u f %u npass %d", idbits, f, p.npass);
            for (int k = 0; k < p.npass; ++k)
                CHECK(width(p.mask[k]) <= 9 && p.mask[k] == (1u << width(p.mask[k])) - 1u,
                      "idbits %u f %u pass %d mask %x", idbits, f, k, p.mask[k]);
            CHECK(p.mask[0] <= 255u, "idbits %u f %u pass-0 mask %x", idbits, f, p.mask[0]);
            CHECK(p.nhist >= 1 && (int)p.nhist <= p.npass, "idbits %u f %u nhist %u", idbits, f, p.nhist);
            for (uint32_t k = 0; k < p.nhist; ++k)
                CHECK(p.mask[k] <= 255u, "idbits %u f %u counted digit %u mask %x", idbits, f, k, p.mask[k]);
            CHECK(p.tile_bases == ((p.heavy_sort && p.wide9) || p.plain9), "idbits %u f %u tile_bases", idbits, f);
            CHECK(p.tile_bases == (p.nhist == 1 && p.npass > 1 && (p.heavy_sort || p.plain9)),
                  "idbits %u f %u nhist %u tile_bases %d", idbits, f, p.nhist, (int)p.tile_bases);
            if (p.heavy_sort) {
                CHECK(!q.admit && !q.onesweep && !q.full_digits && !q.no_heavy, "idbits %u f %u heavy with a switch off",
                      idbits, f);
                CHECK(idbits >= 17 && idbits <= 25, "idbits %u f %u heavy", idbits, f);
                CHECK(p.bshift == 56 && p.mask[0] == 255u && p.light_b == 128u, "idbits %u f %u bucket", idbits, f);
                CHECK(fsx::kPlanIdShift + idbits <= p.bshift, "idbits %u f %u id under the bucket", idbits, f);
                CHECK((p.npass & 1) || q.lists_ok, "idbits %u f %u even count without the fixed window's lists",
                      idbits, f);
                // the light digit (bits 31..37) then the light passes, contiguous, covering the id
                uint32_t at = fsx::kPlanIdShift + p.lbits;
                for (int k = 1; k < p.npass; ++k) {
                    CHECK(p.shift[k] == at, "idbits %u f %u light pass %d at %u, want %u", idbits, f, k, p.shift[k], at);
                    at += width(p.mask[k]);
                }
                CHECK(at == fsx::kPlanIdShift + idbits, "idbits %u f %u light passes end at %u", idbits, f, at);
                if (p.wide9) CHECK(p.npass == 3 && width(p.mask[1]) == 9, "idbits %u f %u wide9", idbits, f);
            } else {
                CHECK(p.light_b == 0, "idbits %u f %u plain light_b", idbits, f);
                uint32_t at = fsx::kPlanIdShift;
                for (int k = 0; k < p.npass; ++k) {
                    CHECK(p.shift[k] == at, "idbits %u f %u pass %d at %u, want %u", idbits, f, k, p.shift[k], at);
                    at += width(p.mask[k]);
                }
                // every id bit sorted; (full_digits: 8-bit digits may run past the id into bits
                // that are zero)
                CHECK(at >= fsx::kPlanIdShift + idbits, "idbits %u f %u digits end at %u", idbits, f, at);
                CHECK(q.full_digits || at - (fsx::kPlanIdShift + idbits) < (uint32_t)p.npass,
                      "idbits %u f %u digits run %u bits past the id", idbits, f, at - (fsx::kPlanIdShift + idbits));
                CHECK(at <= 64, "idbits %u f %u past the word", idbits, f);
                if (p.plain9) CHECK(p.npass == 3 && (idbits == 25 || idbits == 26) && at == fsx::kPlanIdShift + idbits,
                                    "idbits %u f %u plain9", idbits, f);
            }
        }
    }
    // the product's plans at the BASELINE tables (limiter batches with verdicts)
    auto plan_of = [](uint32_t idbits, bool fixed) {
        SortPlanIn q;
        q.idbits = idbits;
        q.lists_any = true;
        q.lists_ok = fixed;
        return fsx::make_sort_plan(q);
    };
    const SortPlan c2 = plan_of(21, true), c3 = plan_of(23, true), c4 = plan_of(25, true), c4sw = plan_of(25, false);
    CHECK(c2.heavy_sort && c2.npass == 3 && width(c2.mask[1]) == 7 && width(c2.mask[2]) == 7, "config 2 plan");
    CHECK(c3.heavy_sort && c3.npass == 3 && width(c3.mask[1]) == 8 && width(c3.mask[2]) == 8, "config 3 plan");
    CHECK(c4.heavy_sort && c4.wide9 && c4.npass == 3 && width(c4.mask[1]) == 9 && width(c4.mask[2]) == 9,
          "config 4 plan");
    CHECK(c4sw.heavy_sort && c4sw.wide9 && c4sw.npass == 3, "config 4 sliding window / token bucket plan");
    SortPlanIn fo;   // a flow-only batch on a 2^25-slot table: the plain three-pass sort
    fo.idbits = 25;
    const SortPlan f25 = fsx::make_sort_plan(fo);
    CHECK(!f25.heavy_sort && f25.plain9 && f25.npass == 3, "flow-only 25-bit plan");
    SortPlanIn od;   // home-ordered key hashes: four 8-bit passes
    od.idbits = 32;
    od.lists_any = od.lists_ok = true;
    const SortPlan o32 = fsx::make_sort_plan(od);
    CHECK(!o32.heavy_sort && !o32.plain9 && o32.npass == 4 && o32.mask[3] == 255u, "ordered 32-bit plan");
    if (fails) {
        std::printf("%d failures\n", fails);
        return 1;
    }
    std::printf("ok %ld plans (%ld heavy, %ld with 9-bit light passes, %ld plain 3-pass)\n", plans, heavy, wide9,
                plain9);
    return 0;
}
