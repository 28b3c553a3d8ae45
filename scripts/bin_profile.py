#!/usr/bin/env python3
"""Summarise the per-bin phase times of a -DFSX_BIN_PROFILE build (FSX_BIN_PROFILE_OUT file):
per batch, the k_bin_tail span, the bin-duration distribution and the slowest bins.
    python3 scripts/bin_profile.py gpurun_out/binprof.bin [nbins]"""
import sys

import numpy as np


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8)
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 15
    for k in range(len(a) // nb):
        r = a[k * nb:(k + 1) * nb]
        r = r[r[:, 2] > 0]
        t0 = r[:, 2].min()
        dur = (r[:, 7] - r[:, 2]) * 10 / 1000.0   # us (100 MHz ticks)
        span = (r[:, 7].max() - t0) * 10 / 1000.0
        ph = r[:, 3:7].astype(np.float64) * 10 / 1000.0
        print(f"batch {k}: {len(r)} bins, span {span:.1f} us, entries {r[:, 1].sum()}, "
              f"dur us p50 {np.percentile(dur, 50):.1f} p90 {np.percentile(dur, 90):.1f} "
              f"p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f}, sum {dur.sum() / 1e3:.1f} ms")
        print("   phase sums ms (count, place, walk, long):", np.round(ph.sum(0) / 1e3, 2))
        big = r[:, 1] > 2048
        print(f"   multi-chunk bins {big.sum()}, their dur sum {dur[big].sum() / 1e3:.2f} ms")
        late = np.argsort(-(r[:, 7]))[:8]
        for i in late:
            print(f"   late: bin {r[i, 0]} entries {r[i, 1]} start {(r[i, 2] - t0) / 100:.1f} us dur {dur[i]:.1f} us "
                  f"phases {np.round(ph[i], 1)}")
        slow = np.argsort(-dur)[:5]
        for i in slow:
            print(f"   slow: bin {r[i, 0]} entries {r[i, 1]} dur {dur[i]:.1f} us phases {np.round(ph[i], 1)}")
        # entries vs duration
        for lo, hi in ((0, 512), (512, 1024), (1024, 2048), (2048, 8192), (8192, 1 << 40)):
            m = (r[:, 1] >= lo) & (r[:, 1] < hi)
            if m.any():
                print(f"   entries [{lo},{hi}): {m.sum()} bins, mean dur {dur[m].mean():.1f} us")


if __name__ == "__main__":
    main()
