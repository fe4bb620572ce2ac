"""Summarises a bench.py --join-trace .npz: per-partition phase durations of join_partition (us) and the
occupancy over time (how many partitions are in flight)."""
import sys

import numpy as np

z = np.load(sys.argv[1])
t = z["stamps_us"]
t = t - t[:, 0].min()
ph = np.diff(t, axis=1)
names = ["build", "probe+count", "allocate", "write"]
print(f"partitions {len(t)}  kernel span {t[:, 4].max() - t[:, 0].min():.1f} us")
for i, n in enumerate(names):
    print(f"{n:12s} mean {ph[:, i].mean():7.2f}  p50 {np.median(ph[:, i]):7.2f}  p99 {np.percentile(ph[:, i], 99):7.2f}")
life = t[:, 4] - t[:, 0]
print(f"{'lifetime':12s} mean {life.mean():7.2f}  p50 {np.median(life):7.2f}  p99 {np.percentile(life, 99):7.2f}")
grid = np.linspace(0, t[:, 4].max(), 20)
inflight = [int(((t[:, 0] <= g) & (t[:, 4] > g)).sum()) for g in grid]
print("in flight over time:", inflight)
