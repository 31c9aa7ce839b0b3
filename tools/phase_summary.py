"""Summarises the TGSIM_PHASE_PROF printf lines of the fused bucket kernels (debug builds only):
per kernel, the median clock cycles of each phase and the spread of workgroup start/end times."""
import sys
from collections import defaultdict
import numpy as np

rows = defaultdict(list)
for line in open(sys.argv[1]):
    if not line.startswith("PH "):
        continue
    f = line.split()
    rows[f[1]].append([int(x) for x in f[2:]])
for k, v in rows.items():
    a = np.array(v, dtype=np.int64)
    print(f"{k}: {len(a)} samples, nb median {np.median(a[:, 1]):.0f} max {a[:, 1].max()}")
    print("  phase cycles (median / p90):", " ".join(f"{np.median(a[:, 2 + i]):.0f}/{np.percentile(a[:, 2 + i], 90):.0f}" for i in range(8)))
    dur = (a[:, 11] - a[:, 10]) / 100.0  # wall clock 100 MHz -> us
    print(f"  wg duration us median {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f}")
