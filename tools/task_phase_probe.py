"""Debug builds only (-DTGSIM_PHASE_PROF, TGSIM_LIB=<that .so>): config-3 splitbrain windows (bench.py
splitbrain), then the timeline of the last task-parallel long-segment pass (tgsim_debug_task_phases:
the probed target's ~10k-request inbox in the wheel-insert launch): per task its claim, ready (chunk
sorted / its segment's chunks counted) and done times, in microseconds from the first claim."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
from testground_amd import _abi as A
from testground_amd.sim import Simulator

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
windows = int(sys.argv[2]) if len(sys.argv) > 2 else 40
hip = A.bind(os.environ["TGSIM_LIB"], "tgsim_", "hip")
sim = Simulator(bench.sb_config(n), binding=hip)
bench.sb_setup(sim, n, "accept")
for w in range(windows):
    sim.advance((w + 1) * bench.SB_WINDOW_NS)
    sim.probe_react()
raw = np.zeros(4 * 4096 + 8, np.uint64)
assert hip.cdll.tgsim_debug_task_phases(raw.ctypes.data_as(ctypes.c_void_p)) == 0
buf = raw[: 4 * 4096].reshape(4096, 4)
ck = raw[4 * 4096:].astype(np.int64)
live = buf[:, 1] != 0
a = buf[live]
t0 = a[:, 1].min()
us = lambda x: (x.astype(np.int64) - int(t0)) / 100.0  # 100 MHz
rank = (a[:, 0] >> np.uint64(63)) == 1
blk = (a[:, 0] >> np.uint64(32)) & np.uint64(0x7FFFFFFF)
for name, m in (("chunk", ~rank), ("rank", rank)):
    if not m.any():
        continue
    c, r, d = us(a[m, 1]), us(a[m, 2]), us(a[m, 3])
    print(f"{name:5s} tasks {m.sum():4d}  claim {c.min():6.1f}..{c.max():6.1f}  ready {r.min():6.1f}..{r.max():6.1f}"
          f"  done {d.min():6.1f}..{d.max():6.1f}  work median {np.median(d - r):5.1f} us  xcds {np.unique(blk[m] % 8).size}")
# the last chunk task: claimed -> keys loaded -> sorted (ck) -> ready
last = np.argmax(np.where(rank, 0, a[:, 1]))
print(f"last chunk task: keys loaded {(int(ck[0]) - int(a[last, 1])) / 100:.1f} us after its claim, "
      f"sorted {(int(ck[1]) - int(ck[0])) / 100:.1f} us later (clocks of the last chunk sort of any launch)")
if ck[2]:
    print("last 1024-key packed sort: " + ", ".join(f"{n} {(int(ck[i + 1]) - int(ck[i])) / 100:.1f} us" for i, n in
          ((2, "min/max"), (3, "pack"), (4, "network"), (5, "restore"))))
sim.close()
