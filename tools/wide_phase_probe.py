"""Debug builds only (-DTGSIM_PHASE_PROF, TGSIM_LIB=<that .so>): config-2 all-to-all rounds (bench.py
a2a), then the phase times of the last k_shape_seq_wide launch per block (tgsim_debug_wide_phases):
sort, K (due records), copies drawn, decided, appended, tail - medians in microseconds."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
from testground_amd import _abi as A
from testground_amd.sim import Simulator

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 12
hip = A.bind(os.environ["TGSIM_LIB"], "tgsim_", "hip")
sim = Simulator(bench.a2a_config(n), binding=hip)
sim.set_shapes(np.arange(n), bench.a2a_shapes(n))
sim.profile(["k_shape_seq_wide"])
for r in range(rounds):
    sim.enqueue(*bench.a2a_round(n, r))
    sim.advance((r + 1) * bench.A2A_ROUND_NS)
ms, cnt = sim.profile_read()["k_shape_seq_wide"]
print(f"k_shape_seq_wide: {cnt} launches, {ms / max(cnt, 1) * 1e3:.1f} us average (HIP events)")
buf = np.zeros((4096, 12), np.uint64)
assert hip.cdll.tgsim_debug_wide_phases(buf.ctypes.data_as(ctypes.c_void_p)) == 0
a = buf[: min(n, 4096)].astype(np.int64)
a = a[a[:, 6] > 0]
d = np.diff(a[:, :7], axis=1) / 100.0  # s_memrealtime ticks / 100 (us if it runs at 100 MHz)
names = ["sort", "K", "draw", "decide", "append", "tail"]
print("blocks", len(a), "block span (us) median", np.median((a[:, 6] - a[:, 0]) / 100.0),
      "launch span (us)", (a[:, 6].max() - a[:, 0].min()) / 100.0)
for k, nm in enumerate(names):
    print(f"{nm:7s} median {np.median(d[:, k]):7.2f} us   p90 {np.percentile(d[:, k], 90):7.2f}")
# inside the sort phase: loads (0 -> 7), block min/max (7 -> 8), bitonic (8 -> 9), permutation (9 -> 1)
for nm, x, y in (("loads", 0, 7), ("minmax", 7, 8), ("bitonic", 8, 9), ("perm", 9, 1)):
    v = (a[:, y] - a[:, x]) / 100.0
    print(f"  {nm:7s} median {np.median(v):7.2f} us")
sim.close()
