"""Debug builds only (-DTGSIM_PHASE_PROF, TGSIM_LIB=<that .so>): config-2 all-to-all rounds (bench.py
a2a), then the per-sender phase cycles of the last k_shape_seq launch (tgsim_debug_seq_phases)."""
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
for r in range(rounds):
    sim.enqueue(*bench.a2a_round(n, r))
    sim.advance((r + 1) * bench.A2A_ROUND_NS)
buf = np.zeros((1024, 8), np.uint64)
assert hip.cdll.tgsim_debug_seq_phases(buf.ctypes.data_as(ctypes.c_void_p)) == 0
a = buf[: min(n, 1024)].astype(np.int64)
names = ["K setup", "loads+philox", "decide", "queue", "append"]
print("chunks per sender (median):", np.median(a[:, 5]))
for k, nm in enumerate(names):
    print(f"{nm:14s} cycles median {np.median(a[:, k]):10.0f}  per chunk {np.median(a[:, k] / np.maximum(a[:, 5], 1)):8.0f}")
print("total cycles median", np.median(a[:, :5].sum(1)))
sim.close()
