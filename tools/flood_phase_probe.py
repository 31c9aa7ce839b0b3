"""Debug builds only (-DTGSIM_PHASE_PROF, TGSIM_LIB=testground_amd/libtgsim_phase.so): runs the bench's
1M-instance flood (bench.py main_flood's step, one publication every 4 windows) for a number of
windows, then prints the per-phase clock cycles of the last k_tb_bucket / k_emit_bucket launches."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from testground_amd import _abi as A
from testground_amd import workloads as W
from testground_amd.sim import SimConfig, Simulator

MS = 1_000_000
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
windows = int(sys.argv[2]) if len(sys.argv) > 2 else 120
hip = A.hip_library()
print('lib', hip.cdll._name)
sim = Simulator(SimConfig(n_instances=N, seed=5, data_prefix_len=11, max_msgs_per_window=1 << 23,
                          max_records=1 << 25))
shapes = W.pubsub_shapes(N, 5)
sim.set_shapes(np.arange(N), shapes)
sim.flood_set_graph(*W.random_regular_graph(N, 8, 5), windows // 4 + 4)
for w in range(windows):
    if w % 4 == 0:
        sim.flood_publish(W.publishers(N, 1, w // 4, 5), np.arange(1) + w // 4, sim.now, 512)
    sim.advance(sim.now + 10 * MS, wait=False)
    sim.flood_react(512, count=False)
sim.delivery_count()
buf = np.zeros((2, 1024, 12), np.uint64)
rc = hip.cdll.tgsim_debug_phases(buf.ctypes.data_as(ctypes.c_void_p))
assert rc == 0, rc
for kid, name in enumerate(["k_tb_bucket", "k_emit_bucket"]):
    a = buf[kid].astype(np.int64)
    g = int(a[0, 11])
    a = a[: min(g, 1024)]
    print(f"{name}: grid {g}, items/bucket median {np.median(a[:, 0]):.0f} max {a[:, 0].max()}")
    print("  phase cycles median/p90:", " ".join(f"{np.median(a[:, 1 + i]):.0f}/{np.percentile(a[:, 1 + i], 90):.0f}"
                                                for i in range(8)))
    t0 = a[:, 9].min()
    st = (a[:, 9] - t0) / 100.0
    en = (a[:, 10] - t0) / 100.0
    print(f"  wg start us: p50 {np.median(st):.2f} max {st.max():.2f}; wg dur us p50 {np.median(en - st):.2f} "
          f"max {(en - st).max():.2f}; span of the first 1024 wgs us {en.max():.2f}")
