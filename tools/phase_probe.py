"""Debug builds only (-DTGSIM_PHASE_PROF): runs storm rounds at the bench size (or, with argv[1] ==
'a2a', config 2's all-to-all rounds), then prints the per-phase clock cycles of the last k_tb_bucket /
k_emit_bucket launches and the workgroup timeline."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator, make_shape

MS = 1_000_000
A2A = len(sys.argv) > 1 and sys.argv[1] == 'a2a'
if A2A:
    sys.argv.pop(1)
N = int(sys.argv[1]) if len(sys.argv) > 1 else (1000 if A2A else 100_000)
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
hip = A.bind(os.environ['TGSIM_LIB'], 'tgsim_', 'hip') if os.environ.get('TGSIM_LIB') else A.hip_library()
print('lib', hip.cdll._name)
if A2A:
    import bench
    sim = Simulator(bench.a2a_config(N), binding=hip)
    sim.set_shapes(np.arange(N), bench.a2a_shapes(N))
    for r_ in range(rounds):
        src, dst, seq, size, t = bench.a2a_round(N, r_)
        sim.enqueue(src, dst, seq, size, t)
        sim.advance((r_ + 1) * bench.A2A_ROUND_NS)
    rounds = 0
else:
    sim = Simulator(SimConfig(n_instances=N, seed=4, data_prefix_len=12, max_msgs_per_window=1 << 20,
                              max_records=1 << 23, max_states=1024), binding=hip)
    rng = np.random.default_rng(4)
    lat = rng.integers(20, 101, N) * MS
    for g in range(N):
        sim.set_shape(g, make_shape(latency_ns=int(lat[g]), jitter_ns=5 * MS, bandwidth_bps=10_000_000, loss=0.5))
for r_ in range(rounds):
    sim.gen_storm_round(r_, A.T_NOW, 8, 1024, 10 * MS, r_)
    w = sim.barrier(r_, N, A.T_NOW)
    sim.advance_to_barrier(w, 1 * MS)
sim.delivery_count()
buf = np.zeros((2, 1024, 12), np.uint64)
rc = hip.cdll.tgsim_debug_phases(buf.ctypes.data_as(ctypes.c_void_p))
assert rc == 0, rc
for kid, name in enumerate(["k_tb_bucket", "k_emit_bucket"]):
    a = buf[kid].astype(np.int64)
    g = int(a[0, 11])
    if g == 0:
        print(f"{name}: not launched")
        continue
    a = a[: min(g, 1024)]
    print(f"{name}: grid {g}, items/bucket median {np.median(a[:, 0]):.0f} max {a[:, 0].max()}")
    print("  phase cycles median/p90:", " ".join(f"{np.median(a[:, 1 + i]):.0f}/{np.percentile(a[:, 1 + i], 90):.0f}"
                                                for i in range(8)))
    t0 = a[:, 9].min()
    st = (a[:, 9] - t0) / 100.0
    en = (a[:, 10] - t0) / 100.0
    print(f"  wg start us: p50 {np.median(st):.2f} max {st.max():.2f}; wg dur us p50 {np.median(en - st):.2f} "
          f"max {(en - st).max():.2f}; kernel span us {en.max():.2f}")
    hist = np.histogram(st, bins=8)[0]
    print("  start histogram:", list(hist))
