"""Debug builds only: config 3's splitbrain windows (bench.py's setup), then the phase clocks of the
last one-workgroup inbox sort (whole_sort; build with -DTGSIM_PHASE_PROF -DTGSIM_WHOLE_SORT) or of the
last task-parallel pass (-DTGSIM_PHASE_PROF):
    tools/build_variant.sh phase -DTGSIM_PHASE_PROF [-DTGSIM_WHOLE_SORT]
    TGSIM_LIB=$PWD/testground_amd/libtgsim_phase.so python3 tools/whole_probe.py [n] [windows]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
from testground_amd import _abi as A
from testground_amd.sim import Simulator

hip = A.bind(os.environ['TGSIM_LIB'], 'tgsim_', 'hip')
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
windows = int(sys.argv[2]) if len(sys.argv) > 2 else 12
sim = Simulator(bench.sb_config(n), binding=hip)
bench.sb_setup(sim, n, "accept")
sim.advance(bench.SB_WINDOW_NS)
sim.probe_react()
for w in range(windows):
    sim.advance(bench.SB_WINDOW_NS * (w + 2))
    sim.probe_react()
sim.delivery_count()
print("inbox sizes of the last window: max", int(np.diff(sim.inbox_offsets()).max()))
print("kernel counters", sim.kernel_counters())
buf = np.zeros(8, np.uint64)
rc = getattr(hip.cdll, "tgsim_debug_whole_phases", None)
if rc is not None:
    assert rc(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    n_, bits = int(buf[0]) & 0xFFFFFFFF, int(buf[0]) >> 32
    c = buf[1:7].astype(np.int64)
    d = np.diff(c) / 100.0
    print(f"whole sort: n {n_} key bits {bits}; us: A {d[0]:.2f} B {d[1]:.2f} C {d[2]:.2f} eq {d[3]:.2f} D {d[4]:.2f} "
          f"total {(c[5] - c[0]) / 100.0:.2f}" if c[5] else f"whole sort: n {n_} bits {bits} clocks {c.tolist()}")
tp = np.zeros(4 * 4096 + 64, np.uint64)
assert hip.cdll.tgsim_debug_task_phases(tp.ctypes.data_as(ctypes.c_void_p)) == 0
t = tp[: 4 * 4096].reshape(4096, 4).astype(np.int64)
t = t[t[:, 1] != 0]
if len(t):
    t0 = t[:, 1].min()
    kind = (t[:, 0].astype(np.uint64) >> np.uint64(63)).astype(int)
    for k, name in ((0, "chunk"), (1, "rank")):
        x = t[kind == k]
        if len(x):
            print(f"{name} tasks {len(x)}: claimed {(x[:, 1] - t0).min() / 100:.2f}-{(x[:, 1] - t0).max() / 100:.2f} us, "
                  f"ready by {(x[:, 2] - t0).max() / 100:.2f}, done by {(x[:, 3] - t0).max() / 100:.2f}")
