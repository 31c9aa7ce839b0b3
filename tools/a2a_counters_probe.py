import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import bench
from testground_amd.sim import Simulator
n = 1000
sim = Simulator(bench.a2a_config(n))
sim.set_shapes(np.arange(n), bench.a2a_shapes(n))
prev = None
for r in range(14):
    sim.enqueue(*bench.a2a_round(n, r))
    sim.advance((r + 1) * bench.A2A_ROUND_NS)
    d = sim.stats(); d.update(sim.kernel_counters())
    if prev and r >= 8:
        print(r, {k: d[k] - prev[k] for k in ("delivered", "deferred", "wide", "long_emit", "long_tb") if k in d})
    prev = d
sim.close()
