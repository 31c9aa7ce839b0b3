"""Quick GPU probe: confirms which library runs, and times storm rounds at the bench size."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from testground_amd import _abi as A
from testground_amd.sim import Simulator, SimConfig, make_shape
from tests import scenarios as S

hip = A.hip_library()
print("hip lib:", hip.version().decode(), hip.cdll._name)
r = S.run_random(hip, 1)
print("random deliveries per window:", [len(x["deliv"]["t_deliver"]) for x in r[:-1]])
MS = 1_000_000
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 30
sim = Simulator(SimConfig(n_instances=N, seed=4, data_prefix_len=12, max_msgs_per_window=1 << 20,
                          max_records=1 << 23, max_states=1024), binding=hip)
rng = np.random.default_rng(4)
lat = rng.integers(20, 101, N) * MS
for g in range(N):
    sim.set_shape(g, make_shape(latency_ns=int(lat[g]), jitter_ns=5 * MS, bandwidth_bps=10_000_000, loss=0.5))
ts = []
tot = 0
for r_ in range(rounds):
    t0 = time.perf_counter()
    now = sim.now
    sim.gen_storm_round(r_, now, 8, 1024, 10 * MS, r_)
    w = sim.barrier(r_, N, now)
    sim.advance_to_barrier(w, 1 * MS)
    n = sim.delivery_count()
    ts.append(time.perf_counter() - t0)
    tot += n
    print(f"round {r_}: now={sim.now/1e6:.3f}ms delivered={n} wall={ts[-1]*1e3:.2f}ms", flush=True)
print(sim.stats())
steady = ts[12:]
print("steady ms/round", np.median(steady) * 1e3, "msgs/s", 8 * N / np.median(steady))
