#!/usr/bin/env python3
"""Headline benchmark: simulated messages delivered per second on the 100k-instance gossip storm
(BASELINE.json metric), with the dominant kernel's HBM roofline fraction
and the single-threaded CPU oracle timed beside it.

A step is one storm round: every instance sends `fanout` 1 KiB messages to Philox-chosen peers
within `spread` of the round start and SignalAndWait("round-r", N)s; the round window ends at the
barrier release + the sync-service RTT, and everything due in it is delivered into inboxes.
N GPUs = N shards of the same 100k instances (strong scaling), one process per GPU. The library owns
the cross-shard transport (tgsim_comm_init: an RCCL communicator over xGMI): every shard makes the
single-shard calls, the window's exchange (the peer blocks, whole - no host read of their counts) and
the storm batch's MAX all-reduce run inside them on the simulator's stream.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

MS = 1_000_000
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "simulated msgs delivered/sec (100k-inst storm) + % HBM roofline, 1/2/4/8 GPU"

# SURVEY.md 8(d)'s algorithmic bytes, attributed to the kernel that does that part of the path:
#   per input message: read the 24 B record + write its 1 B status (netem + routing: k_extract_shape /
#   k_shape); per delivered copy: write the 24 B delivery record (k_emit_bucket); per window: read the
#   48 B shape table entry of every local sender (with the netem pass) and read + write its 16 B
#   token-bucket state (k_tb_bucket). Kernels that only move the implementation's own structures
#   (wheel extraction and insertion, partition passes) have none. roofline.frac uses these.
#   Messages a sender's queue limit or correlation defers are decided by the sequential lane
#   (k_shape_seq: 25 B each, counted on the device, d["deferred"]); deliveries of long inboxes are
#   written by the wheel-insert launch's k_rest part (24 B each, d["long_emit"]), the others by
#   k_emit_bucket.
ALG_MODELS = {
    "k_extract_shape": lambda d, n, w: 25 * (d["msgs_in"] - d.get("deferred", 0)) + 48 * n * w,
    "k_shape_seq": lambda d, n, w: 25 * (d.get("deferred", 0) - d.get("wide", 0)),
    "k_shape_seq_wide": lambda d, n, w: 25 * d.get("wide", 0),
    "k_tb_bucket": lambda d, n, w: 16 * n * w,
    "k_emit_bucket": lambda d, n, w: 24 * (d["delivered"] - d.get("long_emit", 0)),
    "k_wheel_scatter": lambda d, n, w: 24 * d.get("long_emit", 0),
    "k_gen_storm": lambda d, n, w: 24 * d["msgs_in"],
    # the plans' reactions after a window: the flood reads every delivery once
    # (k_flood_count) and writes every forward, the next window's input message (k_flood_emit); the
    # probe / storm reactors read the window's statuses and deliveries and write the messages they
    # stage (requests, replies, SYNs, chunks: the next window's inputs)
    "k_flood_count": lambda d, n, w: 24 * d["delivered"],
    "k_flood_emit": lambda d, n, w: 24 * d["msgs_in"],
    "k_probe": lambda d, n, w: 24 * d["delivered"] + 25 * d["msgs_in"],
    "k_storm": lambda d, n, w: 24 * d["delivered"] + 25 * d["msgs_in"],
}


def alg_bytes_step(d: dict, n_local: int, windows: int) -> int:
    """SURVEY.md 8(d) B_total of one shard: 25 B per input + 24 B per delivery + 48 B shape + 16 B
    token state per local sender and window (no rules in these workloads; sync counters ~0)."""
    return 25 * d["msgs_in"] + 24 * d["delivered"] + (48 + 16) * n_local * windows


# The implementation's own bytes per launch (what each kernel reads and writes):
# roofline.kernel_bw_eff ("how close does the kernel run to HBM speed") uses these; it is not the
# algorithmic fraction.
#   k_extract_shape (one launch, two passes): netem reads the 24 B message + writes its 1 B status
#     + writes each 32 B copy record; the extraction reads + writes each due 32 B wheel record
#   k_tb_bucket: per copy, read the 32 B record + its 8 B (key, index), write the 32 B departed record
#   k_emit_bucket: per delivery, read the 32 B record + 8 B (key, index), write the 32 B SoA delivery
#   k_extract: read + write one 32 B wheel record; k_wheel_scatter: read 32 + 8 B key/index, write 32 B
#   k_gen_storm: write the 24 B message
BYTE_MODELS = {
    "k_extract_shape": lambda d: 25 * d["msgs_in"] + 32 * d["copies"] + 64 * d["extracted"],
    "k_tb_bucket": lambda d: 72 * d["tb_items"],
    "k_emit_bucket": lambda d: 72 * d["delivered"],
    "k_extract": lambda d: 64 * d["extracted"],
    # the insert moves each later record (4 B key + 32 B read, 32 B written); its k_rest part sorts and
    # rewrites long inboxes (72 B per delivery: key and record read, record written)
    "k_wheel_scatter": lambda d: 72 * d["inserted"] + 72 * d.get("long_emit", 0),
    "k_gen_storm": lambda d: 24 * d["msgs_in"],
    # the sequential lane: per deferred message its 24 B record and 16 B (t, seq) order entry read,
    # its 1 B status and a 32 B copy record written; k_seg_small orders them: per deferred message
    # the (key, index) pair read, (t_send, seq) gathered (12 B), the index written (4 B)
    "k_shape_seq": lambda d: 73 * (d.get("deferred", 0) - d.get("wide", 0)),
    "k_seg_small": lambda d: 24 * d.get("deferred", 0),
    # the whole-sender closed form: as the sequential lane plus its own ordering (the index read and
    # written back in place, (t_send, seq) gathered)
    "k_shape_seq_wide": lambda d: 81 * d.get("wide", 0),
    # flood (config 5): count reads (dst, src, seq) and writes count + first flag per delivery;
    # emit writes the 24 B staged message per forward after re-reading the 17 B per delivery
    "k_flood_count": lambda d: 21 * d["delivered"],
    "k_flood_emit": lambda d: 24 * d["msgs_in"] + 17 * d["delivered"],
}


def source_hash() -> str:
    """SHA-256 (16 hex) of the kernel sources and the ABI header: a committed PMC summary is this
    run's measurement only if it was taken on the same code."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "testground_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "testground_amd", "csrc", "*.h")) +
                   [os.path.join(ROOT, "include", "tgsim.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel: str, workload: str, n_gpus: int):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary of this same command
    (tools/pmc_traffic.py; FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section) - only from a
    summary stamped with this source hash, workload and GPU count; otherwise None."""
    import glob
    want = source_hash()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic*.json")), reverse=True):
        try:
            j = json.load(open(path))
        except (OSError, ValueError):
            continue
        if j.get("source_hash") != want or j.get("workload") != workload or j.get("n_gpus") != n_gpus:
            continue
        ks = j.get("kernels", {})
        k = ks.get(kernel)
        if k:
            return k["traffic_bytes"], os.path.relpath(path, ROOT)
        # a templated kernel (k_extract_shape<false> / <true>): the launch-weighted mean of its forms
        forms = [v for name, v in ks.items() if name.startswith(kernel + "<") and v.get("launches")]
        if forms:
            n = sum(v["launches"] for v in forms)
            return sum(v["traffic_bytes"] * v["launches"] for v in forms) / n, os.path.relpath(path, ROOT)
    return None, None


def host_cpu() -> dict:
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"nproc": avail, "cpu_count": os.cpu_count(), "cpu_model": model}


def roofline(dominant: str, delta: dict, kern_ms: float, kern_n: int, n_local: int, windows: int,
             workload: str, n_gpus: int, b_total: int, elapsed: float) -> dict:
    """roofline.frac = SURVEY.md 8(d) algorithmic bytes of the dominant kernel per launch / its
    average launch time / 8 TB/s; frac_step = the whole path's B_total / wall time / (n_gpus x 8 TB/s);
    kernel_bw_eff = the kernel's own bytes (BYTE_MODELS) at its launch time, as a fraction of peak."""
    avg_ms = kern_ms / max(kern_n, 1)
    alg = ALG_MODELS.get(dominant, lambda d, n, w: 0)(delta, n_local, windows) / max(kern_n, 1)
    impl = BYTE_MODELS.get(dominant, lambda d: 0)(delta) / max(kern_n, 1)
    achieved = alg / (avg_ms * 1e-3) / 1e9 if kern_n else 0.0
    impl_gbs = impl / (avg_ms * 1e-3) / 1e9 if kern_n else 0.0
    traffic, src = pmc_traffic(dominant, workload, n_gpus)
    step_gbs = b_total / elapsed / 1e9
    return {
        "bound": "hbm", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
        "alg_bytes_per_launch": alg, "avg_launch_ms": avg_ms,
        "step_achieved": step_gbs, "frac_step": step_gbs / (n_gpus * HBM_PEAK_GBS),
        "step_alg_bytes": b_total,
        "kernel_bw_eff": impl_gbs / HBM_PEAK_GBS, "impl_bytes_per_launch": impl,
        "source_hash": source_hash(),
    }


def probe_steps(args) -> int:
    """Probe steps before the timed region: as many as it has (at least 10), so the dominant kernel
    is chosen over as many launches as the timed region makes (a 5-step probe flipped
    between two kernels within 2 %)."""
    return max(10, args.steps)


def probe_kernels(sim, step, first: int, probe: int):
    """Every kernel class timed (HIP events on the context stream) over `probe` steps; returns
    ({kernel: avg_us, launches, total_ms}, the kernel with the largest total time among those
    with a byte model)."""
    sim.profile(None)
    base = sim.profile_read()
    for r in range(first, first + probe):
        step(r)
    prof = sim.profile_read()
    ks = {k: {"avg_us": 1e3 * (ms - base[k][0]) / (n - base[k][1]), "launches": n - base[k][1],
              "total_ms": ms - base[k][0]} for k, (ms, n) in prof.items() if n > base[k][1]}
    # the dominant kernel is the one with the most time, whether or not SURVEY.md
    # 8(d) assigns it bytes (its roofline then says so with frac 0)
    ranked = sorted(((v["total_ms"], k) for k, v in ks.items() if k not in COLLECTIVES), reverse=True)
    return ks, (ranked[0][1] if ranked else "k_emit_bucket")


def counters(sim) -> dict:
    """tgsim_stats plus the device's implementation counters (deferred messages, long segments)."""
    d = sim.stats()
    d.update(sim.kernel_counters())
    return d


def kernel_fracs(kernels: dict, delta: dict, n_local: int, windows: int, probe: int) -> dict:
    """SURVEY.md 8(d) bytes per launch / the probe's average launch time, for every kernel with an
    algorithmic byte model (delta: the timed region's counters over `windows` steps, scaled to one
    launch of the probe's cadence)."""
    out = {}
    for k, v in kernels.items():
        if k not in ALG_MODELS or not v["launches"]:
            continue
        per_launch = ALG_MODELS[k](delta, n_local, windows) / max(1, windows) * probe / v["launches"]
        out[k] = {"alg_bytes_per_launch": per_launch, "avg_us": v["avg_us"],
                  "frac": per_launch / (v["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS}
    return out


COLLECTIVES = ("exchange", "allreduce")


def collective_stats(sim, dist, world: int, base: dict, steps: int, transport: str) -> dict | None:
    """Per-rank time of the window's exchange (the peer blocks, tgsim_advance*) and of the storm
    batch's MAX all-reduce over the timed steps (HIP events around the transport calls on the
    context stream), max / mean over the ranks, and the bytes each rank sends per step (whole padded
    peer blocks of exchange_cap 32-B records): what a SCALE curve needs to be attributed."""
    if world == 1:
        return None
    import torch
    prof = sim.profile_read()
    mine = []
    for k in COLLECTIVES:
        ms, n = prof[k][0] - base[k][0], prof[k][1] - base[k][1]
        mine += [ms / max(steps, 1), n / max(steps, 1)]
    t = torch.tensor(mine, dtype=torch.float64)
    tmax, tsum = t.clone(), t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    xbytes = (world - 1) * sim.cfg.exchange_cap * 32
    ex_ms = float(tmax[0].item())
    return {"transport": transport.lstrip("-"), "rehearsal": "rehearsal" in transport or "fallback" in transport,
            "exchange_ms_per_step": {"max": ex_ms, "mean": float(tsum[0].item()) / world},
            "exchange_calls_per_step": float(tmax[1].item()),
            "allreduce_ms_per_step": {"max": float(tmax[2].item()), "mean": float(tsum[2].item()) / world},
            "allreduce_calls_per_step": float(tmax[3].item()),
            "exchange_bytes_per_step_per_rank": xbytes * float(tmax[1].item()),
            "exchange_gbs_per_rank": xbytes * float(tmax[1].item()) / (ex_ms * 1e-3) / 1e9 if ex_ms > 0 else None}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--instances", type=int, default=100_000)
    p.add_argument("--fanout", type=int, default=8)
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--spread-ms", type=float, default=10.0)
    p.add_argument("--rtt-ms", type=float, default=1.0)
    p.add_argument("--seed", type=int, default=4)
    p.add_argument("--max-records", type=int, default=1 << 23)
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    # config 5 (not the headline): 1M-instance random-regular pubsub flood, one window per step
    p.add_argument("--workload", choices=("storm", "flood", "a2a", "splitbrain"), default="storm")
    p.add_argument("--a2a-instances", type=int, default=1000)
    p.add_argument("--sb-instances", type=int, default=10_000)
    p.add_argument("--sb-case", choices=("accept", "drop", "reject"), default="accept")
    p.add_argument("--tcp", action="store_true",
                   help="storm over TCP mode (DESIGN.md 2.11): writes, retransmissions, one reaction per window")
    p.add_argument("--tcp-acks", action="store_true",
                   help="with --tcp: ACK packets on the reverse path and retransmission timers (tgsim.h acks = 1)")
    p.add_argument("--flood-instances", type=int, default=1_000_000)
    p.add_argument("--flood-size", type=int, default=512)
    p.add_argument("--pub-every", type=int, default=4, help="windows between publication waves (flood)")
    p.add_argument("--pubs-per-wave", type=int, default=1,
                   help="publications per wave (flood; distinct publishers; SURVEY's literal 1%% of 1M "
                        "instances = 10000 floods per wave does not fit in memory: DESIGN.md 5.4)")
    p.add_argument("--window-ms", type=float, default=10.0, help="window length (flood)")
    p.add_argument("--flood-records-per-pub", type=int, default=1 << 25,
                   help="flood: max_records per publication of a wave (the wheel arena is twice it; "
                        "heavier waves need more than the default's headroom: tools/flood_load.sh)")
    p.add_argument("--no-beside", action="store_true",
                   help="storm: skip config 5 (the 1M flood, same GPU count) reported beside the headline")
    a = p.parse_args()
    if a.workload == "splitbrain":
        a.warmup = a.warmup if "--warmup" in sys.argv else 200
        a.steps = a.steps if "--steps" in sys.argv else 500
    if a.workload == "flood":
        # the flood reaches steady state after a publication's lifetime (~80 windows)
        a.warmup = a.warmup if "--warmup" in sys.argv else 100
        a.steps = a.steps if "--steps" in sys.argv else 50
    return a


def storm_shapes(n: int, seed: int):
    from testground_amd.sim import make_shape
    rng = np.random.default_rng(seed)
    lat = rng.integers(20, 101, n) * MS  # per-sender latency U[20,100] ms
    return [make_shape(latency_ns=int(lat[g]), jitter_ns=5 * MS, bandwidth_bps=10_000_000, loss=0.5)
            for g in range(n)]


def exchange_cap(per_window: int, n_shards: int) -> int:
    """Records per peer block: the copies due in a window between one pair of shards (about
    per_window / S^2 with uniform peers), 1.25x plus 4096 of headroom. Blocks travel whole, so the
    bound is also the exchange's volume; an overflow is reported (ECAPACITY), never truncated."""
    s = max(n_shards, 1)
    return int(1.25 * per_window / (s * s)) + 4096


def sim_config(args, shard=0, n_shards=1, device=0):
    from testground_amd.sim import SimConfig
    # TCP with ACKs: a window stages the round's writes plus the last window's ACKs (one per
    # delivered data packet) plus the fired timers, and keeps about twice the records in flight
    acks = getattr(args, "tcp", False) and getattr(args, "tcp_acks", False)
    per_window = args.instances * args.fanout * (2 if acks else 1) + (1 << 16 if acks else 0)
    return SimConfig(n_instances=args.instances, seed=args.seed, shard_id=shard, n_shards=n_shards, device=device,
                     data_prefix_len=12, max_msgs_per_window=max(1 << 20, per_window),
                     max_records=args.max_records * (2 if acks else 1) // max(1, n_shards // 2), max_states=4096,
                     exchange_cap=exchange_cap(per_window, n_shards))


def cpu_baseline(args, shapes):
    """The CPU oracle (single thread) on the same storm: warm up to steady state, then time a
    bounded number of rounds (about args.cpu_seconds of work)."""
    from oracle.pyoracle import oracle_binding
    from testground_amd.sim import Simulator
    sim = Simulator(sim_config(args), binding=oracle_binding())
    sim.set_shapes(np.arange(args.instances), shapes)
    spread, rtt = int(args.spread_ms * MS), int(args.rtt_ms * MS)

    def round_(r):
        now = sim.now
        sim.gen_storm_round(r, now, args.fanout, args.size, spread, r)
        sim.advance_to_barrier(sim.barrier(r, args.instances, now), rtt)

    warm = 10
    for r in range(warm):
        round_(r)
    d0 = sim.stats()["delivered"]
    t0 = time.perf_counter()
    r = warm
    while True:
        round_(r)
        r += 1
        el = time.perf_counter() - t0
        if (el >= args.cpu_seconds and r - warm >= 3) or r - warm >= 60:
            break
    delivered = sim.stats()["delivered"] - d0
    sim.close()
    return {"value": delivered / el, "unit": "msgs/s", "cores": 1, "kind": "port", **host_cpu(),
            "sample": f"oracle/ (single-threaded C restatement), same {args.instances}-instance storm: "
                      f"rounds {warm}..{r - 1} timed ({el:.1f} s, {delivered} deliveries) after {warm} "
                      f"warm-up rounds"}




def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv=None, script=None) -> int:
    """`python bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment): start the N
    ranks as child processes of this one, one per GPU, with the variables torch.distributed.run would
    set, and forward rank 0's output. This process never touches the GPU (no torch.cuda call, no
    libtgsim.so load: it imports neither), so nothing here is initialised when the children start.
    Returns the exit status: the first failing rank's, else 0. A rank that fails makes the others'
    collectives fail or hang, so after the first failure the rest get a grace period and are killed."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = None if r == 0 else subprocess.DEVNULL  # rank 0 prints the JSON line; others' stdout is quiet
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] +
                                      list(sys.argv[1:] if argv is None else argv), env=env,
                                      stdout=out, start_new_session=True))
    rc = 0
    failed_at = None
    while any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            code = p.poll()
            if code not in (None, 0) and rc == 0:
                rc, failed_at = code, time.monotonic()
                print(f"bench: rank {r} exited with {code}", file=sys.stderr, flush=True)
        if failed_at is not None and time.monotonic() - failed_at > 30:
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, signal.SIGKILL)
        time.sleep(0.2)
    for r, p in enumerate(procs):
        if p.returncode and rc == 0:
            rc = p.returncode
            print(f"bench: rank {r} exited with {p.returncode}", file=sys.stderr, flush=True)
    return rc if rc > 0 else (1 if rc else 0)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.workload in ("a2a", "splitbrain"):
            raise SystemExit(f"--workload {args.workload} is a single-GPU configuration")
        sys.exit(spawn_ranks(args.gpus))
    if args.workload == "flood":
        return main_flood(args)
    if args.workload == "a2a":
        return main_a2a(args)
    if args.workload == "splitbrain":
        return main_splitbrain(args)
    torch, dist, world, rank, local, rehearsal, stream = _dist_setup(args)
    from testground_amd._abi import T_NOW
    from testground_amd.sim import Simulator

    shapes = storm_shapes(args.instances, args.seed)
    sim = Simulator(sim_config(args, rank, world, local))
    sim.set_stream(stream.cuda_stream)
    transport = _attach_transport(sim, dist, world, rank, rehearsal)
    sim.set_shapes(np.arange(sim.lo, sim.hi), shapes[sim.lo:sim.hi])
    spread, rtt = int(args.spread_ms * MS), int(args.rtt_ms * MS)
    N, F = args.instances, args.fanout

    if args.tcp:  # sharded: each rank's writers (arrivals forwarded to the writer's shard)
        rounds = args.warmup + probe_steps(args) + args.steps + 1
        nl = sim.hi - sim.lo
        sim.tcp_enable(max_writes=rounds * nl * F, max_segments=rounds * nl * F, acks=args.tcp_acks)

    def step(r: int):
        # t0 / t_wait = TGSIM_T_NOW: the round starts where the device's last window ended, so a
        # step issues its launches without any host round trip (sharded: the same calls, collective)
        if args.tcp:  # the same round as TCP writes; the reaction is queued without a read-back
            sim.tcp_gen_storm_round(r, T_NOW, F, args.size, spread, r)
            sim.advance_to_barrier(sim.barrier(r, N, T_NOW), rtt)
            sim.tcp_react(wait=False)
            return
        sim.gen_storm_round(r, T_NOW, F, args.size, spread, r)
        sim.advance_to_barrier(sim.barrier(r, N, T_NOW), rtt)

    # warm-up (untimed, unprofiled), then probe steps (as many as the timed region) that time every
    # kernel class: the dominant one is the largest total time; the timed region carries HIP events
    # around that kernel only
    for r in range(args.warmup):
        step(r)
    probe = probe_steps(args)
    warm_kernels, dominant = probe_kernels(sim, step, args.warmup, probe)
    sim.profile([dominant] + (list(COLLECTIVES) if world > 1 else []))
    base_all = sim.profile_read()
    base_prof = base_all[dominant]
    first = args.warmup + probe

    s0 = counters(sim)
    tcp0 = sim.tcp_stats() if args.tcp else None
    sim_t0 = sim.now
    sim.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for r in range(first, first + args.steps):
        step(r)
    sim.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    s1 = counters(sim)
    tcp1 = sim.tcp_stats() if args.tcp else None
    sim_t1 = sim.now
    prof = sim.profile_read()[dominant]
    delta = {k: s1[k] - s0[k] for k in s1}

    kern_ms = prof[0] - base_prof[0]
    kern_n = prof[1] - base_prof[1]
    delivered = delta["delivered"]
    b_total = alg_bytes_step(delta, sim.hi - sim.lo, args.steps)
    if world > 1:  # the process group is gloo: host tensors
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        v = torch.tensor([delivered, b_total], dtype=torch.int64)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        delivered, b_total = int(v[0].item()), int(v[1].item())
    # (TCP lines: the PMC summaries are the message storm's, so their traffic is looked up under
    # their own workload name, which no committed summary carries: null)
    wl = ("tcp_acks" if args.tcp_acks else "tcp") if args.tcp else "storm"
    roof = roofline(dominant, delta, kern_ms, kern_n, sim.hi - sim.lo, args.steps, wl, world, b_total, elapsed)
    roof["kernels"] = kernel_fracs(warm_kernels, delta, sim.hi - sim.lo, args.steps, probe)
    coll = collective_stats(sim, dist, world, base_all, args.steps, transport)
    if coll:
        roof["collectives"] = coll
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.tcp:
        cpu = cpu_baseline(args, shapes)

    if args.tcp:
        dt = {k: tcp1[k] - tcp0[k] for k in tcp1}
        if world > 1:  # every rank's writers' counters (gloo: host tensors)
            keys = sorted(dt)
            v = torch.tensor([dt[k] for k in keys], dtype=torch.int64)
            dist.all_reduce(v, op=dist.ReduceOp.SUM)
            dt = {k: int(x) for k, x in zip(keys, v.tolist())}
        if rank == 0:
            print(json.dumps({
                "metric": "TCP writes delivered/sec (100k-inst storm over TCP mode, DESIGN.md 2.11)"
                          + (", ACKs on the reverse path" if args.tcp_acks else ""),
                "value": dt["delivered"] / elapsed, "unit": "writes/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
                "scaling": "strong", "parallelism": f"shard{world}{transport}",
                "packets_delivered_per_s": delivered / elapsed, "tcp_in_timed_steps": dt,
                "collectives": coll, "dtype": "int64", "data": "synthetic", "roofline": roof,
                "cpu_baseline": None, "kernels_probe": warm_kernels}),
                flush=True)
        sim.close()
        if world > 1:
            dist.destroy_process_group()
        return
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": delivered / elapsed,
            "unit": "msgs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {
                "workload": "gossip storm (SURVEY.md 8(d) config 4): 100k instances, fanout 8 Philox peers, "
                            "1 KiB messages within 10 ms, per-sender 10 Mbit/s HTB, latency U[20,100] ms, "
                            "jitter 5 ms, loss 0.5%, SignalAndWait(round, N) + 1 ms sync RTT per round",
                "instances": N, "fanout": F, "msg_bytes": args.size,
                "parallelism": f"shard{world}{transport}",
                "delivered_in_timed_steps": delivered,
                "simulated_ms_per_step": (sim_t1 - sim_t0) / 1e6 / args.steps,
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "kernels_probe": warm_kernels,
        }
    sim.close()
    if not args.no_beside:
        # config 5 at the same GPU count (the weak-scaling-friendly config beside
        # the headline, so a SCALE run carries both curves); its own defaults, no CPU baseline
        fa = argparse.Namespace(**vars(args))
        fa.warmup, fa.steps, fa.no_cpu_baseline, fa.seed = 100, 50, True, 5
        fl = main_flood(fa, ctx=(torch, dist, world, rank, local, rehearsal, stream), emit=False)
        if rank == 0:
            line["beside"] = {"flood": {k: fl[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup",
                                                            "config", "roofline")}}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()



def _dist_setup(args):
    """One process per GPU. torch.distributed (gloo, host side) only distributes the RCCL unique id
    and reduces the timing; the simulator's data path uses its own communicator. More ranks than
    GPUs = a rehearsal on shared devices over a gloo transport (RCCL refuses two ranks on a GPU)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    # TGSIM_BENCH_TRY_RCCL=1: ranks sharing a GPU still try the RCCL communicator (which refuses a
    # duplicate GPU), exercising the agreed gloo fallback of _attach_transport on a one-GPU box
    rehearsal = world > ndev and os.environ.get("TGSIM_BENCH_TRY_RCCL") != "1"
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")
    stream = torch.cuda.Stream()  # one stream shared by torch and the simulator
    torch.cuda.set_stream(stream)
    return torch, dist, world, rank, local, rehearsal, stream


def _attach_transport(sim, dist, world: int, rank: int, rehearsal: bool) -> str:
    """The shards' transport: the library's RCCL communicator, or (rehearsal, or when any rank's
    communicator fails to come up) the gloo transport - agreed over all ranks, and named in the
    JSON line's parallelism so a fallback is never mistaken for the RCCL path."""
    if world == 1:
        return ""
    from testground_amd.exchange import GlooTransport
    if rehearsal:
        sim.set_transport(GlooTransport(dist, device=True))
        return "-gloo-rehearsal"
    import torch
    from testground_amd.sim import Simulator
    uid = [None]
    if rank == 0:
        try:
            uid[0] = Simulator.comm_unique_id()
        except Exception as e:  # noqa: BLE001 - every rank sees None and takes the fallback
            print(f"rank 0: RCCL unique id failed ({e}); falling back to the gloo transport",
                  file=sys.stderr, flush=True)
    dist.broadcast_object_list(uid, src=0)
    # ncclCommInitRank blocks until every rank joins: agree over gloo first that every rank can
    # (a unique id, a working device of its own), so that one rank failing fast cannot leave the
    # others waiting in RCCL's bootstrap
    import socket
    pre = 1
    dev = None
    try:
        if uid[0] is None:
            raise RuntimeError("no RCCL unique id")
        dev = torch.cuda.current_device()
        torch.cuda.synchronize(dev)
    except Exception as e:  # noqa: BLE001 - reported, then every rank takes the same path
        print(f"rank {rank}: RCCL preconditions failed ({e})", file=sys.stderr, flush=True)
        pre = 0
    where = [None] * world
    dist.all_gather_object(where, (socket.gethostname(), dev))
    if pre and len(set(where)) != world:
        print(f"rank {rank}: ranks share a device ({where}); no RCCL communicator", file=sys.stderr, flush=True)
        pre = 0
    flag = torch.tensor([pre], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    ok = 1
    try:
        if int(flag.item()) != 1:
            raise RuntimeError("a rank failed the RCCL preconditions")
        sim.comm_init(uid[0], world, rank)
    except Exception as e:  # noqa: BLE001 - reported, then every rank takes the same path
        print(f"rank {rank}: RCCL communicator failed ({e}); falling back to the gloo transport",
              file=sys.stderr, flush=True)
        ok = 0
    flag = torch.tensor([ok], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:
        return "-rccl"
    sim.set_transport(GlooTransport(dist, device=True))
    return "-gloo-fallback"


def flood_cpu_baseline(args, shapes, graph):
    """The CPU oracle on the same flood from its first window, for a bounded sample (about
    args.cpu_seconds): the per-message cost does not depend on the flood's phase."""
    from oracle.pyoracle import oracle_binding
    from testground_amd import workloads as W
    from testground_amd.sim import Simulator
    N = args.flood_instances
    sim = Simulator(flood_config(args), binding=oracle_binding())
    sim.set_shapes(np.arange(N), shapes)
    sim.flood_set_graph(*graph, flood_max_pubs(args))
    win = int(args.window_ms * MS)
    t0 = time.perf_counter()
    w = 0
    while True:
        if w % args.pub_every == 0:
            k, P = w // args.pub_every, args.pubs_per_wave
            sim.flood_publish(W.publishers(N, P, k, args.seed), np.arange(P) + k * P, sim.now, args.flood_size)
        sim.advance(sim.now + win)
        sim.flood_react(args.flood_size, count=False)
        w += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or w >= 400:
            break
    delivered = sim.stats()["delivered"]
    sim.close()
    return {"value": delivered / el, "unit": "msgs/s", "cores": 1, "kind": "port", **host_cpu(),
            "sample": f"oracle/ (single-threaded C restatement), same {N}-instance flood: windows 0..{w - 1} "
                      f"from the first publication ({el:.1f} s, {delivered} deliveries, incl. the reaction)"}


def flood_config(args, shard=0, n_shards=1, device=0):
    from testground_amd.sim import SimConfig
    return SimConfig(n_instances=args.flood_instances, seed=args.seed, shard_id=shard, n_shards=n_shards,
                     device=device, data_prefix_len=11, max_msgs_per_window=(1 << 23) * args.pubs_per_wave,
                     max_records=args.flood_records_per_pub * args.pubs_per_wave,
                     exchange_cap=exchange_cap(3 << 20, n_shards))


def flood_max_pubs(args) -> int:
    # every window of the run publishes on schedule: warm-up, the kernel probe and the timed steps
    return ((args.warmup + probe_steps(args) + args.steps + 20) // args.pub_every + 2) * args.pubs_per_wave


def main_flood(args, ctx=None, emit=True):
    """Config 5 (BASELINE.json configs[4]): 1M instances on a random 8-regular graph
    with heterogeneous LinkShapes; one publication every `pub_every` windows floods the graph with
    first-receipt dedup (tgsim_flood_react after every window). A step is one window; `value` =
    deliveries of all ranks in the K timed windows / the max-over-ranks wall time. ctx: the process
    group and stream of a storm run that reports this line beside its own (emit=False: returned)."""
    torch, dist, world, rank, local, rehearsal, stream = ctx or _dist_setup(args)
    from testground_amd import workloads as W
    from testground_amd.sim import Simulator
    args.seed = 5 if "--seed" not in sys.argv else args.seed
    N = args.flood_instances
    shapes = W.pubsub_shapes(N, args.seed)
    graph = W.random_regular_graph(N, 8, args.seed)
    sim = Simulator(flood_config(args, rank, world, local))
    sim.set_stream(stream.cuda_stream)
    transport = _attach_transport(sim, dist, world, rank, rehearsal)
    sim.set_shapes(np.arange(sim.lo, sim.hi), shapes[sim.lo:sim.hi])
    sim.flood_set_graph(*graph, flood_max_pubs(args))
    win = int(args.window_ms * MS)

    def step(w: int):
        if w % args.pub_every == 0:
            k, P = w // args.pub_every, args.pubs_per_wave
            sim.flood_publish(W.publishers(N, P, k, args.seed), np.arange(P) + k * P, sim.now, args.flood_size)
        sim.advance(sim.now + win, wait=False)  # sharded: collective, the exchange inside; no host sync
        sim.flood_react(args.flood_size, count=False)

    for w in range(args.warmup):
        step(w)
    probe = probe_steps(args)
    warm_kernels, dominant = probe_kernels(sim, step, args.warmup, probe)
    sim.profile([dominant] + (list(COLLECTIVES) if world > 1 else []))
    base_all = sim.profile_read()
    base_prof = base_all[dominant]
    first = args.warmup + probe
    s0 = counters(sim)
    sim.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for w in range(first, first + args.steps):
        step(w)
    sim.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    s1 = counters(sim)
    prof = sim.profile_read()[dominant]
    delta = {k: s1[k] - s0[k] for k in s1}
    kern_ms, kern_n = prof[0] - base_prof[0], prof[1] - base_prof[1]
    delivered = delta["delivered"]
    b_total = alg_bytes_step(delta, sim.hi - sim.lo, args.steps)
    if world > 1:  # gloo process group: host tensors
        t = torch.tensor([elapsed], dtype=torch.float64)
        v = torch.tensor([delivered, b_total], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        elapsed, delivered, b_total = float(t.item()), int(v[0].item()), int(v[1].item())
    roof = roofline(dominant, delta, kern_ms, kern_n, sim.hi - sim.lo, args.steps, "flood", world, b_total,
                    elapsed)
    roof["kernels"] = kernel_fracs(warm_kernels, delta, sim.hi - sim.lo, args.steps, probe)
    coll = collective_stats(sim, dist, world, base_all, args.steps, transport)
    if coll:
        roof["collectives"] = coll
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = flood_cpu_baseline(args, shapes, graph)
    out = None
    if rank == 0:
        out = {
            "metric": "simulated msgs delivered/sec (1M-inst random-regular pubsub flood) + % HBM roofline",
            "value": delivered / elapsed, "unit": "msgs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": "pubsub flood (SURVEY.md 8(d) config 5): 1M instances, random 8-regular graph, "
                                   "first-receipt dedup, latency {10,50,100,200} ms, jitter U[0,20] ms, loss "
                                   "{0,0.1,1}%, bandwidth {1,10,100} Mbit/s; "
                                   f"{args.pubs_per_wave} publication(s) every {args.pub_every} windows of "
                                   f"{args.window_ms} ms",
                       "pubs_per_wave": args.pubs_per_wave,
                       "instances": N, "msg_bytes": args.flood_size,
                       "parallelism": f"shard{world}{transport}",
                       "delivered_in_timed_steps": delivered},
            "roofline": roof,
            "cpu_baseline": cpu,
            "kernels_probe": warm_kernels,
        }
        if emit:
            print(json.dumps(out), flush=True)
    sim.close()
    if world > 1 and ctx is None:
        dist.destroy_process_group()
    return out


# ---- config 2: 1k instances all-to-all (BASELINE.json configs[1]) -------------

A2A_ROUND_NS = 10 * MS


def a2a_round(n: int, r: int, senders=None):
    """Round r of config 2: every sender to every other instance, 4 KiB, t_send = r * 10 ms +
    U[0, 1 ms) as a pure function of (src, seq), seq = r * n + dst (tests/test_full_size.py)."""
    snd = np.arange(n, dtype=np.uint32) if senders is None else np.asarray(senders, np.uint32)
    src = np.repeat(snd, n - 1)
    dst = (src + np.tile(np.arange(1, n, dtype=np.uint32), len(snd))) % np.uint32(n)
    seq = np.uint32(r * n) + dst
    h = (src.astype(np.uint64) * np.uint64(2654435761) + seq.astype(np.uint64) * np.uint64(40503)) & np.uint64(0xFFFFFFFF)
    t = r * A2A_ROUND_NS + (h % np.uint64(MS)).astype(np.int64)
    return src, dst, seq, np.full(len(src), 4096, np.uint32), t


def a2a_shapes(n: int):
    from testground_amd.sim import make_shape
    return [make_shape(latency_ns=50 * MS, jitter_ns=10 * MS, loss=1.0)] * n


def a2a_config(n: int):
    from testground_amd.sim import SimConfig
    return SimConfig(n_instances=n, seed=2, max_msgs_per_window=1 << 20, max_records=1 << 23)


def main_a2a(args):
    """Config 2: 1k instances all-to-all, 4 KiB, latency 50 ms, jitter 10 ms, loss 1 %, one round of
    999k messages per 10 ms window (the synthetic all-at-once pattern SURVEY.md 8(d) states: every
    sender's queue holds ~5 rounds, so netem's 1000-packet limit tail-drops ~80 % and every sender
    takes the sequential queue-limit lane, k_shape_seq). A step = one round. The rounds' messages
    are generated into HBM before the timed region; a step stages one (tgsim_enqueue_device)."""
    import torch
    from testground_amd.sim import Simulator
    n = args.a2a_instances
    rounds = args.warmup + probe_steps(args) + args.steps
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    cols = []
    for r in range(rounds):
        src, dst, seq, size, t = a2a_round(n, r)
        cols.append(tuple(torch.from_numpy(x.view(np.int32) if x.dtype == np.uint32 else x).to(dev)
                          for x in (src, dst, seq, size, t)))
    torch.cuda.synchronize()
    sim = Simulator(a2a_config(n))
    sim.set_stream(stream.cuda_stream)
    sim.set_shapes(np.arange(n), a2a_shapes(n))
    m = n * (n - 1)

    def step(r: int):
        c = cols[r]
        sim.enqueue_device(c[0].data_ptr(), c[1].data_ptr(), c[2].data_ptr(), c[3].data_ptr(), c[4].data_ptr(), m)
        sim.advance((r + 1) * A2A_ROUND_NS, wait=False)

    for r in range(args.warmup):
        step(r)
    probe = probe_steps(args)
    warm_kernels, dominant = probe_kernels(sim, step, args.warmup, probe)
    sim.profile([dominant])
    base_prof = sim.profile_read()[dominant]
    first = args.warmup + probe
    s0 = counters(sim)
    sim.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(first, first + args.steps):
        step(r)
    sim.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    s1 = counters(sim)
    prof = sim.profile_read()[dominant]
    delta = {k: s1[k] - s0[k] for k in s1}
    b_total = alg_bytes_step(delta, n, args.steps)
    roof = roofline(dominant, delta, prof[0] - base_prof[0], prof[1] - base_prof[1], n, args.steps, "a2a", 1,
                    b_total, elapsed)
    roof["kernels"] = kernel_fracs(warm_kernels, delta, n, args.steps, probe)
    cpu = None if args.no_cpu_baseline else a2a_cpu_baseline(args, n)
    print(json.dumps({
        "metric": "simulated msgs delivered/sec (1k-inst all-to-all storm, config 2) + % HBM roofline",
        "value": delta["delivered"] / elapsed, "unit": "msgs/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
        "config": {"workload": "all-to-all (SURVEY.md 8(d) config 2): 1000 instances, 4 KiB, t_send U[0,1 ms) per "
                               "10 ms round, latency 50 ms, jitter 10 ms, loss 1%; synthetic all-at-once rounds "
                               "(a stress pattern: the reference's storm paces its writes - tests/test_plans_oracle.py)",
                   "instances": n, "msgs_per_round": m, "parallelism": "shard1",
                   "msgs_in_timed_steps": delta["msgs_in"], "overlimit_in_timed_steps": delta["overlimit"],
                   "delivered_in_timed_steps": delta["delivered"]},
        "roofline": roof, "cpu_baseline": cpu, "kernels_probe": warm_kernels}), flush=True)
    sim.close()


def a2a_cpu_baseline(args, n):
    from oracle.pyoracle import oracle_binding
    from testground_amd.sim import Simulator
    sim = Simulator(a2a_config(n), binding=oracle_binding())
    sim.set_shapes(np.arange(n), a2a_shapes(n))
    warm = 8
    for r in range(warm):
        sim.enqueue(*a2a_round(n, r))
        sim.advance((r + 1) * A2A_ROUND_NS)
    d0 = sim.stats()["delivered"]
    t0 = time.perf_counter()
    r = warm
    while True:
        src, dst, seq, size, t = a2a_round(n, r)
        sim.enqueue(src, dst, seq, size, t)
        sim.advance((r + 1) * A2A_ROUND_NS)
        r += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or r - warm >= 40:
            break
    delivered = sim.stats()["delivered"] - d0
    sim.close()
    return {"value": delivered / el, "unit": "msgs/s", "cores": 1, "kind": "port", **host_cpu(),
            "sample": f"oracle/ (single-threaded C restatement), same {n}-instance all-to-all: rounds {warm}..{r - 1} "
                      f"timed ({el:.1f} s, {delivered} deliveries) after {warm} warm-up rounds"}


# ---- config 3: 10k-instance splitbrain with sequential probes (BASELINE.json configs[2]) --------------

SB_WINDOW_NS = 100_000
SB_TIMEOUT_NS = 60_000 * MS


def sb_setup(sim, n: int, case: str):
    """plans/splitbrain at config 3: region = seq % 3 with seq = g + 1; region A holds a /32 rule
    (Drop / Reject) toward every region-B address (accept: none); probes in instance order."""
    from testground_amd import _abi as A
    region = (np.arange(n) + 1) % 3
    if case != "accept":
        action = A.FILTER_DROP if case == "drop" else A.FILTER_REJECT
        b = np.flatnonzero(region == 1)
        rules = (A.LinkRule * len(b))()
        for i, g in enumerate(b):
            rules[i].subnet_ip = sim.get_ip(int(g))
            rules[i].prefix_len = 32
            rules[i].shape.filter = action
        for g in np.flatnonzero(region == 0):
            sim._check(sim.lib.add_rules(sim._ctx, int(g), rules, len(b)))
    sim.probe_setup(np.arange(n), 66, 66, SB_TIMEOUT_NS, SB_WINDOW_NS)
    sim.probe_start(0)


def sb_config(n: int):
    from testground_amd.sim import SimConfig
    return SimConfig(n_instances=n, seed=3, max_msgs_per_window=1 << 16, max_records=1 << 18)


def main_splitbrain(args):
    """Config 3 as the reference plan generates it: every node probes every other node one request /
    reply at a time (tgsim_probe_*). A step is one window; the window's end is the
    device's proposal (tgsim_probe_state_device -> tgsim_advance_begin_device), so the loop never
    reads the device. value = deliveries / wall time."""
    import torch
    from testground_amd.sim import Simulator
    n = args.sb_instances
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sim = Simulator(sb_config(n))
    sim.set_stream(stream.cuda_stream)
    sb_setup(sim, n, args.sb_case)
    sim.advance(SB_WINDOW_NS)
    sim.probe_react(wait=False)
    ne_ptr, act_ptr = sim.probe_state_device()

    def step(_w: int):
        sim.advance_begin_device(ne_ptr, 0)
        sim.advance_end()
        sim.probe_react(wait=False)

    for w in range(args.warmup):
        step(w)
    probe = probe_steps(args)
    warm_kernels, dominant = probe_kernels(sim, step, args.warmup, probe)
    sim.profile([dominant])
    base_prof = sim.profile_read()[dominant]
    s0 = counters(sim)
    sim.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for w in range(args.steps):
        step(w)
    sim.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    s1 = counters(sim)
    prof = sim.profile_read()[dominant]
    sim.advance_begin_device(ne_ptr, 0)  # one more window and reaction, synchronised: the state after
    sim.advance_end()                    # the timed region
    ne, act = sim.probe_react()
    delta = {k: s1[k] - s0[k] for k in s1}
    b_total = alg_bytes_step(delta, n, args.steps)
    roof = roofline(dominant, delta, prof[0] - base_prof[0], prof[1] - base_prof[1], n, args.steps, "splitbrain", 1,
                    b_total, elapsed)
    roof["kernels"] = kernel_fracs(warm_kernels, delta, n, args.steps, probe)
    cpu = None if args.no_cpu_baseline else sb_cpu_baseline(args, n)
    print(json.dumps({
        "metric": "simulated msgs delivered/sec (10k-inst splitbrain, sequential probes, config 3) + % HBM roofline",
        "value": delta["delivered"] / elapsed, "unit": "msgs/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
        "config": {"workload": f"splitbrain {args.sb_case} (SURVEY.md 8(d) config 3, plans/splitbrain/main.go:153-175): "
                               f"{n} instances, region = seq % 3, each GETs every other one at a time "
                               f"(request + reply, 60 s timeout), {SB_WINDOW_NS // 1000} us reaction windows",
                   "instances": n, "case": args.sb_case, "parallelism": "shard1", "step": "one window",
                   "delivered_in_timed_steps": delta["delivered"], "active_probers_after": act},
        "roofline": roof, "cpu_baseline": cpu, "kernels_probe": warm_kernels}), flush=True)
    sim.close()


def sb_cpu_baseline(args, n):
    from oracle.pyoracle import oracle_binding
    from testground_amd.sim import Simulator
    sim = Simulator(sb_config(n), binding=oracle_binding())
    sb_setup(sim, n, args.sb_case)
    ne = SB_WINDOW_NS
    d0, w = sim.stats()["delivered"], 0
    t0 = time.perf_counter()
    while True:
        sim.advance(ne)
        ne, act = sim.probe_react()
        w += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or act == 0 or w >= 20_000:
            break
    delivered = sim.stats()["delivered"] - d0
    sim.close()
    return {"value": delivered / el, "unit": "msgs/s", "cores": 1, "kind": "port", **host_cpu(),
            "sample": f"oracle/ (single-threaded C restatement), same {n}-instance splitbrain {args.sb_case}: "
                      f"windows 0..{w - 1} ({el:.1f} s, {delivered} deliveries, incl. the probe reaction)"}


if __name__ == "__main__":
    main()
