"""sdk-go ``sync.Client`` restated over the simulator's device-side sync service.

Reference: ``github.com/testground/sdk-go`` ``sync.Client`` and ``sync-service v0.1.0`` (``go.mod:33``,
``go.mod:100``; neither is vendored). Call sites that pin the semantics:
``pkg/sidecar/sidecar_handler.go:40-43`` (SignalAndWait), ``:75-79`` (SignalEntry),
``plans/splitbrain/main.go:85`` (seq % 3 from SignalEntry), ``plans/network/pingpong.go:54``
(seq in {1, 2}), ``plans/benchmarks/benchmarks.go:109-141`` (barrier ladders).

* ``signal_entry(state, instances, t)`` increments the state's counter once per instance and
  returns the new values: 1-based sequence numbers, assigned in (t, instance) order. This
  deterministic order stands in for the sync service's arrival order, so results do
  not depend on the number of GPUs.
* ``barrier(state, target, t_wait)`` releases at max(t_wait, time of the target-th signal).
* ``publish`` / ``subscribe``: ordered topics with full history replay, kept as append logs in
  device memory (``tgsim_sync_publish`` / ``tgsim_sync_subscribe``). A topic counts like a state,
  so positions follow (t, instance) order within a batch. Payloads travel as JSON (tuples come
  back as lists).

States are named by strings, as in the SDK; names map to dense device ids in first-use order.
"""
from __future__ import annotations

import json

import numpy as np

from . import _abi as A


class SyncService:
    def __init__(self, sim):
        self.sim = sim
        self._ids: dict[str, int] = {}

    def state_id(self, state: str) -> int:
        if state not in self._ids:
            if len(self._ids) >= self.sim.cfg.max_states:
                raise A.TgsimError(A.ECAPACITY, f"more than {self.sim.cfg.max_states} sync states")
            self._ids[state] = len(self._ids)
        return self._ids[state]

    # ---- counters / barriers ----------------------------------------------------------------
    def signal_entry(self, state: str, instances, t) -> np.ndarray:
        """SignalEntry by each instance at its time; returns the 1-based sequence numbers."""
        inst = np.atleast_1d(np.asarray(instances, dtype=np.uint32))
        tt = np.broadcast_to(np.asarray(t, dtype=np.int64), inst.shape)
        sid = np.full(inst.shape, self.state_id(state), np.uint32)
        return self.sim.signal(sid, inst, tt)

    def barrier(self, state: str, target: int, t_wait: int) -> int:
        """Barrier(state, target) entered at t_wait. Returns the release time, or -1 if the counter
        has not reached target yet (poll again after more signals)."""
        w = self.sim.barrier(self.state_id(state), int(target), int(t_wait))
        return self.sim.poll(w)

    def barrier_waiter(self, state: str, target: int, t_wait: int) -> int:
        """Registers a waiter and returns its id (for Simulator.advance_to_barrier)."""
        return self.sim.barrier(self.state_id(state), int(target), int(t_wait))

    def signal_and_wait(self, state: str, instances, t, target: int):
        """SignalAndWait: every instance signals at its t, then waits for target signals.
        Returns (seq numbers, release time of the barrier for the latest signaller)."""
        seq = self.signal_entry(state, instances, t)
        t_last = int(np.max(np.asarray(t, dtype=np.int64)))
        rel = self.barrier(state, target, t_last)
        if rel < 0:
            raise A.TgsimError(A.ESTATE, f"SignalAndWait({state!r}, {target}): only {self.count(state)} signals")
        return seq, rel

    def count(self, state: str) -> int:
        return self.sim.count(self.state_id(state))

    # ---- topics -----------------------------------------------------------------------------
    def publish(self, topic: str, instances, t, payloads) -> np.ndarray:
        """Publish one payload per instance; returns the 1-based position of each in the topic.
        Order within one call: (t, instance), as for signals; a call must not go back in time."""
        inst = np.atleast_1d(np.asarray(instances, dtype=np.int64))
        tt = np.broadcast_to(np.asarray(t, dtype=np.int64), inst.shape)
        blobs = [json.dumps(p).encode() for p in payloads]
        return self.sim.publish(self.state_id("topic:" + topic), inst, tt, blobs).astype(np.int64)

    def subscribe(self, topic: str, until_t: int | None = None) -> list:
        """All payloads published so far (history replay), in topic order."""
        _, _, blobs = self.sim.subscribe(self.state_id("topic:" + topic),
                                         until_t=(1 << 63) - 1 if until_t is None else until_t)
        return [json.loads(b) for b in blobs]
