"""Runner ``local:mi355x``: the ``api.Runner`` plugin a Testground engine would register beside
local:exec, local:docker and cluster:k8s (``pkg/engine/engine.go:33-38``).

Mirrors ``api.Runner`` (``pkg/api/runner.go:17-34``): ``ID``, ``Run``, ``ConfigType``,
``CompatibleBuilders``, ``CollectOutputs``, with ``RunInput``/``RunGroup`` (``runner.go:37-85``),
``RunOutput`` (``runner.go:87-102``) and ``runner.Result`` (``pkg/runner/common_result.go:8-58``).
The Go side of the same plugin (cgo over include/tgsim.h) is in INTEGRATION.md; this Python
restatement drives the identical C ABI through ctypes and is what the tests exercise.

Instances are simulated: the group's artifact is not executed; the (plan, case) pair selects a
workload descriptor from :data:`testground_amd.plans.PLANS`. Instance ids are assigned group by
group in composition order (the order ``local_exec.go:108-160`` starts them in).

Outcomes travel as the instances' runtime events (sdk-go ``runtime.Event`` [EXT]: StartEvent,
SuccessEvent{TestGroupID}, FailureEvent{TestGroupID, Error}, stamped with the simulated time), and
the result is counted from them exactly as ``LocalDockerRunner.collectOutcomes`` does
(``local_docker.go:216-255``). :class:`PrettyPrinter` renders the same stream the way
``pkg/runner/pretty.go:113-232`` renders an instance's stdout.
"""
from __future__ import annotations

import enum
import io
import json
import os
import tarfile
import time
from dataclasses import asdict, dataclass, field

import numpy as np

from . import plans as P
from .network import MS, IPNet, int_to_ip

OUTCOME_SUCCESS, OUTCOME_FAILURE, OUTCOME_CANCELED, OUTCOME_UNKNOWN = "success", "failure", "canceled", "unknown"


def next_data_network(n_networks: int):
    """pkg/runner/common.go:28-40 nextDataNetwork: the n-th run's data subnet is
    (16 + n/256).(n%256).0.0/16 with gateway .1; more than 4096 concurrent networks is an error.
    Returns (IPNet, gateway)."""
    if n_networks > 4095 or n_networks < 0:
        raise ValueError("space exhausted")
    a, b = 16 + n_networks // 256, n_networks % 256
    net = IPNet((a << 24) | (b << 16), 16)
    return net, net.ip | 1


class EventType(enum.IntEnum):
    """pretty.go:21-33, in its order (the printer's classes index by it)."""
    Error = 0
    Start = 1
    Ok = 2
    Fail = 3
    Crash = 4
    Incomplete = 5
    Message = 6
    Metric = 7
    Other = 8
    InternalErr = 9


_CLASS = ["ERROR", "START", "OK", "FAIL", "CRASH", "INCOMPLETE", "MESSAGE", "METRIC", "OTHER", "INTERNAL_ERR"]


def start_event(group: str, runenv: dict) -> dict:
    return {"StartEvent": {"Runenv": {**runenv, "TestGroupID": group}}}


def success_event(group: str) -> dict:
    return {"SuccessEvent": {"TestGroupID": group}}


def failure_event(group: str, error: str) -> dict:
    return {"FailureEvent": {"TestGroupID": group, "Error": error}}


def crash_event(group: str, error: str) -> dict:
    return {"CrashEvent": {"TestGroupID": group, "Error": error, "Stacktrace": ""}}


def collect_outcomes(events, result: "Result") -> None:
    """local_docker.go:216-255: count SuccessEvent per group; FailureEvent and CrashEvent count as
    reported but not ok; stop once every instance has reported; then update the outcome."""
    expecting = sum(g.total for g in result.outcomes.values())
    for e in events:
        if expecting <= 0:
            break
        ev = e["event"]
        if "SuccessEvent" in ev:
            result.outcomes[ev["SuccessEvent"]["TestGroupID"]].ok += 1
            expecting -= 1
        elif "FailureEvent" in ev or "CrashEvent" in ev:
            expecting -= 1
    result.update_outcome()


class PrettyPrinter:
    """pretty.go:39-232 for simulated instances: one line per event, ``%5.4fs %10s << id >> msg``
    with the elapsed time measured from the run's start (here: simulated time); an instance that
    ends without a success or failure event is INCOMPLETE; wait() reports "N nodes failed"."""

    def __init__(self, ow):
        self.ow = ow
        self.failed = 0
        self.count = 0

    def manage(self, instance_id: str, events) -> None:
        """processStdout for one instance (pretty.go:113-182)."""
        self.count += 1
        ok = failed = False
        for e in events:
            ev, ts = e["event"], e["ts"]
            if "SuccessEvent" in ev:
                ok = True
                self._print(instance_id, ts, EventType.Ok, "")
            elif "FailureEvent" in ev:
                failed = True
                self._print(instance_id, ts, EventType.Fail, ev["FailureEvent"]["Error"])
            elif "CrashEvent" in ev:
                failed = True
                self._print(instance_id, ts, EventType.Crash, ev["CrashEvent"]["Error"])
            elif "MessageEvent" in ev:
                self._print(instance_id, ts, EventType.Message, ev["MessageEvent"]["Message"])
            elif "StartEvent" in ev:
                self._print(instance_id, ts, EventType.Start, json.dumps(ev["StartEvent"]["Runenv"], sort_keys=True))
            else:
                self._print(instance_id, ts, EventType.InternalErr, f"unknown event: {ev}")
                return
        if not ok and not failed:
            self._print(instance_id, None, EventType.Incomplete, "")
        if not ok or failed:
            self.failed += 1

    def wait(self):
        """pretty.go:82-94: an error message if any instance failed, else None."""
        return f"{self.failed} nodes failed" if self.failed else None

    def _print(self, instance_id: str, ts_ns, et: EventType, msg: str) -> None:
        elapsed = max(0, ts_ns or 0) / 1e9
        self.ow.write(f"{elapsed:5.4f}s {_CLASS[et]:>10s} << {instance_id} >> {msg}\n")


@dataclass
class LocalMI355XRunnerConfig:
    """Coalesced from .env.toml [runners."local:mi355x"] and the composition's [global.run_config]
    (supervisor.go:561-579), exactly like the other runners' config types."""
    seed: int = 1
    num_gpus: int = 1
    window_ns: int = 1 * MS
    max_msgs_per_window: int = 1 << 18
    max_records: int = 1 << 20
    outputs_dir: str = ""
    pretty: bool = True          # print every instance's events (pretty.go) when an output writer is given


@dataclass
class RunGroup:
    id: str
    instances: int
    artifact_path: str = ""
    parameters: dict = field(default_factory=dict)
    resources: dict = field(default_factory=dict)
    profiles: dict = field(default_factory=dict)


@dataclass
class RunInput:
    run_id: str
    test_plan: str
    test_case: str
    total_instances: int
    groups: list
    runner_config: LocalMI355XRunnerConfig = field(default_factory=LocalMI355XRunnerConfig)
    env_config: dict = field(default_factory=dict)
    disable_metrics: bool = False


@dataclass
class GroupOutcome:
    total: int
    ok: int = 0


@dataclass
class Result:
    """runner.Result: outcome + per-group {total, ok} (common_result.go:8-58)."""
    outcome: str = OUTCOME_UNKNOWN
    outcomes: dict = field(default_factory=dict)
    journal: dict = field(default_factory=lambda: {"events": {}, "failures": []})

    def update_outcome(self) -> None:
        self.outcome = OUTCOME_SUCCESS
        for g in self.outcomes.values():
            if g.total != g.ok:
                self.outcome = OUTCOME_FAILURE
                return


@dataclass
class RunOutput:
    run_id: str
    result: Result


class LocalMI355XRunner:
    """api.Runner for simulated instances on MI355X."""

    def __init__(self, binding=None):
        self._binding = binding   # test infrastructure only (the CPU oracle); None = libtgsim.so
        self._outputs: dict[str, dict] = {}
        self._active = 0          # concurrently running simulations (data-subnet allocation)

    def id(self) -> str:
        return "local:mi355x"

    def config_type(self):
        return LocalMI355XRunnerConfig

    def compatible_builders(self) -> list[str]:
        # The artifact is not executed; any builder the plan supports may be named.
        return ["exec:go", "docker:go", "docker:generic"]

    def run(self, job: RunInput, ow=None) -> RunOutput:
        key = (job.test_plan, job.test_case)
        if key not in P.PLANS:
            raise ValueError(f"local:mi355x: no workload descriptor for plan {job.test_plan!r} case {job.test_case!r}")
        total = sum(g.instances for g in job.groups)
        if total != job.total_instances:
            raise ValueError(f"groups hold {total} instances, TotalInstances is {job.total_instances}")
        cfg = job.runner_config
        # the workload descriptors take one value per parameter for the whole run: a parameter the
        # groups set differently is ambiguous and fails the run if the descriptor reads it
        params, ambiguous = {}, set()
        for g in job.groups:
            for k, v in g.parameters.items():
                if k in params and params[k] != v:
                    ambiguous.add(k)
                params.setdefault(k, v)
        params = P.RunParams(params, ambiguous)
        result = Result(outcomes={g.id: GroupOutcome(total=g.instances) for g in job.groups})
        t0 = time.perf_counter()
        subnet, _ = next_data_network(self._active)
        prefix = 16 if total + 3 <= 1 << 16 else 32 - (total + 3 - 1).bit_length()  # wider for > 65533 instances
        self._active += 1
        try:
            env = P.PlanEnv(total, seed=cfg.seed, test_case=job.test_case, params=params, binding=self._binding,
                            window_ns=cfg.window_ns,
                            sim_kw=dict(max_msgs_per_window=cfg.max_msgs_per_window, max_records=cfg.max_records,
                                        data_subnet=int_to_ip(subnet.ip), data_prefix_len=prefix))
        except Exception:
            self._active -= 1
            raise
        crash = None
        try:
            try:
                ok = np.asarray(P.PLANS[key](env), bool)
            except P.PlanPanic as e:   # the test case panicked: every instance crashes
                crash = str(e)
                ok = np.zeros(total, bool)
            stats = env.sim.stats()
            sim_now = env.sim.now
            failures = list(env.failures)
        finally:
            env.close()
            self._active -= 1
        events = self._events(job, ok, sim_now, failures, crash)
        collect_outcomes((e for per in events for e in per[1]), result)
        result.journal["failures"] = failures
        result.journal["events"] = {"simulated_ns": str(sim_now), "wall_s": f"{time.perf_counter() - t0:.3f}"}
        self._outputs[job.run_id] = {"run_id": job.run_id, "plan": job.test_plan, "case": job.test_case,
                                     "result": _jsonable(asdict(result)), "stats": stats}
        if ow is not None:
            if cfg.pretty:
                pp = PrettyPrinter(ow)
                for iid, evs in events:
                    pp.manage(iid, evs)
                err = pp.wait()
                if err:
                    ow.write(f"{err}\n")
            ow.write(f"local:mi355x run {job.run_id}: {result.outcome}\n")
        return RunOutput(run_id=job.run_id, result=result)

    @staticmethod
    def _events(job: RunInput, ok, t_end: int, failures: list, crash: str | None = None) -> list:
        """Each simulated instance's runtime events: StartEvent at time 0, then SuccessEvent,
        FailureEvent or (the case panicked) CrashEvent at the plan's end (the instance's id is
        <group>[<index in group>])."""
        out, base = [], 0
        err = failures[0] if failures else "the instance did not complete the test case"
        for g in job.groups:
            runenv = {"TestPlan": job.test_plan, "TestCase": job.test_case, "TestRun": job.run_id,
                      "TestInstanceCount": job.total_instances, "TestGroupInstanceCount": g.instances}
            for i in range(g.instances):
                done = (crash_event(g.id, crash) if crash is not None else
                        success_event(g.id) if ok[base + i] else failure_event(g.id, err))
                out.append((f"{g.id}[{i}]", [{"ts": 0, "event": start_event(g.id, runenv)},
                                             {"ts": int(t_end), "event": done}]))
            base += g.instances
        return out

    def collect_outputs(self, run_id: str, w) -> None:
        """Writes a tar.gz with the run's result and counters (CollectOutputs, runner.go:31-33)."""
        if run_id not in self._outputs:
            raise KeyError(f"unknown run {run_id}")
        data = json.dumps(self._outputs[run_id], indent=1).encode()
        with tarfile.open(fileobj=w, mode="w:gz") as tar:
            info = tarfile.TarInfo(os.path.join(run_id, "result.json"))
            info.size = len(data)
            tar.addfile(info, io.BytesIO(data))


def _jsonable(x):
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, (np.integer,)):
        return int(x)
    return x
