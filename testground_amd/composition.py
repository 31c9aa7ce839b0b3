"""Composition and manifest plumbing for ``local:mi355x``: what happens
between ``testground run composition -f <file> --runner local:mi355x`` and ``api.Runner.Run``.

* the composition TOML (``pkg/api/composition.go:41-151``: ``[metadata]``, ``[global]`` with
  ``plan`` / ``case`` / ``total_instances`` / ``builder`` / ``runner`` / ``run_config`` / ``run``,
  ``[[groups]]`` with ``instances = {count | percentage}`` and ``[groups.run]``);
* ``validate_for_run`` = ``Composition.ValidateForRun`` (``composition.go:291-320`` + the struct
  validation it runs: required plan / case / runner, at least one group, count xor percentage
  (``ValidateInstances`` ``:555-567``), unique group ids and a builder per group
  (``Groups.Validate`` ``:21-40``)): group sizes from count or round(percentage * total), a
  percentage needs ``total_instances``, the computed total must equal a given one;
* ``prepare_for_run`` = ``Composition.PrepareForRun`` (``composition.go:413-530``) against the plan's
  manifest (``pkg/api/manifest.go:13-49``): the test case exists, the runner is one the manifest
  enables, the manifest's run config fills keys the composition leaves unset, the instance count is
  within the case's bounds, the global ``[global.run]`` artifact / test params / profiles trickle
  into groups that do not set them, and the case's parameter defaults fill absent test params
  (strings as they are, everything else JSON-encoded);
* ``to_run_input`` = the run input ``Engine.doRun`` builds (``pkg/engine/supervisor.go:553-602``): the
  runner config coalesced from ``.env.toml``'s ``[runners."local:mi355x"]`` then the composition's
  ``[global.run_config]`` (the composition wins) into ``LocalMI355XRunnerConfig``, one ``RunGroup``
  per group.

Errors are ``ValueError`` with the reference's messages. A plan runs on ``local:mi355x`` once its
manifest enables that runner (``[runners."local:mi355x"] enabled = true``)."""
from __future__ import annotations

import bisect
import copy
import json
import math
from dataclasses import dataclass, field, fields

import numpy as np
import tomli

from .runner import LocalMI355XRunnerConfig, RunGroup, RunInput


@dataclass
class Instances:
    count: int = 0
    percentage: float = 0.0


@dataclass
class Run:
    artifact: str = ""
    test_params: dict | None = None
    profiles: dict | None = None


@dataclass
class Group:
    id: str
    instances: Instances = field(default_factory=Instances)
    builder: str = ""
    build_config: dict | None = None
    resources: dict = field(default_factory=dict)
    run: Run = field(default_factory=Run)
    calculated_instances: int = 0   # set by validate_for_run (CalculatedInstanceCount)


@dataclass
class Global:
    plan: str = ""
    case: str = ""
    total_instances: int = 0
    builder: str = ""
    runner: str = ""
    build_config: dict | None = None
    run_config: dict | None = None
    run: Run | None = None
    disable_metrics: bool = False


@dataclass
class Composition:
    global_: Global
    groups: list
    metadata: dict = field(default_factory=dict)


@dataclass
class Parameter:
    type: str = ""
    desc: str = ""
    unit: str = ""
    default: object = None


@dataclass
class TestCase:
    name: str
    minimum: int = 0
    maximum: int = 0
    parameters: dict = field(default_factory=dict)


@dataclass
class Manifest:
    name: str
    builders: dict = field(default_factory=dict)
    runners: dict = field(default_factory=dict)
    testcases: list = field(default_factory=list)

    def test_case(self, name: str) -> TestCase | None:
        return next((tc for tc in self.testcases if tc.name == name), None)


def _run(d: dict | None) -> Run:
    d = d or {}
    return Run(artifact=d.get("artifact", ""), test_params=_strs(d.get("test_params")),
               profiles=_strs(d.get("profiles")))


def _strs(m):
    """A TOML table decoded into Go's map[string]string: a non-string value is a decoding error
    there (BurntSushi/toml refuses to store an integer, float, boolean or table in a string)."""
    if m is None:
        return None
    out = {}
    for k, v in m.items():
        if not isinstance(v, str):
            raise ValueError(f"toml: cannot load TOML value of type {type(v).__name__} into a Go string "
                             f"(key {k!r}); quote the value")
        out[str(k)] = v
    return out


def _go_float(x: float) -> str:
    """encoding/json's float64 text: the shortest round-trip digits, 'f' form for magnitudes in
    [1e-6, 1e21) (so 1.0 is "1"), else 'e' form: "1e+21", and "1e-7" (a negative exponent's leading
    zero is dropped, encoding/json's "e-09 to e-9" clean-up)."""
    if x != x or x in (float("inf"), float("-inf")):
        raise ValueError(f"json: unsupported value: {x}")
    if x == 0 or 1e-6 <= abs(x) < 1e21:
        return np.format_float_positional(x, trim="-")
    s = np.format_float_scientific(x, trim="-", exp_digits=2)
    # encoding/json "clean up e-09 to e-9": a negative exponent loses its leading zero (1e-7);
    # positive ones keep two digits (1e+21)
    if len(s) >= 4 and s[-4:-2] == "e-" and s[-2] == "0":
        s = s[:-2] + s[-1]
    return s


def _go_json(v) -> str:
    """json.Marshal of a TOML-decoded interface{} value: map keys sorted, floats as Go prints them."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return _go_float(v)
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False).replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
    if v is None:
        return "null"
    if isinstance(v, dict):
        return "{" + ",".join(f"{_go_json(str(k))}:{_go_json(v[k])}" for k in sorted(v)) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_go_json(x) for x in v) + "]"
    if hasattr(v, "isoformat"):   # TOML datetimes: time.Time marshals as RFC 3339
        return json.dumps(v.isoformat())
    raise ValueError(f"json: unsupported type {type(v).__name__}")


def parse_composition(text: str) -> Composition:
    doc = tomli.loads(text)
    g = doc.get("global", {})
    glob = Global(plan=g.get("plan", ""), case=g.get("case", ""), total_instances=int(g.get("total_instances", 0)),
                  builder=g.get("builder", ""), runner=g.get("runner", ""), build_config=g.get("build_config"),
                  run_config=g.get("run_config"), run=_run(g["run"]) if "run" in g else None,
                  disable_metrics=bool(g.get("disable_metrics", False)))
    groups = []
    for gr in doc.get("groups", []):
        inst = gr.get("instances", {})
        groups.append(Group(id=gr.get("id", ""), instances=Instances(int(inst.get("count", 0)),
                                                                      float(inst.get("percentage", 0.0))),
                            builder=gr.get("builder", ""), build_config=gr.get("build_config"),
                            resources=dict(gr.get("resources", {})), run=_run(gr.get("run"))))
    return Composition(global_=glob, groups=groups, metadata=dict(doc.get("metadata", {})))


def load_composition(path: str) -> Composition:
    with open(path, encoding="utf-8") as f:
        return parse_composition(f.read())


def parse_manifest(text: str) -> Manifest:
    doc = tomli.loads(text)
    cases = []
    for tc in doc.get("testcases", []):
        inst = tc.get("instances", {})
        params = {n: Parameter(type=p.get("type", ""), desc=p.get("desc", ""), unit=p.get("unit", ""),
                               default=p.get("default")) for n, p in tc.get("params", {}).items()}
        cases.append(TestCase(name=tc["name"], minimum=int(inst.get("min", 0)), maximum=int(inst.get("max", 0)),
                              parameters=params))
    return Manifest(name=doc.get("name", ""), builders=dict(doc.get("builders", {})),
                    runners=dict(doc.get("runners", {})), testcases=cases)


def validate_for_run(c: Composition) -> None:
    """Composition.ValidateForRun (composition.go:291-320); fills calculated_instances and, when
    it was 0, global_.total_instances."""
    g = c.global_
    for name, v in (("Plan", g.plan), ("Case", g.case), ("Runner", g.runner)):
        if not v:
            raise ValueError(f"Key: 'Composition.Global.{name}' Error:Field validation for '{name}' failed on the 'required' tag")
    if not c.groups:
        raise ValueError("Key: 'Composition.Groups' Error:Field validation for 'Groups' failed on the 'gt' tag")
    for gr in c.groups:
        i = gr.instances
        if (i.count == 0 or i.percentage == 0) and (i.count + i.percentage > 0):
            continue
        raise ValueError(f"group {gr.id}: instances need exactly one of count or percentage")
    total = g.total_instances
    computed = 0
    for gr in c.groups:
        if gr.instances.percentage > 0 and total == 0:
            raise ValueError("groups count percentage requires a total_instance configuration")
        gr.calculated_instances = gr.instances.count or int(math.floor(gr.instances.percentage * total + 0.5))
        computed += gr.calculated_instances
    if total > 0 and total != computed:
        raise ValueError(f"sum of calculated instances per group doesn't match total; total={total}, calculated={computed}")
    g.total_instances = computed
    seen = set()
    for gr in c.groups:
        if gr.id in seen:
            raise ValueError(f"group ids not unique; found duplicate: {gr.id}")
        seen.add(gr.id)
    for gr in c.groups:
        if not gr.builder and not g.builder:
            raise ValueError(f"group {gr.id} is missing a builder")


def prepare_for_run(c: Composition, manifest: Manifest) -> Composition:
    """Composition.PrepareForRun (composition.go:413-530): a prepared copy; c is unchanged."""
    c = copy.deepcopy(c)
    g = c.global_
    g.plan = manifest.name
    tc = manifest.test_case(g.case)
    if tc is None:
        raise ValueError(f"test case {g.case} not found in plan {manifest.name}")
    if not manifest.runners:
        raise ValueError("plan supports no runners; review the manifest")
    runners = sorted(manifest.runners)
    # sort.SearchStrings(runners, runner) == len(runners) (composition.go:444): the insertion index,
    # so an unlisted runner that sorts before the last listed one passes this check, as it does there
    if bisect.bisect_left(runners, g.runner) == len(runners):
        raise ValueError(f"plan does not support runner {g.runner}; supported: [{' '.join(runners)}]")
    rcfg = manifest.runners.get(g.runner)
    if rcfg:
        g.run_config = dict(g.run_config or {})
        for k, v in rcfg.items():
            g.run_config.setdefault(k, v)
    t = g.total_instances
    if t < tc.minimum or t > tc.maximum:
        raise ValueError(f"total instance count ({t}) outside of allowable range [{tc.minimum}, {tc.maximum}] "
                         f"for test case {tc.name}")

    def trickle(src, dst):
        if dst is None:
            return dict(src or {})
        for k, v in (src or {}).items():
            dst.setdefault(k, v)
        return dst

    if g.run is not None:
        for gr in c.groups:
            if not gr.run.artifact:
                gr.run.artifact = g.run.artifact
            gr.run.test_params = trickle(g.run.test_params, gr.run.test_params)
            gr.run.profiles = trickle(g.run.profiles, gr.run.profiles)
    defaults = {n: (p.default if isinstance(p.default, str) else _go_json(p.default))
                for n, p in tc.parameters.items()}
    for gr in c.groups:
        if gr.run.test_params is None:
            gr.run.test_params = {}
        for k, v in defaults.items():
            gr.run.test_params.setdefault(k, v)
    return c


def coalesce_runner_config(env_runner_cfg: dict | None, composition_run_config: dict | None) -> LocalMI355XRunnerConfig:
    """CoalescedConfig (supervisor.go:553-579): .env.toml's [runners."local:mi355x"], overridden by the
    composition's [global.run_config], into the runner's config type (unknown keys are ignored, as
    the TOML decoding into the struct does)."""
    merged = {}
    for m in (env_runner_cfg or {}, composition_run_config or {}):
        merged.update(m)
    known = {f.name: f.type for f in fields(LocalMI355XRunnerConfig)}
    kw = {}
    for k, v in merged.items():
        if k not in known:
            continue
        kw[k] = bool(v) if known[k] in (bool, "bool") else (str(v) if known[k] in (str, "str") else int(v))
    return LocalMI355XRunnerConfig(**kw)


def to_run_input(c: Composition, run_id: str, env_config: dict | None = None) -> RunInput:
    """The RunInput Engine.doRun hands the runner (supervisor.go:580-602) for a validated, prepared
    composition."""
    env_config = env_config or {}
    rcfg = coalesce_runner_config(env_config.get("runners", {}).get(c.global_.runner), c.global_.run_config)
    groups = [RunGroup(id=gr.id, instances=gr.calculated_instances, artifact_path=gr.run.artifact,
                       parameters=dict(gr.run.test_params or {}), resources=dict(gr.resources),
                       profiles=dict(gr.run.profiles or {})) for gr in c.groups]
    return RunInput(run_id=run_id, test_plan=c.global_.plan, test_case=c.global_.case,
                    total_instances=c.global_.total_instances, groups=groups, runner_config=rcfg,
                    env_config=env_config, disable_metrics=c.global_.disable_metrics)
