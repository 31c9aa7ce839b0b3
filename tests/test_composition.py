"""Composition / manifest plumbing (testground_amd/composition.py): the
known answers of pkg/api/composition_test.go (unique group ids, the computed total, percentages
needing a total, test-parameter trickling and manifest defaults) restated on TOML inputs, and a
composition file run end to end through LocalMI355XRunner on the CPU oracle."""
import io

import pytest

from testground_amd import composition as CP
from testground_amd.runner import OUTCOME_SUCCESS, LocalMI355XRunner

MANIFEST = """
name = "benchmarks"

[defaults]
builder = "exec:go"
runner = "local:exec"

[builders."docker:go"]
enabled = true

[runners."local:docker"]
enabled = true

[runners."local:mi355x"]
enabled = true
window_ns = 2000000

[[testcases]]
name = "storm"
instances = { min = 1, max = 20000, default = 5 }

  [testcases.params]
  conn_count = { type = "int", default = 5 }
  conn_outgoing = { type = "int", default = 5 }
  conn_delay_ms = { type = "int", default = 5000 }
  data_size_kb = { type = "int", default = 128 }
  verbose = { type = "bool", default = false }
  region = { type = "string", default = "eu" }
"""

STORM = """
[metadata]
name = "storm-mi355x"

[global]
plan = "benchmarks"
case = "storm"
builder = "docker:go"
runner = "local:mi355x"
total_instances = 40

[global.run_config]
seed = 7

[global.run.test_params]
conn_outgoing = "3"
conn_delay_ms = "200"
data_size_kb = "8"

[[groups]]
id = "dialers"
instances = { percentage = 0.75 }

  [groups.run.test_params]
  role = "dialer"

[[groups]]
id = "listeners"
instances = { count = 10 }
"""


def test_groups_unique():
    """composition_test.go TestValidateGroupsUnique"""
    c = CP.parse_composition('[global]\nplan="p"\ncase="c"\nbuilder="docker:go"\nrunner="local:mi355x"\n'
                             '[[groups]]\nid="repeated"\ninstances={count=1}\n[[groups]]\nid="repeated"\n'
                             'instances={count=1}\n')
    with pytest.raises(ValueError, match="group ids not unique; found duplicate: repeated"):
        CP.validate_for_run(c)


def test_total_instances_computed_when_possible():
    """composition_test.go TestTotalInstancesIsComputedWhenPossible"""
    head = '[global]\nplan="p"\ncase="c"\nbuilder="docker:go"\nrunner="local:docker"\n'
    c = CP.parse_composition(head + '[[groups]]\nid="a"\nbuilder="docker:generic"\ninstances={count=3}\n'
                             '[[groups]]\nid="b"\ninstances={count=2}\n[[groups]]\nid="c"\ninstances={count=1}\n')
    CP.validate_for_run(c)
    assert c.global_.total_instances == 6
    c = CP.parse_composition(head + '[[groups]]\nid="a"\ninstances={count=3}\n'
                             '[[groups]]\nid="b"\ninstances={percentage=0.5}\n')
    with pytest.raises(ValueError, match="requires a total_instance configuration"):
        CP.validate_for_run(c)
    c = CP.parse_composition(head.replace('runner="local:docker"\n', 'runner="local:docker"\ntotal_instances=10\n') +
                             '[[groups]]\nid="a"\ninstances={count=3}\n[[groups]]\nid="b"\ninstances={percentage=0.5}\n')
    with pytest.raises(ValueError, match="total=10, calculated=8"):
        CP.validate_for_run(c)
    c = CP.parse_composition(head + '[[groups]]\nid="a"\ninstances={count=3, percentage=0.5}\n')
    with pytest.raises(ValueError, match="exactly one of count or percentage"):
        CP.validate_for_run(c)


def test_default_test_params_applied():
    """composition_test.go TestDefaultTestParamsApplied, plus JSON-encoded non-string defaults"""
    c = CP.parse_composition("""
[global]
plan = "foo_plan"
case = "foo_case"
total_instances = 3
builder = "docker:go"
runner = "local:docker"
[global.run.test_params]
param1 = "value1:default:composition"
param2 = "value2:default:composition"
param3 = "value3:default:composition"
[[groups]]
id = "all_set"
instances = { count = 1 }
[groups.run.test_params]
param1 = "value1:set"
param2 = "value2:set"
param3 = "value3:set"
[[groups]]
id = "none_set"
instances = { count = 1 }
[[groups]]
id = "first_set"
instances = { count = 1 }
[groups.run.test_params]
param1 = "value1:set"
""")
    m = CP.parse_manifest("""
name = "foo_plan"
[builders."docker:go"]
[runners."local:docker"]
[[testcases]]
name = "foo_case"
instances = { min = 1, max = 100 }
[testcases.params]
param4 = { type = "string", default = "value4:default:manifest" }
param5 = { type = "int", default = 10 }
param6 = { type = "bool", default = true }
""")
    CP.validate_for_run(c)
    r = CP.prepare_for_run(c, m)
    p = [g.run.test_params for g in r.groups]
    assert p[0] == {"param1": "value1:set", "param2": "value2:set", "param3": "value3:set",
                    "param4": "value4:default:manifest", "param5": "10", "param6": "true"}
    assert p[1] == {"param1": "value1:default:composition", "param2": "value2:default:composition",
                    "param3": "value3:default:composition", "param4": "value4:default:manifest",
                    "param5": "10", "param6": "true"}
    assert p[2]["param1"] == "value1:set" and p[2]["param2"] == "value2:default:composition"
    assert c.groups[1].run.test_params is None      # the input composition is not modified


def test_prepare_refusals():
    m = CP.parse_manifest(MANIFEST)
    c = CP.parse_composition(STORM.replace('runner = "local:mi355x"', 'runner = "local:zzz"'))
    CP.validate_for_run(c)
    with pytest.raises(ValueError, match=r"plan does not support runner local:zzz; supported: \[local:docker local:mi355x\]"):
        CP.prepare_for_run(c, m)
    # sort.SearchStrings returns the insertion index (composition.go:444): an unlisted runner that
    # sorts before the last listed one passes the check, exactly as in the reference
    for runner in ("cluster:k8s", "local:exec"):
        c = CP.parse_composition(STORM.replace('runner = "local:mi355x"', f'runner = "{runner}"'))
        CP.validate_for_run(c)
        assert CP.prepare_for_run(c, m).global_.runner == runner
    c = CP.parse_composition(STORM.replace('case = "storm"', 'case = "nope"'))
    CP.validate_for_run(c)
    with pytest.raises(ValueError, match="test case nope not found in plan benchmarks"):
        CP.prepare_for_run(c, m)
    c = CP.parse_composition(STORM.replace("total_instances = 40", "total_instances = 30000")
                             .replace("count = 10", "count = 7500"))
    CP.validate_for_run(c)
    with pytest.raises(ValueError, match=r"total instance count \(30000\) outside of allowable range \[1, 20000\]"):
        CP.prepare_for_run(c, m)


def test_run_input_from_composition():
    c = CP.parse_composition(STORM)
    CP.validate_for_run(c)
    r = CP.prepare_for_run(c, CP.parse_manifest(MANIFEST))
    env = {"runners": {"local:mi355x": {"seed": 3, "max_records": 1 << 18, "num_gpus": 1}}}
    job = CP.to_run_input(r, "run-1", env)
    assert [(g.id, g.instances) for g in job.groups] == [("dialers", 30), ("listeners", 10)]
    assert job.total_instances == 40 and job.test_plan == "benchmarks" and job.test_case == "storm"
    # composition run_config (seed 7) over .env.toml (seed 3); the manifest's runner section fills
    # window_ns; .env.toml's max_records stays
    assert job.runner_config.seed == 7 and job.runner_config.window_ns == 2_000_000
    assert job.runner_config.max_records == 1 << 18
    d, l = (g.parameters for g in job.groups)
    assert d["role"] == "dialer" and "role" not in l                    # group-only value
    assert d["data_size_kb"] == l["data_size_kb"] == "8" and d["conn_count"] == "5"   # manifest default
    assert d["conn_outgoing"] == l["conn_outgoing"] == "3"              # [global.run] trickled down
    assert d["verbose"] == "false" and d["region"] == "eu"


def test_composition_runs_on_the_runner(oracle):
    """the storm composition end to end: TOML -> ValidateForRun -> PrepareForRun -> RunInput ->
    local:mi355x (the CPU oracle stands in for the device here) -> every instance succeeds"""
    c = CP.parse_composition(STORM)
    CP.validate_for_run(c)
    job = CP.to_run_input(CP.prepare_for_run(c, CP.parse_manifest(MANIFEST)), "storm-run")
    out = io.StringIO()
    res = LocalMI355XRunner(binding=oracle).run(job, out)
    assert res.result.outcome == OUTCOME_SUCCESS
    assert {k: (v.total, v.ok) for k, v in res.result.outcomes.items()} == {"dialers": (30, 30), "listeners": (10, 10)}
    assert "local:mi355x run storm-run: success" in out.getvalue()


def test_groups_disagreeing_on_a_read_parameter_fail_the_run(oracle):
    c = CP.parse_composition(STORM.replace('role = "dialer"', 'role = "dialer"\n  conn_outgoing = "4"'))
    CP.validate_for_run(c)
    job = CP.to_run_input(CP.prepare_for_run(c, CP.parse_manifest(MANIFEST)), "ambiguous")
    with pytest.raises(ValueError, match="'conn_outgoing' differs between groups"):
        LocalMI355XRunner(binding=oracle).run(job)


@pytest.mark.gpu
def test_composition_runs_on_the_hip_runner(hip):
    c = CP.parse_composition(STORM)
    CP.validate_for_run(c)
    job = CP.to_run_input(CP.prepare_for_run(c, CP.parse_manifest(MANIFEST)), "storm-run-hip")
    res = LocalMI355XRunner(binding=hip).run(job, io.StringIO())
    assert res.result.outcome == OUTCOME_SUCCESS


def test_test_params_are_strings_as_in_go():
    """[groups.run.test_params] decodes into map[string]string: an unquoted value is an error."""
    with pytest.raises(ValueError, match="cannot load TOML value"):
        CP.parse_composition(STORM.replace('role = "dialer"', 'role = "dialer"\n  verbose = true'))


@pytest.mark.parametrize("value,text", [(10, "10"), (1.0, "1"), (1.5, "1.5"), (True, "true"), (0.1, "0.1"),
                                        (1e21, "1e+21"), (1e-7, "1e-7"), (2.5e-10, "2.5e-10"), (-3e-8, "-3e-8"), (123456789.0, "123456789"),
                                        ({"b": 1, "a": [1, 2.0]}, '{"a":[1,2],"b":1}'), ("x", "x")])
def test_manifest_defaults_marshal_like_go(value, text):
    """PrepareForRun JSON-encodes non-string defaults with encoding/json (composition.go:508-517):
    integral floats without a fraction, exponents in Go's form, map keys sorted."""
    m = CP.parse_manifest(MANIFEST)
    tc = m.test_case("storm")
    tc.parameters = {"p": CP.Parameter(type="x", default=value)}
    c = CP.parse_composition(STORM)
    CP.validate_for_run(c)
    assert CP.prepare_for_run(c, m).groups[0].run.test_params["p"] == text
