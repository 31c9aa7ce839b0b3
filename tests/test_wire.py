"""network.Config on the wire (testground_amd/network.py to_wire / from_wire; sidecar wire mode):
the JSON a config travels in on the sync topic network:<hostname> (sidecar_handler.go:49-80),
decoded as Go's encoding/json would (case-insensitive keys), the JS SDK's literal of
plans/example-js/pingpong.js:25-33 among the inputs; plans run with configs routed through the
device-resident topics give the same answers as the direct path."""
import json

import numpy as np
import pytest

from testground_amd import plans as P
from testground_amd.network import (MS, AllowAll, Config, DenyAll, Drop, IPNet, LinkRule, LinkShape, Reject,
                                    ipnet_from_wire)


def test_js_sdk_literal():
    """plans/example-js/pingpong.js:25-33 (the object the JS plan hands network.configureNetwork),
    then the IP change of :49-50 (IPv4 as "a.b.c.d/len")"""
    js = {"network": "default", "enable": True,
          "default": {"latency": 100 * 1000 * 1000, "bandwidth": 1 << 20},
          "callbackState": "network-configured", "routingPolicy": "deny_all"}
    c = Config.from_wire(json.loads(json.dumps(js)))
    assert c.network == "default" and c.enable and c.callback_state == "network-configured"
    assert c.default.latency == 100 * MS and c.default.bandwidth == 1 << 20 and c.routing_policy == "deny_all"
    assert c.ipv4 is None and c.rules == []
    js["IPv4"] = "16.0.1.2/16"
    js["callbackState"] = "ip-changed"
    c = Config.from_wire(js)
    assert c.ipv4 == IPNet.parse("16.0.1.2/16") and c.callback_state == "ip-changed"


def test_go_json_round_trip_and_case_insensitive_keys():
    c = Config(network="default", enable=True, routing_policy=AllowAll, callback_state="s",
               default=LinkShape(latency=50 * MS, jitter=10 * MS, loss=1.0, duplicate=5.0, duplicate_corr=25.0),
               rules=[LinkRule(IPNet.parse("16.0.0.5/32"), LinkShape(filter=Drop)),
                      LinkRule(IPNet.parse("16.0.8.0/24"), LinkShape(filter=Reject))],
               ipv4=IPNet.parse("16.0.3.9/16"), callback_target=7)
    w = c.to_wire()
    assert w["IPv4"] == {"IP": "16.0.3.9", "Mask": "//8AAA=="} and w["rules"][0]["Subnet"]["Mask"] == "/////w=="
    assert w["rules"][0]["Filter"] == 2 and w["default"]["Latency"] == 50 * MS and "callback_target" not in w
    back = Config.from_wire(json.loads(json.dumps(w)))
    c.callback_target = 0                                  # json:"-": never travels
    assert back == c
    shouty = json.loads(json.dumps(w).replace('"Latency"', '"LATENCY"').replace('"enable"', '"Enable"'))
    assert Config.from_wire(shouty) == back
    with pytest.raises(ValueError):
        ipnet_from_wire({"IP": "16.0.0.0", "Mask": "/wD/AA=="})  # 255.0.255.0: not a prefix mask


@pytest.mark.parametrize("plan,case", [("network", "ping-pong"), ("network", "traffic-blocked"),
                                       ("splitbrain", "reject")])
def test_plans_over_the_config_topics(oracle, plan, case):
    n = 2 if plan == "network" and case == "ping-pong" else 12
    runs = []
    for wire in ("false", "true"):
        env = P.PlanEnv(n, seed=1, test_case=case, params={"sidecar_wire": wire}, binding=oracle)
        ok = np.asarray(P.PLANS[(plan, case)](env), bool)
        runs.append((ok, env.sim.stats(), env.sim.now))
        if wire == "true":
            assert env.sidecar.wire and sum(env.sync.count("topic:" + env.sidecar.topic(i)) for i in range(n)) > 0
        env.close()
    assert runs[0][0].all() and np.array_equal(runs[0][0], runs[1][0])
    assert runs[0][1] == runs[1][1] and runs[0][2] == runs[1][2]


@pytest.mark.gpu
def test_pingpong_over_the_config_topics_hip(hip):
    env = P.PlanEnv(2, seed=1, test_case="ping-pong", params={"sidecar_wire": "true"}, binding=hip)
    assert np.asarray(P.pingpong(env), bool).all()
    env.close()
