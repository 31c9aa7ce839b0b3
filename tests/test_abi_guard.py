"""C-ABI exception safety: no C++ exception crosses extern "C". An allocation
failure inside the library's host tables (forced through tgsim_debug_fail_alloc) is TGSIM_ENOMEM,
and the context keeps working - its tables are rebuilt into temporaries and swapped in whole."""
import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd import workloads as W
from testground_amd.network import int_to_ip
from testground_amd.sim import SimConfig, Simulator, make_rule

pytestmark = pytest.mark.gpu
MS = 1_000_000


def test_add_rules_bad_alloc_is_enomem_and_context_survives(hip):
    s = Simulator(SimConfig(n_instances=8, seed=1), binding=hip)
    ip = [int_to_ip(s.get_ip(g)) + "/32" for g in range(8)]
    s.add_rules(0, [make_rule(ip[1], A.FILTER_DROP)])
    s._check(hip.debug_fail_alloc(s._ctx, 1))
    with pytest.raises(A.TgsimError) as e:
        s.add_rules(0, [make_rule(ip[2], A.FILTER_REJECT), make_rule(ip[3], A.FILTER_DROP)])
    assert e.value.code == A.ENOMEM
    # the failed batch changed nothing; the next one applies normally
    s.enqueue([0, 0, 0], [1, 2, 3], [0, 1, 2], [10] * 3, [0] * 3)
    s.advance(1 * MS)
    assert list(s.status()) == [A.ST_DROPPED, A.ST_QUEUED, A.ST_QUEUED]
    s.add_rules(0, [make_rule(ip[2], A.FILTER_REJECT)])
    s.enqueue([0], [2], [3], [10], [1 * MS])
    s.advance(2 * MS)
    assert list(s.status()) == [A.ST_REJECTED]
    s.close()


def test_flood_set_graph_bad_alloc_keeps_the_previous_graph(hip):
    n = 64
    s = Simulator(SimConfig(n_instances=n, seed=1), binding=hip)
    off, nbr = W.random_regular_graph(n, 4, 5)
    s.flood_set_graph(off, nbr, 4)
    s._check(hip.debug_fail_alloc(s._ctx, 1))
    with pytest.raises(A.TgsimError) as e:
        s.flood_set_graph(off, nbr, 8)
    assert e.value.code == A.ENOMEM
    s.flood_publish([0], [0], 0, 64)          # the old graph (max_pubs 4) still serves
    s.advance(1 * MS)
    assert s.flood_react(64) > 0
    s.close()
