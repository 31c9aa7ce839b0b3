"""GPU parity: the HIP path (via the C ABI) against the CPU oracle on identical seeded inputs.
Bit-exact on every observable: statuses, delivery records (all fields), inbox offsets, counters,
sync sequence numbers and barrier release times."""
import pytest

from tests import scenarios as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_random_windows(hip, oracle, seed):
    S.assert_same(S.run_random(hip, seed), S.run_random(oracle, seed))


def test_random_windows_small_wheel(hip, oracle):
    kw = dict(wheel_slot_ns=3_000_000, wheel_slots=8)
    S.assert_same(S.run_random(hip, 11, cfg_kw=kw), S.run_random(oracle, 11, cfg_kw=kw))


def test_large_segments(hip, oracle):
    S.assert_same(S.run_heavy(hip, 7), S.run_heavy(oracle, 7))


def test_sync_service(hip, oracle):
    S.assert_same(S.run_sync(hip, 3), S.run_sync(oracle, 3))


def test_storm_rounds(hip, oracle):
    S.assert_same(S.run_storm(hip), S.run_storm(oracle))
