"""CPU: the oracle reproduces the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py): every observable of the seeded scenarios and the plan outcomes.
The GPU tests check the HIP library against the same files."""
import pytest

from tests import golden_check as GC
from tests.golden import make_golden as G


@pytest.mark.parametrize("name", [s[0] for s in G.SCENARIOS])
def test_oracle_matches_golden_scenario(oracle, name):
    assert GC.check_scenario(oracle, name) > 0


def test_oracle_matches_golden_plans(oracle):
    GC.check_plans(oracle)
