"""CPU: hand-computed known answers of the pinned semantics on the CPU oracle (the same cases run
on the GPU in tests/test_gpu_parity.py)."""
import pytest

from tests import semantics_cases as SC


@pytest.mark.parametrize("case", SC.CASES, ids=lambda f: f.__name__[5:])
def test_semantics_oracle(oracle, case):
    case(oracle)
