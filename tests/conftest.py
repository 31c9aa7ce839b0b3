import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and the built libtgsim.so")


@pytest.fixture(scope="session")
def oracle():
    from oracle.pyoracle import oracle_binding
    return oracle_binding()


@pytest.fixture(scope="session")
def hip():
    from testground_amd import _abi
    return _abi.hip_library()
