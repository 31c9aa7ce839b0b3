"""testground_amd — MI355X-native simulator for Testground's per-message data path (runner local:mi355x).

HIP kernels + C ABI live in testground_amd/csrc (built to testground_amd/libtgsim.so); this package
holds the ctypes binding and the host-side mirror of the reference interfaces (sidecar.Network,
sync.Client, api.Runner). See DESIGN.md.
"""
from . import _abi  # noqa: F401
from .sim import SimConfig, Simulator, make_rule, make_shape, ip_to_int, int_to_ip  # noqa: F401

__version__ = "0.1.0"
