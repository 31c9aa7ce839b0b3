"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (oracle/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The oracle exposes the same entry points as libtgsim.so with the tgo_ prefix, so
``testground_amd.sim.Simulator(cfg, binding=oracle_binding())`` drives it through the identical
interface as the HIP path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "tgsim_oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB


_B = None


def oracle_binding():
    global _B
    if _B is None:
        from testground_amd import _abi
        _B = _abi.bind(build(), "tgo_", "oracle")
        lib = _B.cdll
        lib.tgo_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.tgo_philox4x32_10.restype = None
        lib.tgo_percentage2u32.argtypes = [C.c_float]
        lib.tgo_percentage2u32.restype = C.c_uint32
        lib.tgo_time2tick.argtypes = [C.c_uint32]
        lib.tgo_time2tick.restype = C.c_uint32
        lib.tgo_to_microseconds.argtypes = [C.c_int64]
        lib.tgo_to_microseconds.restype = C.c_uint32
        lib.tgo_ratecfg.argtypes = [C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.tgo_ratecfg.restype = None
        lib.tgo_derive_shape.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
        lib.tgo_derive_shape.restype = C.c_int
        lib.tgo_next_data_network.argtypes = [C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                              C.POINTER(C.c_uint32)]
        lib.tgo_next_data_network.restype = C.c_int
    return _B


def philox(ctr, key):
    lib = oracle_binding().cdll
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib.tgo_philox4x32_10(c, k, o)
    return list(o)


def percentage2u32(p: float) -> int:
    return oracle_binding().cdll.tgo_percentage2u32(p)


def derive_shape(shape) -> list[int] | int:
    out = (C.c_int64 * 10)()
    rc = oracle_binding().cdll.tgo_derive_shape(C.byref(shape), out)
    return rc if rc else list(out)
