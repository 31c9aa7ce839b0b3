"""CPU: the oracle's primitives against independent known answers.

* Philox4x32-10: the Random123 published known-answer vectors (Salmon et al., SC'11, kat_vectors)
  and 64 vectors from rocRAND's host engine (tests/golden/philox_rocrand.json), plus a pure-Python
  restatement.
* netlink/kernel conversions [EXT]: Percentage2u32 against a numpy float32
  restatement, time2tick, toMicroseconds (pkg/sidecar/link.go:143-151), psched ratecfg.
* pkg/runner/common_test.go:14-20: the data-subnet allocation table.
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O
from testground_amd import _abi as A
from testground_amd.sim import make_shape

HERE = os.path.dirname(os.path.abspath(__file__))
M32 = 0xFFFFFFFF

# Random123 kat_vectors, philox4x32_10 (ctr, key, expected)
RANDOM123_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([M32, M32, M32, M32], [M32, M32], [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


def py_philox(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & M32
            k1 = (k1 + 0xBB67AE85) & M32
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
    return [c0, c1, c2, c3]


@pytest.mark.parametrize("ctr,key,want", RANDOM123_KAT)
def test_philox_random123_kat(ctr, key, want):
    assert O.philox(ctr, key) == want
    assert py_philox(ctr, key) == want


def test_philox_matches_rocrand_host_engine():
    with open(os.path.join(HERE, "golden", "philox_rocrand.json")) as f:
        vec = json.load(f)
    assert len(vec) == 64
    for v in vec:
        assert O.philox(v["ctr"], v["key"]) == v["out"]
        assert py_philox(v["ctr"], v["key"]) == v["out"]


def np_percentage2u32(p: float) -> int:
    """netlink Percentage2u32: 100 -> MaxUint32, else uint32(float32(MaxUint32) * (p/100)) in float32."""
    if np.float32(p) == np.float32(100.0):
        return M32
    v = np.float32(4294967296.0) * (np.float32(p) / np.float32(100.0))
    return int(np.int64(v)) & M32 if v < 2 ** 63 else 0


@pytest.mark.parametrize("p", [0.0, 1e-6, 0.1, 0.5, 1.0, 2.0, 5.0, 10.0, 20.0, 25.0, 33.3, 50.0, 99.0, 99.9999, 100.0])
def test_percentage2u32(p):
    assert O.percentage2u32(p) == np_percentage2u32(p)


def test_percentage2u32_known_answers():
    assert O.percentage2u32(0.0) == 0
    assert O.percentage2u32(100.0) == M32
    assert O.percentage2u32(50.0) == 0x80000000
    # float32(2^32) * 0.25 is exact
    assert O.percentage2u32(25.0) == 0x40000000


def test_time_conversions():
    lib = O.oracle_binding().cdll
    assert lib.tgo_time2tick(100_000) == 1_562_500          # 100 ms in 64-ns ticks
    assert lib.tgo_time2tick(1) == 15                       # 15.625 truncated
    assert lib.tgo_to_microseconds(100_000_000) == 100_000
    assert lib.tgo_to_microseconds(1_999) == 1              # Duration.Microseconds truncates
    assert lib.tgo_to_microseconds(10 ** 18) == M32         # link.go:147-149 cap
    assert lib.tgo_to_microseconds(-5_000) == (-5) & M32    # uint32() of a negative value wraps


def test_derive_shape_known_answers():
    mu, sigma, loss_t, dup_t, cor_t, reo_t, mult, shift, tau, limited = O.derive_shape(
        make_shape(latency_ns=100_000_000, jitter_ns=10_000_000, bandwidth_bps=1 << 20, loss=50.0))
    assert mu == 100_000_000 and sigma == 10_000_000       # ticks << 6 round-trips whole milliseconds
    assert loss_t == 0x80000000 and dup_t == 0 and cor_t == 0 and reo_t == 0
    assert limited == 1
    # 1 Mibit/s = 131072 B/s: 1 byte costs 1e9/131072 = 7629.39 ns
    assert ((1 * mult) >> shift) in (7629, 7630)
    assert (((1500 * mult) >> shift) - 11_444_091) ** 2 <= 4
    # zero latency: jitter is kept in microseconds (netlink NewNetem converts it only if latency > 0)
    out = O.derive_shape(make_shape(latency_ns=0, jitter_ns=2_000_000))
    assert out[0] == 0 and out[1] == (2_000 << 6)
    # unlimited bandwidth
    assert O.derive_shape(make_shape())[9] == 0


def test_derive_shape_rejects():
    assert O.derive_shape(make_shape(bandwidth_bps=7)) == A.EINVAL      # 7 bits/s -> rate 0 B/s
    assert isinstance(O.derive_shape(make_shape(duplicate_corr=1.0)), list)  # correlated netem: supported


# pkg/runner/common_test.go:14-20
@pytest.mark.parametrize("n,subnet,gateway,err", [
    (0, "16.0.0.0/16", "16.0.0.1", False), (1, "16.1.0.0/16", "16.1.0.1", False),
    (2, "16.2.0.0/16", "16.2.0.1", False), (255, "16.255.0.0/16", "16.255.0.1", False),
    (256, "17.0.0.0/16", "17.0.0.1", False), (4095, "31.255.0.0/16", "31.255.0.1", False),
    (4096, "", "", True)])
def test_next_data_network(n, subnet, gateway, err):
    import ctypes as C
    from testground_amd.network import int_to_ip
    from testground_amd.runner import next_data_network
    lib = O.oracle_binding().cdll
    s, p, g = C.c_uint32(), C.c_uint32(), C.c_uint32()
    rc = lib.tgo_next_data_network(n, C.byref(s), C.byref(p), C.byref(g))
    if err:
        assert rc != 0
        with pytest.raises(ValueError):
            next_data_network(n)
        return
    assert rc == 0
    assert f"{int_to_ip(s.value)}/{p.value}" == subnet and int_to_ip(g.value) == gateway
    net, gw = next_data_network(n)
    assert str(net) == subnet and int_to_ip(gw) == gateway
