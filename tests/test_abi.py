"""CPU: the C-ABI boundary. libtgsim.so loads without a GPU and exports every function
include/tgsim.h declares; the oracle exports the tgo_ twin of every data-path entry point; the
product path fails loudly (ENODEV) instead of falling back to a CPU implementation."""
import ctypes as C
import os

import pytest

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# entry points that only the device library has (no CPU meaning): streams, device buffers, profiling
HIP_ONLY = {"tgsim_version", "tgsim_abi_version", "tgsim_set_stream", "tgsim_shard_range", "tgsim_sync",
            "tgsim_enqueue_device", "tgsim_deliveries_device", "tgsim_profile_set", "tgsim_profile_read",
            "tgsim_kernel_classes", "tgsim_kernel_name", "tgsim_set_exchange_buffers",
            "tgsim_advance_begin_device", "tgsim_storm_release_device", "tgsim_comm_unique_id", "tgsim_comm_init",
            "tgsim_sync_subscribe_device", "tgsim_topic_arena_device",
            # checkpoint / resume is a runtime facility of the product library; the oracle's run is the
            # uninterrupted reference a restored run is compared with (tests/test_snapshot.py)
            "tgsim_snapshot", "tgsim_restore",
            # allocation-failure injection into the library's C++ host tables (no C++ in the oracle)
            "tgsim_debug_fail_alloc",
            # device address of the proposed window end (tgsim_advance_begin_device has no oracle twin)
            "tgsim_probe_state_device", "tgsim_storm_state_device",
            # implementation counters of the device pipeline (bench.py's per-kernel byte attribution)
            "tgsim_kernel_counters"}


def test_header_declares_expected_surface():
    syms = A.header_symbols()
    for s in ("tgsim_create", "tgsim_destroy", "tgsim_configure_network", "tgsim_enqueue", "tgsim_advance",
              "tgsim_advance_begin", "tgsim_advance_end", "tgsim_sync_signal", "tgsim_sync_barrier",
              "tgsim_copy_deliveries", "tgsim_last_error", "tgsim_horizon"):
        assert s in syms


def test_library_exports_every_header_symbol():
    assert os.path.exists(A.LIB_PATH), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    lib = C.CDLL(A.LIB_PATH)
    missing = [s for s in A.header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_oracle_exports_twins():
    from oracle.pyoracle import oracle_binding
    lib = oracle_binding().cdll
    missing = [s for s in A.header_symbols() if s not in HIP_ONLY and not hasattr(lib, "tgo_" + s[len("tgsim_"):])]
    assert not missing, missing


def test_binding_covers_header():
    hip = A.hip_library()
    bound = {"tgsim_" + k for k in list(A._SIGS) + list(A._SIGS_HIP)}
    assert set(A.header_symbols()) <= bound, set(A.header_symbols()) - bound
    assert hip.version().decode().startswith("tgsim-mi355x")
    assert hip.abi_version() == 2
    names = [hip.kernel_name(k).decode() for k in range(hip.kernel_classes())]
    assert "k_extract_shape" in names and "k_emit_bucket" in names and "k_tb_bucket" in names


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the header structs have the C compiler's sizes and field offsets."""
    import subprocess
    structs = {"tgsim_link_shape": A.LinkShape, "tgsim_link_rule": A.LinkRule,
               "tgsim_network_config": A.NetworkConfig, "tgsim_config": A.Config, "tgsim_msg_soa": A.MsgSoA,
               "tgsim_tcp_config": A.TcpConfig, "tgsim_tcp_stats": A.TcpStats,
               "tgsim_delivery_soa": A.DeliverySoA, "tgsim_stats": A.Stats, "tgsim_transport": A.Transport,
               "tgsim_probe_config": A.ProbeConfig, "tgsim_storm_config": A.StormConfig,
               "tgsim_storm_totals": A.StormTotals}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "tgsim.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, f"{cname}.{f}"


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device behaviour")
def test_product_path_fails_loudly_without_gpu():
    with pytest.raises(A.TgsimError) as e:
        Simulator(SimConfig(n_instances=4))
    assert e.value.code == A.ENODEV


def test_create_rejects_bad_config(oracle):
    for kw in (dict(n_instances=0), dict(n_instances=4, n_shards=2, shard_id=2),
               dict(n_instances=70000, data_prefix_len=16), dict(n_instances=4, data_prefix_len=31)):
        with pytest.raises(A.TgsimError) as e:
            Simulator(SimConfig(**kw), binding=oracle)
        assert e.value.code == A.EINVAL


def test_one_rccl_per_process():
    """libtgsim.so needs librccl.so.1 (soname); torch's bundled RCCL has the same soname, so in a
    process that imported torch first (bench.py, the tests) the dynamic loader satisfies libtgsim's
    dependency with torch's copy: exactly one RCCL build is mapped. Without torch
    (a Go runner) /opt/rocm's is the one."""
    import subprocess
    import sys
    code = ("import torch, ctypes, sys; ctypes.CDLL(sys.argv[1]); "
            "print(sorted({l.split()[-1] for l in open('/proc/self/maps') if 'librccl' in l}))")
    out = subprocess.run([sys.executable, "-c", code, A.LIB_PATH], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    paths = eval(out.stdout.strip().splitlines()[-1])
    assert len(paths) == 1, paths
