"""CPU: static checks of the gfx950 device assembly (hipcc cross-compiles here, no GPU needed).

* the ROCm 7.2 loop-exit miscompile: tools/loopexit_audit.py flags a lane mask
  computed inside a divergent loop and read after its exit. It must flag the standalone reproducer
  without the empty asm (tools/loopexit_repro.hip, which fails on the MI355X: profiles/r06/
  loopexit_repro.txt), pass it with the asm, and find nothing in the reaction kernels' sources;
* every agent-scope release's L2 write-back is followed by its wait (tools/fence_isa.sh's check).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _asm(src, out, *defs):
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only", "-S",
                           *defs, "-o", str(out), src], stderr=subprocess.DEVNULL)
    return str(out)


def test_loopexit_audit_flags_the_reproducer(tmp_path):
    import loopexit_audit as LA
    src = os.path.join(ROOT, "tools", "loopexit_repro.hip")
    bad = LA.audit(_asm(src, tmp_path / "w0.s", "-DWALK_ASM=0"))
    assert len(bad) == 1 and bad[0][3] == ["vcc"]
    assert LA.audit(_asm(src, tmp_path / "w1.s", "-DWALK_ASM=1")) == []


@pytest.mark.parametrize("name", ["tgsim_tcp", "tgsim_storm", "tgsim_probe", "tgsim_flood"])
def test_reaction_kernels_have_no_stale_loop_exit_mask(tmp_path, name):
    import loopexit_audit as LA
    s = _asm(os.path.join(ROOT, "testground_amd", "csrc", name + ".hip"), tmp_path / f"{name}.s")
    assert LA.audit(s) == []
    txt = open(s).read()
    assert txt.count("buffer_wbl2") == sum(1 for a, b in zip(txt.splitlines(), txt.splitlines()[1:])
                                           if "buffer_wbl2" in a and "s_waitcnt vmcnt(0)" in b)


def test_tcp_walk_without_asm_is_flagged(tmp_path):
    """The product's fast-retransmit walk is the site the asm protects: without it the audit finds it."""
    import loopexit_audit as LA
    s = _asm(os.path.join(ROOT, "testground_amd", "csrc", "tgsim_tcp.hip"), tmp_path / "t.s", "-DTGSIM_NO_WALK_ASM")
    hits = LA.audit(s)
    assert len(hits) == 1 and "k_tcp_conn_release" in hits[0][0]
