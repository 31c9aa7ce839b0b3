#!/usr/bin/env python3
"""Static audit for the ROCm 7.2 loop-exit miscompile (tools/loopexit_repro.hip).

The bad lowering: a lane-mask (`vcc` or an SGPR pair) written by a `v_cmp*` inside a divergent loop is
read after the loop's exit (`s_cbranch_execnz` back-edge, then `s_or_b64 exec, exec, ...`) without
being re-derived: it then holds only the lanes still active in the last iteration, so every lane that
left earlier loses its value. A correct lowering merges such a value into a mask every iteration
(s_andn2 / s_or with exec) or recomputes it after the loop from the VGPR it came from.

Compiles the product's HIP sources to gfx950 device assembly (CPU only) and lists, per kernel, each
loop exit whose following instructions read a compare mask defined inside the loop body before
redefining it. Usage: tools/loopexit_audit.py [file.s ...]   (no argument: the product sources)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["tgsim_kernels", "tgsim_probe", "tgsim_storm", "tgsim_tcp", "tgsim_flood", "tgsim_topics", "tgsim_runtime"]
CMP = re.compile(r"^\s*v_cmpx?_\S+\s+(vcc|s\[\d+:\d+\])")
LABEL = re.compile(r"^(\.LBB\d+_\d+|_Z\S+):")
BACK = re.compile(r"^\s*s_cbranch_execnz\s+(\.LBB\d+_\d+)")


def regs_read(line: str):
    parts = line.split(None, 1)
    if len(parts) < 2:
        return set(), None
    ops = [o.strip() for o in parts[1].split(",")]
    op = parts[0]
    dst = ops[0] if ops and not op.startswith(("s_cbranch", "global_store", "buffer_store", "ds_write",
                                                 "s_store")) else None
    srcs = set(ops[1:]) if dst else set(ops)
    # VOPC / v_cndmask / v_addc read vcc implicitly in their _e32 forms
    if op.endswith("_e32") and (op.startswith("v_cndmask") or op.startswith(("v_addc", "v_subb"))):
        srcs.add("vcc")
    return srcs, dst


def audit(asm_path: str):
    lines = [l.rstrip("\n") for l in open(asm_path)]
    lines = [l for l in lines if l.strip() and not l.strip().startswith((";", "."))
             or LABEL.match(l)]
    labels = {LABEL.match(l).group(1): i for i, l in enumerate(lines) if LABEL.match(l)}
    kernel, out = None, []
    for i, l in enumerate(lines):
        m = LABEL.match(l)
        if m and m.group(1).startswith("_Z"):
            kernel = m.group(1)
        b = BACK.match(l)
        if not b or b.group(1) not in labels or labels[b.group(1)] > i:
            continue
        body = lines[labels[b.group(1)]:i]
        defs = {CMP.match(x).group(1) for x in body if CMP.match(x)}
        if not defs:
            continue
        # the instructions after the exit's exec restore, until each mask is redefined
        j = i + 1
        if j < len(lines) and lines[j].strip().startswith("s_or_b64 exec, exec"):
            j += 1
        live = set(defs)
        for x in lines[j:j + 24]:
            if LABEL.match(x) or not live:
                break
            srcs, dst = regs_read(x.strip())
            hit = live & srcs
            if hit:
                out.append((kernel, b.group(1), x.strip(), sorted(hit)))
                break
            if dst in live:
                live.discard(dst)
    return out


def main():
    paths = sys.argv[1:]
    tmp = None
    if not paths:
        tmp = tempfile.mkdtemp()
        for f in SRCS:
            p = os.path.join(tmp, f + ".s")
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                                   "--offload-device-only", "-S", "-o", p,
                                   os.path.join(ROOT, "testground_amd", "csrc", f + ".hip")],
                                  stderr=subprocess.DEVNULL)
            paths.append(p)
    total = 0
    for p in paths:
        hits = audit(p)
        total += len(hits)
        print(f"{os.path.basename(p)}: {len(hits)} loop exit(s) reading an in-loop compare mask")
        for k, lab, ins, regs in hits:
            print(f"   {k} loop {lab}: `{ins}` reads {regs}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
