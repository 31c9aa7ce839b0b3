#!/bin/bash
# Static check of the release hand-offs (tgsim_internal.h block_release_for_count):
# every L2 write-back (`buffer_wbl2`) an agent-scope release emits in the product kernels must be
# followed by its own `s_waitcnt vmcnt(0)` before the counting atomic. Compiles each source to gfx950
# device assembly (CPU only) and prints per source the write-backs and how many are followed by the wait.
set -e
cd "$(dirname "$0")/../testground_amd/csrc"
T=$(mktemp -d)
hipcc --version | grep -i "HIP version" || true
for f in tgsim_kernels tgsim_probe tgsim_storm tgsim_tcp tgsim_flood tgsim_topics tgsim_runtime; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --offload-device-only -S -o $T/$f.s $f.hip 2>/dev/null
  n=$(grep -c buffer_wbl2 $T/$f.s || true)
  w=$(grep -A1 buffer_wbl2 $T/$f.s | grep -c 's_waitcnt vmcnt(0)' || true)
  echo "$f.hip: buffer_wbl2 $n, followed by s_waitcnt vmcnt(0): $w"
  [ "$n" = "$w" ] || { echo "MISSING WAIT in $f"; grep -n -A2 buffer_wbl2 $T/$f.s; exit 1; }
done
rm -rf $T
