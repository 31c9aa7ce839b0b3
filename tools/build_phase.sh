#!/bin/bash
# Debug build with the phase clocks (-DTGSIM_PHASE_PROF) beside the product library:
# testground_amd/libtgsim_phase.so (load it with TGSIM_LIB=...).
set -e
cd "$(dirname "$0")/../testground_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -DTGSIM_PHASE_PROF -shared \
  -o ../libtgsim_phase.so tgsim_kernels.hip tgsim_runtime.hip tgsim_flood.hip tgsim_topics.hip tgsim_tcp.hip tgsim_probe.hip \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
