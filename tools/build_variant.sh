#!/bin/bash
# Experiment build of the product sources with extra defines, beside the product library:
#   tools/build_variant.sh <name> -DFOO [-DBAR=1 ...]  ->  testground_amd/libtgsim_<name>.so
# (load it with TGSIM_LIB=...; tools/gpu_ab.sh times it against the product build)
set -e
name=$1; shift
cd "$(dirname "$0")/../testground_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -shared \
  -o ../libtgsim_$name.so tgsim_kernels.hip tgsim_runtime.hip tgsim_flood.hip tgsim_topics.hip tgsim_tcp.hip tgsim_probe.hip \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
