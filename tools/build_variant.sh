#!/bin/bash
# Experiment build of the product sources with extra defines, beside the product library:
#   tools/build_variant.sh <name> -DFOO [-DBAR=1 ...]  ->  testground_amd/libtgsim_<name>.so
# (load it with TGSIM_LIB=...; `tools/gpu.sh ab` times it against the product build;
#  tools/build_variant.sh phase -DTGSIM_PHASE_PROF is the phase-clock build of tools/phase_probe.py)
set -e
name=$1; shift
make -s -j8 -C "$(dirname "$0")/../testground_amd/csrc" ARCH=gfx950 OUT=../libtgsim_$name.so OBJDIR=build_$name \
  EXTRA="$*"
