#!/bin/bash
# Builds testground_amd/libtgsim_<name>.so with extra -D flags (A/B experiments only).
# usage: scripts/build_variant.sh NAME -DTGSIM_DEFER=0 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
d=/tmp/tgv_$name; mkdir -p $d
for src in tgsim_kernels.hip tgsim_engine.cpp tgsim_bridge.cpp tgsim_comm.cpp; do
  dev=""; [ "${src##*.}" = hip ] && dev="-mllvm -amdgpu-use-amdgpu-trackers=1"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result $dev "$@" -c testground_amd/csrc/$src -o $d/${src%.*}.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o testground_amd/libtgsim_$name.so $d/*.o
