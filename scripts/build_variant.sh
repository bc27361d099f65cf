#!/bin/bash
# A/B builds: testground_amd/libtgsim_<name>.so from the current sources with extra compiler flags
# (e.g. -DTGSIM_X), for scripts/ab.sh; PROMOTE_ALLOCA=1 lets LLVM promote private arrays to LDS.  usage: build_variant.sh NAME [FLAGS...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
B=testground_amd/build_$name; mkdir -p $B
for f in tgsim_kernels.hip tgsim_engine.cpp tgsim_bridge.cpp tgsim_comm.cpp; do
  dev=""
  if [ "${f##*.}" = hip ]; then
    dev="-mllvm -amdgpu-use-amdgpu-trackers=1"
    [ -z "$PROMOTE_ALLOCA" ] && dev="$dev -mllvm -disable-promote-alloca-to-lds"
  fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall $dev -Wno-unused-result "$@" \
    -c testground_amd/csrc/$f -o $B/${f%.*}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o testground_amd/libtgsim_$name.so $B/*.o
rm -rf $B
