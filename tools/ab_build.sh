#!/bin/bash
# A/B build of libvr_hip.so with one kernel object recompiled under extra -D flags:
#   tools/ab_build.sh NAME KERNEL(e.g. vr_freeflight) "-DFOO=1 ..."  -> _ab/NAME/libvr_hip.so
set -e
cd "$(dirname "$0")/../3dg-vol-renderer_amd/csrc"
name=$1; k=$2; flags=$3
mkdir -p ../../_ab/$name
/opt/rocm/bin/hipcc -std=c++20 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize $flags -c kernels/$k.hip -o ../../_ab/$name/$k.o
objs=$(ls ../build/*.o | grep -v "/$k.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../_ab/$name/libvr_hip.so $objs ../../_ab/$name/$k.o -ldl
rm ../../_ab/$name/$k.o
