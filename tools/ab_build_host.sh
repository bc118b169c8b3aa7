#!/bin/bash
# A/B build of libvr_hip.so with host/vr_device.cpp recompiled under extra -D flags:
#   tools/ab_build_host.sh NAME "-DFOO=1 ..."  -> _ab/NAME/libvr_hip.so
set -e
cd "$(dirname "$0")/../3dg-vol-renderer_amd/csrc"
name=$1; flags=$2
mkdir -p ../../_ab/$name
/opt/rocm/bin/hipcc -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -std=c++20 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-result $flags -c host/vr_device.cpp -o ../../_ab/$name/vr_device.o
objs=$(ls ../build/*.o | grep -v "/vr_device.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../_ab/$name/libvr_hip.so $objs ../../_ab/$name/vr_device.o -ldl
rm ../../_ab/$name/vr_device.o
