#!/bin/bash
# A/B build of libvr_hip.so with host sources recompiled under extra -D flags:
#   tools/ab_build_host.sh NAME "-DFOO=1 ..." [host files, default vr_device]  -> _ab/NAME/libvr_hip.so
set -e
cd "$(dirname "$0")/../3dg-vol-renderer_amd/csrc"
name=$1; flags=$2; files=${3:-vr_device}
mkdir -p ../../_ab/$name
objs=$(ls ../build/*.o)
new=""
for f in $files; do
  /opt/rocm/bin/hipcc -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -std=c++20 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-result $flags -c host/$f.cpp -o ../../_ab/$name/$f.o
  objs=$(echo "$objs" | grep -v "/$f.o")
  new="$new ../../_ab/$name/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../_ab/$name/libvr_hip.so $objs $new -ldl
rm $new
