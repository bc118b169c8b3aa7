#!/bin/bash
# A/B build of the whole libvr_hip.so (host and device objects) under extra flags:
#   tools/ab_build_full.sh NAME "-DFOO=1 ..."  -> _ab/NAME/libvr_hip.so
set -e
cd "$(dirname "$0")/../3dg-vol-renderer_amd/csrc"
name=$1; flags=$2
mkdir -p ../../_ab/$name
make -s -j16 BUILD=../../_ab/$name/build OUT=../../_ab/$name/libvr_hip.so EXTRA="$flags"
rm -rf ../../_ab/$name/build
