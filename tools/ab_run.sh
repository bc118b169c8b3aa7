#!/bin/bash
# usage: ab_run.sh tag1 tag2 ... (tag "cur" = the in-tree library); bench C4 each, one JSON line per tag
set -e
mkdir -p gpurun_out/ab
for t in "$@"; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  VR_LIB_PATH=$lib timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --cpu-budget 0 --flops 0 $BENCH_EXTRA > gpurun_out/ab/$t.log 2>&1
  echo "$t done"
done
