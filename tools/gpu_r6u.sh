#!/bin/bash
# Per-axis node step for every 4-wide secondary variant: ray-march and PureRayMarching frame hashes against an AoS
# build of the same HEAD (_ab/aos), the full -m gpu suite, the C4 line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for t in cur aos; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  echo "$t $(VR_LIB_PATH=$lib timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1) pure $(VR_LIB_PATH=$lib timeout -k 10 120 python3 tools/frame_hash.py pure 2>/dev/null | tail -1)"
done
bash tools/gpu_r6p.sh
