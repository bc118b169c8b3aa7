#!/bin/bash
# March LDS stack vs private-memory overflow A/B (VR_MARCH_STACK4 / VR_MARCH_DEEP): C4 bench per build (twice) + frame hash.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="${T:-cur s24d8 s16d8 s12d12 s10d14}"
for t in $T; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  echo "$t $(VR_LIB_PATH=$lib timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1)"
done
bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T && bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T
