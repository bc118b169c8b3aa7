#!/bin/bash
# Cost of the secondary kernel's rare-case tests: merged branch (VR_WW_RARE_MERGED=1) and no chord band (A/B only).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="cur band2 band1 noband"
for t in cur band2 band1; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  echo "$t $(VR_LIB_PATH=$lib timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1)"
done
bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T && bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T
