#!/bin/bash
# Drain-mode mixed iterations of the secondary kernel (VR_WW_DRAIN_LANES 8 / 16 / 32): frame hash, C4 bench, 8-way
# share balance per build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6y; mkdir -p $O
T="cur d8 d16 d32"
lib() { if [ "$1" = cur ]; then echo $PWD/3dg-vol-renderer_amd/libvr_hip.so; else echo $PWD/_ab/$1/libvr_hip.so; fi; }
for t in $T; do echo "$t $(VR_LIB_PATH=$(lib $t) timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1)"; done
bash tools/ab_run.sh $T > /dev/null && python3 tools/ab_summary.py $T || exit 1
for t in $T; do
  VR_LIB_PATH=$(lib $t) timeout -k 10 300 python3 -u tools/share_balance.py --ranks 8 > $O/share_$t.json 2> $O/share_$t.log || { tail -5 $O/share_$t.log; exit 1; }
  echo "$t $(grep share_balance $O/share_$t.log | tail -1)"
done
