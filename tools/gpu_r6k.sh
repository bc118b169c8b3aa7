#!/bin/bash
# Guided tail of the secondary kernel's claim units (VR_WW_TAIL_UNITS / VR_WW_TAIL_SPLIT): frame hash, 8-way share
# balance per build, C4 bench lines.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6k; mkdir -p $O
T="tail0 cur tail1 tail4 tail2s4"
lib() { if [ "$1" = cur ]; then echo $PWD/3dg-vol-renderer_amd/libvr_hip.so; else echo $PWD/_ab/$1/libvr_hip.so; fi; }
for t in tail0 cur; do echo "$t $(VR_LIB_PATH=$(lib $t) timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1)"; done
for t in $T; do
  VR_LIB_PATH=$(lib $t) timeout -k 10 300 python3 -u tools/share_balance.py --ranks 8 > $O/share_$t.json 2> $O/share_$t.log || { tail -5 $O/share_$t.log; exit 1; }
  echo "$t $(grep share_balance $O/share_$t.log | tail -1)"
done
bash tools/ab_run.sh tail0 cur tail4 && python3 tools/ab_summary.py tail0 cur tail4
