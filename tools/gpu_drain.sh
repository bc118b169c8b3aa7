#!/bin/bash
# Secondary kernel tail census (VR_DIAG_DRAIN build in _ab/drain): the full C4 frame, then each 8-way share.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/drain; mkdir -p $O
VR_LIB_PATH=$PWD/_ab/drain/libvr_hip.so timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --cpu-budget 0 --flops 0 > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
VR_LIB_PATH=$PWD/_ab/drain/libvr_hip.so timeout -k 10 300 python3 -u tools/share_balance.py --ranks 8 --reps 1 > $O/share8.log 2>&1 || { tail -5 $O/share8.log; exit 1; }
grep -E "^drain" $O/c4.log | head -3; grep -E "^drain" $O/share8.log | head -16
