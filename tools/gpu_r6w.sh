#!/bin/bash
# Per-axis node step with the slabs computed per child pair (VR_SEC_SOA_PAIRS=1: 2 spilled VGPRs instead of 12) against
# the all-children form (cur) and the AoS build: frame hash, C4 bench twice, FETCH/WRITE_SIZE passes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="cur pairs aos"
lib() { if [ "$1" = cur ]; then echo $PWD/3dg-vol-renderer_amd/libvr_hip.so; else echo $PWD/_ab/$1/libvr_hip.so; fi; }
for t in $T; do echo "$t $(VR_LIB_PATH=$(lib $t) timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1)"; done
bash tools/ab_run.sh $T > /dev/null && python3 tools/ab_summary.py $T && bash tools/ab_run.sh $T > /dev/null && python3 tools/ab_summary.py $T || exit 1
O=gpurun_out/pmc_ab2; mkdir -p $O
for t in pairs; do
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    VR_LIB_PATH=$(lib $t) timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $O/$t/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > $O/$t.p$i.log 2>&1
    rc=$?; echo "$t pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
