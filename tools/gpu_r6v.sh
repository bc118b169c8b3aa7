#!/bin/bash
# Traffic of the secondary kernel, per-axis node step (cur) vs the AoS build of the same HEAD (_ab/aos): FETCH_SIZE and
# WRITE_SIZE passes of the C4 frame each.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_ab; mkdir -p $O
for t in cur aos; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    VR_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $O/$t/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > $O/$t.p$i.log 2>&1
    rc=$?; echo "$t pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo done
