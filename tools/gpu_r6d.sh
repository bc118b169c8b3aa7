#!/bin/bash
# Phase-scheduled free-flight kernel occupancy A/B on C2 (multi-scatter, 16 spp): 4 (cur) / 3 / 2 waves per SIMD
# (VR_FFSM_WAVES; 128 VGPRs + 65 spilled / 168 + 25 / 206 + 0), bench lines twice, then FETCH_SIZE / WRITE_SIZE
# passes of each.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d; mkdir -p $O
for rep in 1 2; do
for t in cur ffsm3 ffsm2; do
  if [ $t = cur ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$t/libvr_hip.so; fi
  timeout -k 10 200 python3 bench.py --config c2 --integrator multiscatter --spp 16 --steps 5 --warmup 1 --cpu-budget 0 --flops 0 > $O/$t.json 2> $O/$t.log || { echo "$t failed"; tail -5 $O/$t.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$t.json'));print('$t', round(d['value'],2), d['unit'], round(d['ms_per_step'],2), 'ms')"
done
done
for t in cur ffsm3 ffsm2; do
  if [ $t = cur ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$t/libvr_hip.so; fi
  bash tools/pmc_ffsm.sh r6_$t "FETCH_SIZE" "WRITE_SIZE" || exit 1
done
