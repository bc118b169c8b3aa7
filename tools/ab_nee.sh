#!/bin/bash
# A/B: product library vs the diagnostic build without NEE shadow walks (VR_DIAG_FF_NO_NEE), free-flight lines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abnee
for v in base nonee; do
  if [ $v = base ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so; fi
  for c in "c2 multiscatter 16" "c5 multiscatter 16" "c4 multiscatter 1"; do
    set -- $c
    timeout -k 10 120 python3 bench.py --config $1 --integrator $2 --spp $3 --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/abnee/$v.$1.json 2> gpurun_out/abnee/$v.$1.log || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/abnee/$v.$1.json'));print('$v $1 $2',round(d['value'],2),'Mpaths/s',round(d['ms_per_step'],1),'ms')"
  done
done
