#!/bin/bash
# A/B of free-flight bench lines: the product library vs the builds under _ab/*/ (tools/ab_build.sh).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abff
for v in base $(ls _ab); do
  if [ $v = base ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so; fi
  for c in ${AB_CONFIGS:-"c2:multiscatter:16" "c3:freeflight:4" "c4:multiscatter:1"}; do
    IFS=: read cfg integ spp <<< "$c"
    timeout -k 10 120 python3 bench.py --config $cfg --integrator $integ --spp $spp --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > gpurun_out/abff/$v.$cfg.json 2> gpurun_out/abff/$v.$cfg.log || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/abff/$v.$cfg.json'));print('$v $cfg $integ',round(d['value'],2),'Mpaths/s',round(d['ms_per_step'],1),'ms')"
  done
done
