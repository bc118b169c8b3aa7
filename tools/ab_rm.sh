#!/bin/bash
# A/B of the C4 ray-march headline: the product library vs the builds under _ab/*/ (tools/ab_build.sh).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abrm
for v in base $(ls _ab); do
  if [ $v = base ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so; fi
  timeout -k 10 180 python3 bench.py --steps 4 --warmup 1 --cpu-budget 0 --flops 0 > gpurun_out/abrm/$v.json 2> gpurun_out/abrm/$v.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/abrm/$v.json'));r=d['roofline'];print('$v',round(d['value'],2),'Mrays/s',round(d['ms_per_step'],1),'ms secondary',round(r['stage_ms']['secondary'],2))"
done
