#!/bin/bash
# tools/diag_c4.py for the product library and every build under _ab/ (tools/ab_build.sh):
#   tools/diag_ab.sh [diag_c4.py args]  -> gpurun_out/diag/<variant>.json
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/diag
for v in base $(ls _ab 2>/dev/null); do
  if [ $v = base ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so; fi
  timeout -k 10 240 python3 tools/diag_c4.py "$@" > gpurun_out/diag/$v.json 2> gpurun_out/diag/$v.log || { echo "$v failed"; tail -5 gpurun_out/diag/$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/diag/$v.json'));print('$v',round(d['kernel_ms'],2),d['stage_ms'],d.get('work',{}).get('secondary'))"
done
