#!/bin/bash
# tools/share_balance.py --ranks 8 for the product library and every build under _ab/ (timing only).
cd $GRAFT_REPO_ROOT; O=gpurun_out/absb; mkdir -p $O
for v in base $(ls _ab 2>/dev/null); do
  if [ $v = base ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so; fi
  timeout -k 10 400 python3 tools/share_balance.py --config ${SB_CONFIG:-c4} --ranks ${SB_RANKS:-8} > $O/$v.json 2> $O/$v.log || { echo "$v failed"; tail -3 $O/$v.log; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$v.json'));r=d['ranks']['${SB_RANKS:-8}']
print('$v','full',round(d['full_frame_ms'],2),'max share',round(r['max_ms'],2),'x',round(r['predicted_speedup'],3),'with gather',round(r['predicted_speedup_with_gather'],3),{k:round(x,2) for k,x in r['stage_ms_of_slowest'].items()})"
done
