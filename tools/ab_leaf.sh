cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab
for v in base leaf1 leaf2 leaf4; do
  if [ $v = base ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so; fi
  timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));r=d['roofline'];print('$v',round(d['value'],2),{k:round(x,2) for k,x in r['stage_ms'].items()},r['work']['secondary'],r['work']['march']['active_steps'])"
done
