#!/bin/bash
# Ray-march A/B: frame hash (1024x1024 C4 scene, must match) and C4 bench line per library, then the
# ray-march parity tests on the last tag's library.   tools/gpu_march_ab.sh tag1 tag2 ...  ("cur" = in-tree)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mab
for t in "$@"; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  VR_LIB_PATH=$lib timeout -k 10 150 python3 tools/frame_hash.py > gpurun_out/mab/$t.hash 2>&1 || { tail -5 gpurun_out/mab/$t.hash; exit 1; }
  VR_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-budget 0 --flops 0 > gpurun_out/mab/$t.json 2> gpurun_out/mab/$t.log || { tail -5 gpurun_out/mab/$t.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/mab/$t.json'));s=d['roofline']['stage_ms'];print('$t', open('gpurun_out/mab/$t.hash').read().split()[-2:], round(d['value'],2), 'Mrays/s', {k:round(v,2) for k,v in s.items()})"
done
if [ -n "$PARITY" ]; then
  VR_LIB_PATH=$lib timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mab/parity.log 2>&1; rc=$?; tail -2 gpurun_out/mab/parity.log; exit $rc
fi
