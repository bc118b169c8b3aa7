#!/bin/bash
# Free-flight A/B: frame hashes (bit-identical check) and bench lines for the in-tree library and _ab builds.
#   tools/gpu_ffsm.sh tag1 tag2 ...   (tag "cur" = the in-tree library)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ffsm
for t in "$@"; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  VR_LIB_PATH=$lib timeout -k 10 150 python3 -u tools/ff_frame_hash.py ${HASH_CASES} > gpurun_out/ffsm/$t.hash 2>&1 || exit 1
  echo "$t $(cat gpurun_out/ffsm/$t.hash | tr '\n' ' ')"
  for c in ${AB_CONFIGS:-"c2:multiscatter:16" "c3:freeflight:4"}; do
    IFS=: read cfg integ spp <<< "$c"
    VR_LIB_PATH=$lib timeout -k 10 150 python3 bench.py --config $cfg --integrator $integ --spp $spp --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > gpurun_out/ffsm/$t.$cfg.json 2> gpurun_out/ffsm/$t.$cfg.log || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ffsm/$t.$cfg.json'));print('$t $cfg $integ',round(d['value'],2),'Mpaths/s',round(d['ms_per_step'],1),'ms', d['config'].get('frame_kernel_ms'))"
  done
done
