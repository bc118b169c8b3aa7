#!/bin/bash
# Secondary-kernel tail census (VR_DIAG_DRAIN), 8-way share balance without shorter claim units (VR_WW_SPLIT_CPW=0),
# shadow-ray kernel LDS/private stack split at 6 blocks per CU (C2 multiscatter, twice).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_drain.sh || exit 1
O=gpurun_out/r6j; mkdir -p $O
for t in cur nosplit; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  VR_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/share_balance.py --ranks 8 > $O/share_$t.json 2> $O/share_$t.log || { tail -5 $O/share_$t.log; exit 1; }
  echo "$t $(grep share_balance $O/share_$t.log | tail -1)"
done
export BENCH_EXTRA="--config c2 --integrator multiscatter --spp 16"
bash tools/ab_run.sh cur nee16b6 && bash tools/ab_run.sh cur nee16b6 || exit 1
for t in cur nee16b6; do tail -1 gpurun_out/ab/$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$t', round(d['value'],2), d['unit'], round(d['ms_per_step'],2))"; done
