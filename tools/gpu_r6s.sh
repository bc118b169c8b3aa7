#!/bin/bash
# Collection-walk steps per iteration (VR_COLLECT_STEPS 4 / 6 / 8) on every free-flight line, and frame hashes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="cur cs6 cs8"
lib() { if [ "$1" = cur ]; then echo $PWD/3dg-vol-renderer_amd/libvr_hip.so; else echo $PWD/_ab/$1/libvr_hip.so; fi; }
for t in $T; do echo "$t $(VR_LIB_PATH=$(lib $t) timeout -k 10 120 python3 tools/ff_frame_hash.py 2>/dev/null | tr "\n" " ")"; done
for c in "c2 --integrator multiscatter --spp 16" "c3 --integrator freeflight --spp 4" "c4 --integrator multiscatter --spp 1 --steps 3" "main"; do
  export BENCH_EXTRA="--config $c"
  for rep in 1 2; do
    bash tools/ab_run.sh $T > /dev/null || exit 1
    for t in $T; do tail -1 gpurun_out/ab/$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$t', '${c%% *}', round(d['value'],2), d['unit'], round(d['ms_per_step'],2))"; done
  done
done
