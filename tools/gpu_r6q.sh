#!/bin/bash
# Per-axis copy of the shared 4-wide tree for every wide_children walk (march, exact slow path, free-flight): frame
# hashes, C4 / C3 ray-march and C2 / C5 free-flight lines against the previous HEAD's build (_ab/prev).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="cur prev"
lib() { if [ "$1" = cur ]; then echo $PWD/3dg-vol-renderer_amd/libvr_hip.so; else echo $PWD/_ab/$1/libvr_hip.so; fi; }
for t in $T; do echo "$t $(VR_LIB_PATH=$(lib $t) timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1) ff $(VR_LIB_PATH=$(lib $t) timeout -k 10 120 python3 tools/ff_frame_hash.py 2>/dev/null | tr "\n" " ")"; done
bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T && bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T || exit 1
BENCH_EXTRA="--config c3" bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T || exit 1
for c in "c2 --integrator multiscatter --spp 16" "c5 --integrator multiscatter --spp 16"; do
  export BENCH_EXTRA="--config $c"
  bash tools/ab_run.sh $T && bash tools/ab_run.sh $T || exit 1
  for t in $T; do tail -1 gpurun_out/ab/$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$t', '${c%% *}', round(d['value'],2), d['unit'], round(d['ms_per_step'],2))"; done
done
