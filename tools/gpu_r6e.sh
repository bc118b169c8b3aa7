#!/bin/bash
# Wave-coherent (union) walk census of the primary march's window queries (VR_DIAG_UNION build, counters of one
# instrumented frame): C4 and C3 bench frames.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e; mkdir -p $O
export VR_LIB_PATH=$PWD/_ab/dunion/libvr_hip.so
for cfg in c4 c3; do
  timeout -k 10 300 python3 tools/diag_c4.py --config $cfg --frames 1 --counts 1 $( [ $cfg = c3 ] && echo "--size 0" ) > $O/$cfg.json 2> $O/$cfg.log || { echo "$cfg failed"; tail -5 $O/$cfg.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$cfg.json'));print('$cfg', d['work']['march'])"
done
