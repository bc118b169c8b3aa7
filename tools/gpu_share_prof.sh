#!/bin/bash
# Kernel trace of one C4 1/8 share (tools/share_prof.py) and of the full frame (ranks 1), per library tag.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for t in "$@"; do
  if [ "$t" = cur ]; then export VR_LIB_PATH=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else export VR_LIB_PATH=$PWD/_ab/$t/libvr_hip.so; fi
  for R in 8 1; do
    O=gpurun_out/share_prof/$t/r$R; mkdir -p $O
    timeout -k 10 240 rocprofv3 --kernel-trace -d $O -o run --output-format csv -- python3 tools/share_prof.py --ranks $R --reps 2 > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
    f=$(find $O -name "*kernel_trace.csv" | head -1)
    python3 tools/share_timeline.py $f > $O/timeline.txt && tail -1 $O/timeline.txt && grep "share" $O/log.txt | tail -1
  done
done
