#!/bin/bash
# March pre-test (VR_MARCH_PRETEST=1, fast-form certain rejects before the exact intersect) at 5 waves/SIMD: frame hash,
# C4 bench twice, C2/C3 march stage.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="${T:-cur pretest}"
for t in $T; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  echo "$t $(VR_LIB_PATH=$lib timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1)"
done
bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T && bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T || exit 1
BENCH_EXTRA="--config c3" bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T
