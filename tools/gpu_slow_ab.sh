#!/bin/bash
# Exact slow path A/B: latency histogram of the diagnostic builds, then the slow kernel's time per library
# (rocprofv3 kernel statistics over a 3-frame C4 bench) and the frame hash.   tools/gpu_slow_ab.sh "diag tags" "tags"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/slow
for t in $1; do
  VR_LIB_PATH=$PWD/_ab/$t/libvr_hip.so timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --cpu-budget 0 --flops 0 > gpurun_out/slow/$t.txt 2>&1 || exit 1
  echo "== $t"; grep -v "^{" gpurun_out/slow/$t.txt | grep -v "^\[bench\]" | tail -30
done
for t in $2; do
  if [ "$t" = cur ]; then lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so; else lib=$PWD/_ab/$t/libvr_hip.so; fi
  VR_LIB_PATH=$lib timeout -k 10 150 python3 tools/frame_hash.py > gpurun_out/slow/$t.hash 2>&1 || { tail -5 gpurun_out/slow/$t.hash; exit 1; }
  VR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/slow/st_$t -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > gpurun_out/slow/st_$t.log 2>&1 || exit 1
  echo "$t $(tail -1 gpurun_out/slow/$t.hash) $(grep -h secondary_slow gpurun_out/slow/st_$t/run_kernel_stats.csv | cut -d, -f2-4)"
done
