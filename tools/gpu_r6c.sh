#!/bin/bash
# Cleanup check: frame hashes (ray-march C4 scene at 1024^2, free-flight lines) of the pre-cleanup library
# (_ab/head) and the in-tree one must agree; then the -m gpu suite and the C4 bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6c; mkdir -p $OUT
for t in head cur; do
  if [ $t = cur ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$t/libvr_hip.so; fi
  timeout -k 10 200 python3 tools/frame_hash.py > $OUT/hash_$t.txt 2> $OUT/hash_$t.log || { echo "hash $t failed"; tail -5 $OUT/hash_$t.log; exit 1; }
  timeout -k 10 300 python3 tools/ff_frame_hash.py > $OUT/ffhash_$t.txt 2> $OUT/ffhash_$t.log || { echo "ffhash $t failed"; tail -5 $OUT/ffhash_$t.log; exit 1; }
  echo "$t: $(cat $OUT/hash_$t.txt) | $(tr '\n' ' ' < $OUT/ffhash_$t.txt)"
done
unset VR_LIB_PATH
bash tools/gpu_r6.sh r6c
