#!/bin/bash
# rehearsal of bench.py's N>1 path on one GPU: 2 ranks on cuda:0, gloo gather through host memory
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VR_BENCH_GLOO=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --config c2 > gpurun_out/mgpu.json 2> gpurun_out/mgpu.err; rc=$?; echo rc=$rc; cat gpurun_out/mgpu.json; tail -3 gpurun_out/mgpu.err
