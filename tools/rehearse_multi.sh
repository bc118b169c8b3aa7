#!/bin/bash
# N>1 rehearsal of bench.py on a one-GPU box: 2 ranks on cuda:0, slabs gathered through gloo
# (VR_BENCH_GLOO=1), the headline config; the real N>1 run uses RCCL over xGMI.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/multi
VR_BENCH_GLOO=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/multi/n2.json 2> gpurun_out/multi/n2.log || { tail -20 gpurun_out/multi/n2.log; exit 1; }
cut -c1-400 gpurun_out/multi/n2.json
