#!/bin/bash
# Free-flight / inverse round profile: bench lines with CPU baselines + rocprofv3 kernel-trace summaries.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ff; mkdir -p $OUT
timeout -k 10 200 python3 bench.py --config c2 --integrator multiscatter --spp 16 --cpu-budget 15 > $OUT/c2_ms.json 2> $OUT/c2_ms.log || exit 1
timeout -k 10 200 python3 bench.py --config c4 --integrator multiscatter --spp 1 --steps 2 --warmup 1 --cpu-budget 15 > $OUT/c4_ms.json 2> $OUT/c4_ms.log || exit 1
timeout -k 10 200 python3 bench.py --config c3 --integrator freeflight --spp 16 --cpu-budget 15 > $OUT/c3_ff.json 2> $OUT/c3_ff.log || exit 1
timeout -k 10 200 python3 bench.py --config c5 --integrator multiscatter --spp 256 --steps 2 --warmup 1 --cpu-budget 15 > $OUT/c5_ms.json 2> $OUT/c5_ms.log || exit 1
timeout -k 10 300 python3 bench.py --config c5 --integrator sfd --spp 256 --steps 1 --warmup 1 > $OUT/c5_sfd.json 2> $OUT/c5_sfd.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c2 -o run --output-format csv -- python3 bench.py --config c2 --integrator multiscatter --spp 16 --steps 2 --warmup 1 --cpu-budget 0 > $OUT/stats_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c4 -o run --output-format csv -- python3 bench.py --config c4 --integrator multiscatter --spp 1 --steps 1 --warmup 1 --cpu-budget 0 > $OUT/stats_c4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_sfd -o run --output-format csv -- python3 bench.py --config c5 --integrator sfd --spp 16 --steps 1 --warmup 1 > $OUT/stats_sfd.log 2>&1 || exit 1
echo done
