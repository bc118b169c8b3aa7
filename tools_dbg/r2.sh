#!/bin/bash
# bench line + rocprofv3 kernel-trace summary + PMC passes (secondary/march kernels), C4 workload
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo bench rc=$rc; cat gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > gpurun_out/prof.log 2>&1; rc=$?; echo prof rc=$rc
[ $rc -eq 0 ] || exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
