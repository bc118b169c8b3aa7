#!/bin/bash
# The four PMC passes of the C4 ray-march frame (product library) -> gpurun_out/pmc_c4/p1..p4
# (summarise: tools/pmc_summary.py profiles/rNN_c4_pmc_summary.json gpurun_out/pmc_c4/p{1,2,3,4}).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_c4; mkdir -p $O
SETS=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $O/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > $O/p$i.log 2>&1
  rc=$?; echo "c4 pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
