#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, kernel-trace only) of the free-flight lines behind
# profiles/r03_ff_{c2,c4,c5}_pmc_summary.json (tools/pmc_summary.py OUT.json DIR/p1 .. DIR/p4).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_ff; mkdir -p $O
SETS=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES")
for c in ${PMC_FF_CONFIGS:-c2:multiscatter:16 c4:multiscatter:1 c5:multiscatter:16 main:multiscatter:256}; do
  set -- ${c//:/ }
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1)); mkdir -p $O/$1
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $O/$1/p$i -o run --output-format csv -- python3 bench.py --config $1 --integrator $2 --spp $3 --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > $O/$1/p$i.log 2>&1
    rc=$?; echo "$1 pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo done
