#!/bin/bash
# PMC passes (one rocprofv3 run each, kernel-trace only) over one C4 frame; counters listed first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc2; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
