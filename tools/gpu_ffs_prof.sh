#!/bin/bash
# Kernel-time breakdown of the staged free-flight pipeline vs the persistent path kernel (C2, C5):
#   rocprofv3 --kernel-trace --stats of one timed bench step each.  -> gpurun_out/ffs_prof/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ffs_prof; mkdir -p $O
for line in "c2 multiscatter 16" "c5 multiscatter 16"; do
  set -- $line
  for st in 1 0; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$1_$st -o run -- python3 bench.py --config $1 --integrator $2 --spp $3 --steps 1 --warmup 1 --cpu-budget 0 --flops 0 --opt ff_staged=$st > $O/$1_$st.log 2>&1 || { echo "$1 staged=$st failed"; tail -5 $O/$1_$st.log; exit 1; }
    f=$(find $O/$1_$st -name '*kernel_stats.csv' | head -1)
    echo "== $1 staged=$st"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:8]: print(r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2),'ms', round(float(r['AverageNs'])/1e3,1),'us')"
  done
done
