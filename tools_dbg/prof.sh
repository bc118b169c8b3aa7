#!/bin/bash
# kernel-trace summary of a short C4 bench run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/prof}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 "$@" > $OUT/prof.log 2>&1; rc=$?; echo prof rc=$rc
python3 - <<'PY'
import csv,os
p=os.environ.get("OUT","gpurun_out/prof")+"/run_kernel_stats.csv"
for r in csv.DictReader(open(p)):
    print(f'{float(r["AverageNs"])/1e6:10.3f} ms x{r["Calls"]:>3} {float(r["Percentage"]):6.2f}%  {r["Name"][:90]}')
PY
exit $rc
