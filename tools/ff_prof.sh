#!/bin/bash
# rocprofv3 kernel stats of the free-flight bench lines (C2/C5/C4 multi-scatter, C3 free-flight).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ffprof; mkdir -p $O
for c in "c2 multiscatter 16" "c5 multiscatter 16" "c3 freeflight 4" "c4 multiscatter 1"; do
  set -- $c
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$1 -o run --output-format csv -- python3 bench.py --config $1 --integrator $2 --spp $3 --steps 2 --warmup 1 --cpu-budget 0 --flops 0 > $O/$1.log 2>&1 || exit 1
  python3 - "$O/$1" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(sys.argv[1].split('/')[-1], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms", round(float(r["Percentage"]), 1), "%")
PY
done
