#!/bin/bash
# A/B of env_order_kernel changes: the GPU tests that render environment rays, then C4 kernel statistics.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/envab; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -k "env or c4 or secondary or split or multi" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_c4.log 2>&1 || { echo "stats failed"; tail -5 $O/stats_c4.log; exit 1; }
python3 - <<'PY'
import glob, csv
for f in glob.glob('gpurun_out/envab/stats_c4/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e6, 3), 'ms')
PY
echo done
