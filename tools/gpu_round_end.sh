#!/bin/bash
# Round end: the full -m gpu suite, smoke(), the default bench line (C4) and its rocprofv3 kernel statistics.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/round_end; mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log | cut -c1-120
timeout -k 10 400 python3 bench.py > $OUT/c4.json 2> $OUT/c4.log || { tail -5 $OUT/c4.log; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c4.json'));print(round(d['value'],2), d['unit'], round(d['ms_per_step'],2), d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $OUT/stats_c4.log 2>&1 || { echo "stats failed"; exit 1; }
timeout -k 10 600 python3 tools/share_balance.py --ranks 2,4,8 > $OUT/share_balance_c4.json 2> $OUT/share_balance.log || { tail -5 $OUT/share_balance.log; exit 1; }
grep share_balance $OUT/share_balance.log
echo done
