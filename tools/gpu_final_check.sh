#!/bin/bash
# Round check: the full -m gpu suite, smoke(), and the share-balance prediction of the multi-GPU split.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/final; mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 tools/share_balance.py --ranks 2,4,8 > $OUT/share_balance_c4.json 2> $OUT/share_balance.log || { tail -5 $OUT/share_balance.log; exit 1; }
grep share_balance $OUT/share_balance.log

O=gpurun_out/lines; mkdir -p $O
timeout -k 10 300 python3 bench.py --config c2 --steps 5 > $O/c2.json 2> $O/c2.log || { tail -5 $O/c2.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/c2.json'));print('c2', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_c2.log 2>&1 || { echo "stats c2 failed"; exit 1; }
echo done2
