#!/bin/bash
# Full -m gpu suite and smoke at HEAD (per-axis secondary node copy), then the C4 line with kernel statistics.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-100
timeout -k 10 300 python3 bench.py > $O/c4.json 2> $O/c4.log || { tail -5 $O/c4.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/c4.json'));print(round(d['value'],2), d['unit'], round(d['ms_per_step'],2), d['roofline']['stage_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_c4.log 2>&1 || { echo "stats failed"; exit 1; }
echo done
