#!/bin/bash
# Ray-march bench lines (roofline + cpu_baseline), the rocprofv3 kernel statistics of the headline and
# its four PMC passes.  -> gpurun_out/lines/, gpurun_out/pmc_c4/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/lines; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.log || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d.get('roofline') or {};print('$n', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms', 'frac', r.get('frac'), 'alg_s8d', r.get('alg_frac_s8d'))"
}
run c4 --steps 5
run c4_env1 --env-samples 1 --steps 5
run c2 --config c2 --steps 5
run c3 --config c3 --steps 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_c4.log 2>&1 || { echo "stats c4 failed"; exit 1; }
bash tools/pmc_c4.sh
