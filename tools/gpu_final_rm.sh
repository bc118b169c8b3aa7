#!/bin/bash
# Round measurement, ray-march half: C4 PMC passes first (the bench line reads their summary), then the
# ray-march bench lines (C4, C4 env_samples=1, C2, C3; roofline + cpu_baseline) and rocprofv3 kernel
# statistics of each line.  -> gpurun_out/pmc_c4/, gpurun_out/lines/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/lines; mkdir -p $O
bash tools/pmc_c4.sh || exit 1
python3 tools/pmc_summary.py profiles/r04_c4_pmc_summary.json gpurun_out/pmc_c4/p1 gpurun_out/pmc_c4/p2 gpurun_out/pmc_c4/p3 gpurun_out/pmc_c4/p4 > /dev/null || exit 1
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.log || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d.get('roofline') or {};print('$n', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms', 'frac', r.get('frac'), 'alg_s8d', r.get('alg_frac_s8d'), 'traffic', r.get('traffic'))"
}
stats() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$n -o run --output-format csv -- python3 bench.py "$@" --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_$n.log 2>&1 || { echo "stats $n failed"; exit 1; }
}
run c4 --steps 5
run c4_env1 --env-samples 1 --steps 5
run c2 --config c2 --steps 5
run c3 --config c3 --steps 5
stats c4
stats c4_env1 --env-samples 1
stats c2 --config c2
stats c3 --config c3
echo done
