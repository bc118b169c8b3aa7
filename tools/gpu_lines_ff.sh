#!/bin/bash
# Free-flight and SFD bench lines (roofline + cpu_baseline) and the rocprofv3 kernel statistics of the
# C2 multi-scatter line.  -> gpurun_out/lines/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/lines; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.log || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d.get('roofline') or {};print('$n', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms', 'frac', r.get('frac'), 'traffic', r.get('traffic'))"
}
run ff_c2 --config c2 --integrator multiscatter --spp 16 --steps 5
run ff_c3 --config c3 --integrator freeflight --spp 4 --steps 5
run ff_c4 --config c4 --integrator multiscatter --spp 1 --steps 3
run ff_c5 --config c5 --integrator multiscatter --spp 16 --steps 5
run ff_main --config main --steps 3
run sfd_c5 --config c5 --integrator sfd --spp 256 --steps 2 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_ff_c2 -o run --output-format csv -- python3 bench.py --config c2 --integrator multiscatter --spp 16 --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_ff_c2.log 2>&1 || { echo "stats ff c2 failed"; exit 1; }
echo done
