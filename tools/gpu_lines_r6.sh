#!/bin/bash
# Round-6 bench lines (each with roofline + cpu_baseline), rocprofv3 kernel statistics and the 8-way share
# prediction.  PART=rm: the ray-march lines, C4 statistics, share balance; PART=ff: free-flight + SFD lines and
# the C2 free-flight statistics.  -> gpurun_out/lines6/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/lines6; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.log || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d.get('roofline') or {};c=d.get('cpu_baseline') or {};print('$n', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms', 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'cpu', c.get('value'))"
}
if [ "$PART" = rm ]; then
  run c4 --steps 5
  run c4_env1 --env-samples 1 --steps 5
  run c2 --config c2 --steps 5
  run c3 --config c3 --steps 5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_c4.log 2>&1 || { echo "stats c4 failed"; exit 1; }
  timeout -k 10 600 python3 tools/share_balance.py --ranks 2,4,8 > $O/share_balance_c4.json 2> $O/share_balance.log || { tail -5 $O/share_balance.log; exit 1; }
  grep share_balance $O/share_balance.log | tail -3
else
  run ff_c2 --config c2 --integrator multiscatter --spp 16 --steps 5
  run ff_c3 --config c3 --integrator freeflight --spp 4 --steps 5
  run ff_c4 --config c4 --integrator multiscatter --spp 1 --steps 3
  run ff_c5 --config c5 --integrator multiscatter --spp 16 --steps 5
  run ff_main --config main --steps 3
  run sfd_c5 --config c5 --integrator sfd --spp 256 --steps 2 --warmup 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_ff_c2 -o run --output-format csv -- python3 bench.py --config c2 --integrator multiscatter --spp 16 --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_ff_c2.log 2>&1 || { echo "stats ff c2 failed"; exit 1; }
fi
echo done
