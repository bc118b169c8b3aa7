#!/bin/bash
# Round measurement, free-flight half: PMC passes of C2/C4/C5/main, then the free-flight and SFD bench
# lines (their traffic read from those summaries) and rocprofv3 kernel statistics of C2 and C5.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/lines; mkdir -p $O
bash tools/pmc_ff.sh || exit 1
for c in c2 c4 c5 main; do
  python3 tools/pmc_summary.py profiles/r04_ff_${c}_pmc_summary.json gpurun_out/pmc_ff/$c/p1 gpurun_out/pmc_ff/$c/p2 gpurun_out/pmc_ff/$c/p3 gpurun_out/pmc_ff/$c/p4 > /dev/null || exit 1
done
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.log || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d.get('roofline') or {};print('$n', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms', 'frac', r.get('frac'), 'traffic', r.get('traffic'))"
}
run c4_env1 --env-samples 1 --steps 5
run ff_c2 --config c2 --integrator multiscatter --spp 16 --steps 5
run ff_c3 --config c3 --integrator freeflight --spp 4 --steps 5
run ff_c4 --config c4 --integrator multiscatter --spp 1 --steps 3
run ff_c5 --config c5 --integrator multiscatter --spp 16 --steps 5
run ff_main --config main --steps 3
run sfd_c5 --config c5 --integrator sfd --spp 256 --steps 2 --warmup 1
for l in "c2 multiscatter 16" "c5 multiscatter 16"; do
  set -- $l
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_ff_$1 -o run --output-format csv -- python3 bench.py --config $1 --integrator $2 --spp $3 --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_ff_$1.log 2>&1 || { echo "stats ff $1 failed"; exit 1; }
done
echo done
