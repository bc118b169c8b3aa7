#!/bin/bash
# The free-flight and inverse bench lines with their CPU baselines (profiles/rNN_ff_*_bench.json) and
# the rocprofv3 kernel stats of the SFD iteration.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/fflines; mkdir -p $O
for c in "c2 multiscatter 16" "c3 freeflight 4" "c4 multiscatter 1" "c5 multiscatter 16" "main multiscatter 256"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --config $1 --integrator $2 --spp $3 --steps ${FF_STEPS:-10} --warmup 1 > $O/$1.json 2> $O/$1.log || exit 1
  python3 -c "import json;d=json.load(open('$O/$1.json'));c=d['cpu_baseline'] or {};print('$1',round(d['value'],2),'Mpaths/s cpu',c.get('value'),'x',round(d['value']/c['value'],1) if c else None)"
done
timeout -k 10 300 python3 bench.py --config c5 --integrator sfd --spp 256 --steps 2 --warmup 1 > $O/c5_sfd.json 2> $O/c5_sfd.log || exit 1
cut -c1-300 $O/c5_sfd.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sfdprof -o run --output-format csv -- python3 bench.py --config c5 --integrator sfd --spp 256 --steps 1 --warmup 0 > $O/sfdprof.log 2>&1 || exit 1
echo done
