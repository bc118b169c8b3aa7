#!/bin/bash
# Free-flight schedule constants at round-6 HEAD (shadow-ray / collection steps per iteration, SWEEP event budget):
# C2 and C5 multi-scatter lines, twice each.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="${T:-cur ns3 ns6 cs3 cs6 sb16 sb32}"
for c in "c2 --integrator multiscatter --spp 16" "c5 --integrator multiscatter --spp 16"; do
  export BENCH_EXTRA="--config $c"
  for rep in 1 2; do
    bash tools/ab_run.sh $T > /dev/null || exit 1
    for t in $T; do tail -1 gpurun_out/ab/$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$t', '${c%% *}', round(d['value'],2), d['unit'], round(d['ms_per_step'],2))"; done
  done
done
