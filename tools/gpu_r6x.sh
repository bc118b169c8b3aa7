#!/bin/bash
# rocprofv3 kernel statistics of the other ray-march lines (C3, C2, C4 with one environment sample) at round-6 HEAD.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6x; mkdir -p $O
for c in "c3:--config c3" "c2:--config c2" "c4_env1:--env-samples 1"; do
  n=${c%%:*}; a=${c#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$n -o run --output-format csv -- python3 bench.py $a --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/stats_$n.log 2>&1 || { echo "stats $n failed"; exit 1; }
  echo "$n ok"
done
