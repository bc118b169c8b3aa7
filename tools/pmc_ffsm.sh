#!/bin/bash
# PMC passes of the free-flight C2 line for a library (VR_LIB_PATH), one rocprofv3 run per counter set.
#   tools/pmc_ffsm.sh TAG "set1" "set2" ...   -> gpurun_out/pmc_ffsm/TAG/p<i>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
O=gpurun_out/pmc_ffsm/$tag; mkdir -p $O
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $O/p$i -o run --output-format csv -- python3 bench.py --config c2 --integrator multiscatter --spp 16 --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > $O/p$i.log 2>&1
  rc=$?; echo "$tag pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
