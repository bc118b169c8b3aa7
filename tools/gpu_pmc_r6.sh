#!/bin/bash
# Round-6 PMC passes behind the bench lines' `traffic`: the C4 ray-march frame (4 passes) and the free-flight
# lines (4 passes each), summarised on the box into gpurun_out/lines6/r06_*_pmc_summary.json (copied to profiles/).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/lines6; mkdir -p $O
bash tools/pmc_c4.sh || exit 1
python3 tools/pmc_summary.py $O/r06_c4_pmc_summary.json gpurun_out/pmc_c4/p1 gpurun_out/pmc_c4/p2 gpurun_out/pmc_c4/p3 gpurun_out/pmc_c4/p4 || exit 1
bash tools/pmc_ff.sh || exit 1
for c in c2 c4 c5 main; do
  python3 tools/pmc_summary.py $O/r06_ff_${c}_pmc_summary.json gpurun_out/pmc_ff/$c/p1 gpurun_out/pmc_ff/$c/p2 gpurun_out/pmc_ff/$c/p3 gpurun_out/pmc_ff/$c/p4 || exit 1
done
ls $O
