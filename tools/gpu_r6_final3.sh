#!/bin/bash
# Round-6 final, part 2: the free-flight and SFD lines, then the free-flight PMC passes (C2, C4, C5, main).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PART=ff bash tools/gpu_lines_r6.sh || exit 1
bash tools/pmc_ff.sh || exit 1
for c in c2 c4 c5 main; do
  python3 tools/pmc_summary.py gpurun_out/lines6/r06_ff_${c}_pmc_summary.json gpurun_out/pmc_ff/$c/p1 gpurun_out/pmc_ff/$c/p2 gpurun_out/pmc_ff/$c/p3 gpurun_out/pmc_ff/$c/p4 > /dev/null || exit 1
done
echo final2 done
