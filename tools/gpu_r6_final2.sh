#!/bin/bash
# Round-6 final, part 1: the round-end run (full -m gpu suite, smoke, C4 line, kernel statistics, share balance),
# the ray-march lines (C4, C4 1 env sample, C2, C3), the C4 PMC passes (summarised on the box).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_round_end.sh || exit 1
timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1
PART=rm bash tools/gpu_lines_r6.sh || exit 1
bash tools/pmc_c4.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/round_end/r06_c4_pmc_summary.json gpurun_out/pmc_c4/p1 gpurun_out/pmc_c4/p2 gpurun_out/pmc_c4/p3 gpurun_out/pmc_c4/p4 > /dev/null || exit 1
echo final1 done
