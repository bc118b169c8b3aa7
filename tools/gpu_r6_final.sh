#!/bin/bash
# Round-6 final: the round-end run (full -m gpu suite, smoke, C4 bench, kernel statistics, share balance), the frame
# hash, then the four C4 PMC passes behind the bench line's `traffic` (summarised on the box).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_round_end.sh || exit 1
timeout -k 10 120 python3 tools/frame_hash.py 2>/dev/null | tail -1
bash tools/pmc_c4.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/round_end/r06_c4_pmc_summary.json gpurun_out/pmc_c4/p1 gpurun_out/pmc_c4/p2 gpurun_out/pmc_c4/p3 gpurun_out/pmc_c4/p4 || exit 1
echo final done
