#!/bin/bash
# Wave-cooperative exact slow path: parity tests, C4 bench A/B (coop / serial, twice), share timelines.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log; grep -E "t_eps=" $O/tests.log | cut -c1-250
bash tools/ab_run.sh cur nocoop && python3 tools/ab_summary.py cur nocoop
bash tools/ab_run.sh cur nocoop && python3 tools/ab_summary.py cur nocoop
bash tools/gpu_share_prof.sh cur nocoop
for t in cur nocoop; do grep -E "secondary_ww|slow|^frame" gpurun_out/share_prof/$t/r8/timeline.txt gpurun_out/share_prof/$t/r1/timeline.txt; done
