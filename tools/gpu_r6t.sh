#!/bin/bash
# Free-flight GPU tests and the round-6 free-flight / SFD bench lines at HEAD (collection steps 6 / 8).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_freeflight.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PART=ff bash tools/gpu_lines_r6.sh
