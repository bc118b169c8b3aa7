#!/bin/bash
# Full -m gpu suite, then the ray-march bench lines, C4 kernel statistics and share balance (gpu_lines_r6.sh PART=rm).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PART=rm bash tools/gpu_lines_r6.sh
