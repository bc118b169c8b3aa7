#!/bin/bash
# Drain of the exact slow path inside the persistent kernel: parity suite, C4 bench A/B (drain / no drain, twice),
# 8-way share timelines of both.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_run.sh cur nodrain && python3 tools/ab_summary.py cur nodrain
bash tools/ab_run.sh cur nodrain && python3 tools/ab_summary.py cur nodrain
timeout -k 10 200 python3 tools/frame_hash.py
VR_LIB_PATH=$PWD/_ab/nodrain/libvr_hip.so timeout -k 10 200 python3 tools/frame_hash.py
bash tools/gpu_share_prof.sh cur nodrain
for t in cur nodrain; do grep -E "secondary_ww|slow_kernel|^frame" gpurun_out/share_prof/$t/r8/timeline.txt; done
