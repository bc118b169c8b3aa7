#!/bin/bash
# Round-4 validation block: ray-march parity (march pre-test, start subtrees), the staged free-flight
# pipeline (tests + staged/persistent A/B), then the C4 diagnostics A/B.  -> gpurun_out/r4d/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_binned.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
rc=$?; tail -3 $O/parity.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ff_ab.sh || exit 1
bash tools/diag_ab.sh
