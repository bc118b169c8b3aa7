cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m6; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "device_bvh" > $O/t.log 2>&1; rc=$?
grep -E "device_bvh=|tree|PASS|FAIL|Error|error" $O/t.log | head -30
exit $rc
