cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "over_record_capacity" > $O/t0.log 2>&1 || { tail -30 $O/t0.log; exit 1; }
grep -E "PASS|FAIL" $O/t0.log
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inverse.py -x -v -s --timeout 300 --timeout-method thread -k "full_size or c2 or early_out or budget or c5 or sfd" > $O/tests.log 2>&1
rc=$?
grep -E "L-inf|C5|PASS|FAIL|passed|failed|Error" $O/tests.log | tail -40
exit $rc
