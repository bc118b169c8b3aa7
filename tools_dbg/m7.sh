cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m7; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_inverse.py tests/test_cpp_api.py -x -v -s -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
grep -E "C5|PASS|FAIL|Error|error|passed|failed" $O/t.log | head -40
[ $rc -eq 0 ] || { tail -30 $O/t.log; exit $rc; }
timeout -k 10 400 python3 bench.py --config c5 --integrator sfd --spp 256 --steps 2 --warmup 1 --cpu-budget 0 > $O/sfd.json 2> $O/sfd.log || { tail $O/sfd.log; exit 1; }
cut -c1-600 $O/sfd.json
