cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m4; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multi.py -x -v --timeout 120 --timeout-method thread > $O/multi.log 2>&1 || { tail -40 $O/multi.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/multi.log | tail -15
timeout -k 10 400 python3 tools/share_balance.py --config c4 > $O/share_c4.json 2> $O/share_c4.log || { tail $O/share_c4.log; exit 1; }
timeout -k 10 400 python3 tools/share_balance.py --config bias20k > $O/share_bias.json 2> $O/share_bias.log || { tail $O/share_bias.log; exit 1; }
grep share_balance $O/share_*.log
