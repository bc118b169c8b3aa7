#!/bin/bash
# Round check: the full -m gpu suite, smoke(), and the share-balance prediction of the multi-GPU split.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/final; mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 tools/share_balance.py --ranks 2,4,8 > $OUT/share_balance_c4.json 2> $OUT/share_balance.log || { tail -5 $OUT/share_balance.log; exit 1; }
grep share_balance $OUT/share_balance.log
echo done
