#!/bin/bash
# Round-5 check: the full -m gpu suite and smoke() on the in-tree library, then A/B bench lines (tools/ab_run.sh).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r5; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ -n "$AB" ]; then bash tools/ab_run.sh $AB; fi
echo done
