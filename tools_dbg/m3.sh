cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools_dbg/m3.py 1920 1080 100000 0 > gpurun_out/m3.log 2>&1 || exit 1
cat gpurun_out/m3.log | tail -3
