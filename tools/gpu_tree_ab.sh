#!/bin/bash
# Tree / march A/B on the GPU box: C4 diagnostics for every _ab build, then the ray-march parity tests
# against the build named in $1 (default tight32).  -> gpurun_out/diag/, gpurun_out/tree_ab/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/diag_ab.sh || exit 1
O=gpurun_out/tree_ab; mkdir -p $O
v=${1:-tight32}
VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity_$v.log 2>&1
rc=$?; tail -3 $O/parity_$v.log; exit $rc
