#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "full_size or early_out" > gpurun_out/t1.log 2>&1; rc=$?; echo rc=$rc; grep -E "L-inf|passed|failed" gpurun_out/t1.log | tail -8; exit $rc
