#!/bin/bash
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo tests rc=$rc
[ $rc -le 1 ] || exit $rc
for v in default simple; do
  VR_SECONDARY=$v timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --cpu-budget 0 --flops 0 > gpurun_out/ab_$v.log 2> gpurun_out/ab_$v.err; rc=$?; echo $v rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
