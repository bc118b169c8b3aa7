#!/bin/bash
# GPU parity tests, then A/B bench variants on C4 (stage timings in each JSON line)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
run() { name=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-budget 0 --flops 0 $BARGS > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err; rc=$?; echo "$name rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab/$name.json'));r=d['roofline'];print(round(d['value'],3),'Mrays/s',{k:round(v,1) for k,v in r['stage_ms'].items()},r['secondary_rays'])")"; return $rc; }
BARGS="" run fast VR_X=0 && BARGS="" run exact VR_SEC_EXACT=1 && BARGS="--t-eps 1e-6" run fast_teps6 VR_X=0 && BARGS="" run persist_fast VR_SECONDARY=p
