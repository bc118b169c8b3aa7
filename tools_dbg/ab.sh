#!/bin/bash
# GPU parity tests (unless NOTEST=1), then bench variants "name:ENV=VAL:bench args" on C4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
if [ "$NOTEST" != "1" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
fi
for spec in "$@"; do
  IFS=':' read -r name envs bargs <<< "$spec"
  dir=.; [[ $name == WT* ]] && dir=_wt  # WT*: the baseline worktree build (git worktree at _wt)
  env ${envs//,/ } timeout -k 10 240 python $dir/bench.py --steps 2 --warmup 1 --cpu-budget 0 $bargs > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err; rc=$?
  echo "$name rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab/$name.json'));r=d['roofline'];print(round(d['value'],3),'Mrays/s',{k:round(v,1) for k,v in r['stage_ms'].items()},r['secondary_rays'], r.get('work',{}).get('secondary'))" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || exit $rc
done
