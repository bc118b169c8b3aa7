#!/bin/bash
# Staged free-flight pipeline on the GPU box: parity tests, then frame times staged vs persistent
# (bench.py --opt ff_staged=0/1) on the free-flight lines.  -> gpurun_out/ffab/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ffab; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_freeflight.py tests/test_gpu_inverse.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for line in "c2 multiscatter 16" "c3 freeflight 4" "c5 multiscatter 16" "main multiscatter 256" "c4 multiscatter 1"; do
  set -- $line
  for st in 1 0; do
    timeout -k 10 300 python3 bench.py --config $1 --integrator $2 --spp $3 --steps 3 --warmup 1 --cpu-budget 0 --flops 0 --opt ff_staged=$st > $O/$1_$st.json 2> $O/$1_$st.log || { echo "$1 staged=$st failed"; tail -5 $O/$1_$st.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$1_$st.json'));print('$1 staged=$st', round(d['value'],2), d['unit'], round(d['ms_per_step'],2), 'ms')"
  done
done
for v in evb16; do
  [ -f _ab/$v/libvr_hip.so ] || continue
  for line in "c2 multiscatter 16" "c5 multiscatter 16"; do
    set -- $line
    VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so timeout -k 10 300 python3 bench.py --config $1 --integrator $2 --spp $3 --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $O/$1_$v.json 2> $O/$1_$v.log || { echo "$1 $v failed"; tail -5 $O/$1_$v.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$1_$v.json'));print('$1 $v', round(d['value'],2), d['unit'], round(d['ms_per_step'],2), 'ms')"
  done
done
