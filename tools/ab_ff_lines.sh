#!/bin/bash
# Free-flight lines (timing only) for the product library and every build under _ab/:
#   tools/ab_ff_lines.sh -> gpurun_out/abff/<variant>_<line>.json
cd $GRAFT_REPO_ROOT; O=gpurun_out/abff; mkdir -p $O
for v in base $(ls _ab 2>/dev/null); do
  if [ $v = base ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=$PWD/_ab/$v/libvr_hip.so; fi
  for line in "c2 multiscatter 4" "c4 multiscatter 3" "c5 multiscatter 4" "c3 freeflight 4"; do
    set -- $line
    timeout -k 10 240 python3 bench.py --config $1 --integrator $2 --steps $3 --warmup 1 --cpu-budget 0 --flops 0 > $O/${v}_$1.json 2> $O/${v}_$1.log || { echo "$v $1 failed"; tail -3 $O/${v}_$1.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$1.json'));print('$v','$1',round(d['value'],2),d['unit'],round(d['ms_per_step'],2),'ms')"
  done
done
