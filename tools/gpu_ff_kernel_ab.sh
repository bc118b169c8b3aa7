cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ffk
for c in "c3 freeflight 4" "c4 multiscatter 1" "c5 multiscatter 16" "main multiscatter 256"; do set -- $c
  for k in 1 2; do timeout -k 10 200 python3 bench.py --config $1 --integrator $2 --spp $3 --steps 3 --warmup 1 --cpu-budget 0 --flops 0 --opt ff_kernel=$k > gpurun_out/ffk/$1_$k.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ffk/$1_$k.json'));print('$1 kernel=$k', round(d['value'],1), round(d['ms_per_step'],1))"; done; done
