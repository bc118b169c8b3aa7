# Free-flight check: GPU parity tests of the free-flight/inverse paths, then the FF bench lines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ffc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_freeflight.py tests/test_gpu_inverse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ffc/tests.log 2>&1 || { tail -30 gpurun_out/ffc/tests.log; exit 1; }
tail -2 gpurun_out/ffc/tests.log
for c in "c2 multiscatter 16" "c5 multiscatter 16" "c3 freeflight 4" "c4 multiscatter 1"; do
  set -- $c
  timeout -k 10 120 python3 bench.py --config $1 --integrator $2 --spp $3 --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/ffc/$1.json 2> gpurun_out/ffc/$1.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ffc/$1.json'));r=d.get('roofline') or {};print('$1 $2',round(d['value'],2),'Mpaths/s',round(d['ms_per_step'],1),'ms','frac',r.get('frac'),'alg',r.get('alg_frac'),'path_ms',r.get('kernel_ms'),'nee',(r.get('nee_kernel') or {}).get('kernel_ms'))"
done
