cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m8; mkdir -p $O
timeout -k 10 300 python3 bench.py --cpu-budget 0 --flops 0 --steps 5 > $O/b.json 2> $O/b.log || { tail $O/b.log; exit 1; }
python3 -c "
import json;d=json.load(open('$O/b.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['stage_ms'])"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "full_size or raymarch_gaussians_matches or pure or deterministic or tiles or capacity" > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log
exit $rc
