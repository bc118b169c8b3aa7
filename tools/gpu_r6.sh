#!/bin/bash
# Round-6 GPU check: the -m gpu suite (no -x: every failure listed), then the C4 bench line without the CPU
# baseline and one instrumented C4 frame's statistics (slow-path rays with the chord band).
#   gpurun -- bash tools/gpu_r6.sh TAG [pytest -k expression]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6}; mkdir -p $OUT
K=${2:+-k "$2"}
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread ${2:+-k "$2"} > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -2
grep -E "^FAILED|^ERROR" $OUT/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest exit $rc"; tail -20 $OUT/gpu_tests.log; exit 1; }
timeout -k 10 400 python3 bench.py --cpu-budget 0 > $OUT/c4.json 2> $OUT/c4.log || { tail -5 $OUT/c4.log; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c4.json'));r=d['roofline'];print(round(d['value'],2), d['unit'], round(d['ms_per_step'],2), 'frac', round(r['frac'],4), 'alg_s8d', round(r['alg_frac_s8d'],4), r['stage_ms'])"
timeout -k 10 300 python3 tools/diag_c4.py --frames 2 --counts 0 > $OUT/diag.json 2> $OUT/diag.log || { tail -5 $OUT/diag.log; exit 1; }
cat $OUT/diag.json
exit $rc
