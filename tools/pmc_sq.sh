#!/bin/bash
# One SQ-counter pass (rocprofv3 --pmc, kernel trace only) over tools/diag_c4.py for the product library
# and every build under _ab/:  tools/pmc_sq.sh -> gpurun_out/pmc_sq/<variant>.json (tools/pmc_summary.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_sq; mkdir -p $O
SET="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
for v in base ${PMC_VARIANTS:-}; do
  if [ $v = base ]; then lib=""; else lib=$GRAFT_REPO_ROOT/_ab/$v/libvr_hip.so; fi
  VR_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --pmc $SET -d $O/$v -o run --output-format csv -- python3 tools/diag_c4.py --frames 1 --counts 0 > $O/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/pmc_summary.py $O/$v.json $O/$v > /dev/null
  python3 -c "
import json; d=json.load(open('$O/$v.json'))
for k,r in d.items():
  if 'secondary_ww' in k or 'march_kernel' in k or 'record_list' in k:
    print('$v', k[10:40], {x: (round(r[x]/1e9,3) if r[x] > 1e6 else round(r[x],3)) for x in ('SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_WAVE_CYCLES','SQ_WAIT_ANY','SQ_WAIT_INST_ANY','SQ_ACTIVE_INST_ANY','SQ_ACTIVE_INST_VALU','SQ_BUSY_CYCLES') if x in r})
"
done
