#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, kernel-trace only) behind profiles/r02_*_pmc_summary.json
# (summarise with tools/pmc_summary.py OUT.json DIR/p1 DIR/p2 DIR/p3 DIR/p4). The c4_notr leg needs the
# diagnostic build: make -C 3dg-vol-renderer_amd/csrc BUILD=../build-diag OUT=../../tools_dbg/libvr_diag.so
#   DEVFLAGS="... -DVR_DIAG_SKIP_TR_STORES" (see DESIGN.md §3).
#   C4 ray-march frame (product and the diagnostic no-Tr-store build) and C2 multi-scatter (ff_path_kernel).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_r02; mkdir -p $O
SETS=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES")
run() {  # name, lib, bench args...
  local name=$1 lib=$2; shift 2
  local i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    VR_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $O/$name/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --flops 0 "$@" > $O/$name/p$i.log 2>&1
    local rc=$?; echo "$name pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
mkdir -p $O/c4 $O/c4_notr $O/c2ms
run c4 "" 
run c4_notr $GRAFT_REPO_ROOT/tools_dbg/libvr_diag.so
run c2ms "" --config c2 --integrator multiscatter --spp 16
echo done
