#!/bin/bash
# Free-flight determinism + phase diagnostics: frame hashes of the in-tree library (twice) and _ab builds,
# then the phase statistics of _ab/smdiag (VR_DIAG_FFSM).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ffsm
for t in cur cur2 "$@"; do lib=$PWD/_ab/$t/libvr_hip.so; [ $t = cur -o $t = cur2 ] && lib=$PWD/3dg-vol-renderer_amd/libvr_hip.so
  VR_LIB_PATH=$lib FRAME_SAVE=gpurun_out/ffsm/$t timeout -k 10 150 python3 tools/ff_frame_hash.py c2:multiscatter:4 c3:freeflight:1 > gpurun_out/ffsm/$t.hash 2>&1 || exit 1
  echo "$t $(grep -v amdgpu.ids gpurun_out/ffsm/$t.hash | tr '\n' ' ')"; done
if [ -d _ab/smdiag ]; then
VR_LIB_PATH=$PWD/_ab/smdiag/libvr_hip.so DIAG_KIND=ffsm timeout -k 10 150 python3 tools/ff_diag.py c2 multiscatter 16 > gpurun_out/ffsm/smdiag.json 2>gpurun_out/ffsm/smdiag.log && cat gpurun_out/ffsm/smdiag.json; fi
