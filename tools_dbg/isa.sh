#!/bin/bash
# ISA of vr_gauss.hip (gfx950) into /tmp/isa/gauss.s + per-kernel VGPR / scratch / occupancy summary
mkdir -p /tmp/isa && cd /root/repo/3dg-vol-renderer_amd/csrc
/opt/rocm/bin/hipcc -std=c++20 -O3 -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics --cuda-device-only -S \
  kernels/vr_gauss.hip -o /tmp/isa/gauss.s 2>/dev/null
awk '/^_Z[A-Za-z0-9_]*:/{k=$1} /; NumVgprs:|; ScratchSize:|; Occupancy:/{if(k!="")print k, $2, $3}' /tmp/isa/gauss.s \
  | sed 's/_ZN2vr3dev//; s/EEEvNS_10RenderArgs.*:/ /' | grep -E "${1:-secondary_ww}" | paste - - -
