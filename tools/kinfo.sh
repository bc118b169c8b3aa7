#!/bin/bash
# Register / spill / LDS census of the device kernels of one source under extra -D flags:
#   tools/kinfo.sh vr_gauss "-DFOO=1" [kernel-name-regex]
set -e
cd "$(dirname "$0")/../3dg-vol-renderer_amd/csrc"
k=$1; flags=$2; pat=${3:-secondary_ww_kernel}
t=$(mktemp -d)
/opt/rocm/bin/hipcc -std=c++20 -O3 -fPIC -ffp-contract=off -Wno-unused-function -Wno-unused-result --offload-arch=gfx950 \
  -munsafe-fp-atomics -fno-slp-vectorize $flags --cuda-device-only -c kernels/$k.hip -o $t/k.co
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/k.co \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/k.o
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $t/k.o | awk -v pat="$pat" '
  /\.name:/ {name=$2} /\.vgpr_count:/ {v=$2} /\.vgpr_spill_count:/ {vs=$2} /\.sgpr_spill_count:/ {ss=$2}
  /\.group_segment_fixed_size:/ {lds=$2}
  /\.wavefront_size:/ { if (name ~ pat) printf "%-90s vgpr %s vspill %s sspill %s lds %s\n", substr(name,1,90), v, vs, ss, lds }'
rm -rf $t
