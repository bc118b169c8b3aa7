#!/bin/bash
# ISA census of the product secondary kernel (tools/isa_count.py), built with line tables into /tmp/isa.
set -e
mkdir -p /tmp/isa
cd "$(dirname "$0")/../3dg-vol-renderer_amd/csrc"
/opt/rocm/bin/hipcc -std=c++20 -O3 -fPIC -ffp-contract=off -Wno-unused-function -Wno-unused-result --offload-arch=gfx950 \
  -munsafe-fp-atomics -fno-slp-vectorize -gline-tables-only --cuda-device-only $2 -c kernels/vr_gauss.hip -o /tmp/isa/g.co
cd /tmp/isa
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=g.co --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=g.o
/opt/rocm/lib/llvm/bin/llvm-objdump -d g.o > g.s
cd - > /dev/null
python3 ../../tools/isa_count.py /tmp/isa/g.o /tmp/isa/g.s ${1:-secondary_ww_kernelILi256ELi18ELb0ELb0ELi6ELi9ELb1ELb1E} --top ${TOP:-12}
