"""Static ISA census of one kernel: instructions per source function, by class (VALU / SALU /
VMEM / SMEM / LDS / branch), from the disassembly of a device code object built with line tables.

  hipcc ... -gline-tables-only --cuda-device-only -c kernels/vr_gauss.hip -o x.co
  clang-offload-bundler --unbundle --type=o --input=x.co --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=x.o
  llvm-objdump -d x.o > x.s
  python3 tools/isa_count.py x.o x.s secondary_ww_kernelILi256ELi18ELb0ELb0ELi6ELi9ELb1ELb1E [--top 30]

Every instruction address is symbolized with its inline stack (llvm-symbolizer --inlining) and
counted for the innermost frame of our own sources (a header function such as fmaf / erff counts
for the function that called it), and for the kernel-body line the stack starts from (which
loop of the kernel it belongs to). Static counts: code size per region, not executed counts."""
import argparse
import collections
import json
import os
import re
import subprocess

ap = argparse.ArgumentParser()
ap.add_argument("obj")
ap.add_argument("asm")
ap.add_argument("kernel", help="substring of the kernel's mangled name")
ap.add_argument("--top", type=int, default=25, help="kernel-body lines to print")
args = ap.parse_args()
SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def iclass(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_") or (op.startswith("buffer_") and "scratch" in op):
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


lines = open(args.asm).read().splitlines()
start = next((i for i, ln in enumerate(lines)
              if re.match(r"^[0-9a-f]+ <.*" + re.escape(args.kernel) + r".*>:$", ln)), None)
if start is None:
    raise SystemExit(f"kernel {args.kernel!r} not found")
insts = []  # (address, class)
for ln in lines[start + 1:]:
    if re.match(r"^[0-9a-f]+ <(?!L\d+>).*>:$", ln):
        break  # next symbol (local labels <Lnnn> stay inside the kernel)
    m = re.match(r"^\s+([a-z_][a-z0-9_]*)\b.*//\s*([0-9A-Fa-f]+):", ln)
    if m:
        insts.append((int(m.group(2), 16), iclass(m.group(1))))
out = subprocess.run([SYM, f"--obj={args.obj}", "--inlining"], input="\n".join(hex(a) for a, _ in insts) + "\n",
                     capture_output=True, text=True, check=True).stdout
blocks = out.strip("\n").split("\n\n")
if len(blocks) != len(insts):
    raise SystemExit(f"symbolizer returned {len(blocks)} stacks for {len(insts)} instructions")
by_func = collections.defaultdict(collections.Counter)
by_body = collections.defaultdict(collections.Counter)
total = collections.Counter()
for (addr, c), blk in zip(insts, blocks):
    fr = blk.split("\n")
    frames = [(fr[k], fr[k + 1]) for k in range(0, len(fr) - 1, 2)]  # innermost first
    own = next(((f, loc) for f, loc in frames if "/opt/rocm" not in loc), frames[-1])
    fname = own[0].split("(")[0].split("<")[0].split("::")[-1]
    by_func[fname][c] += 1
    body = frames[-1][1].rsplit(":", 1)[0]  # kernel-body file:line
    by_body[os.path.basename(body)][c] += 1
    total[c] += 1
print(json.dumps({"kernel": args.kernel, "instructions": len(insts), "total": dict(total)}))
hdr = f"{'':44s} {'valu':>6s} {'salu':>6s} {'vmem':>5s} {'lds':>5s} {'smem':>5s} {'br':>5s} {'scr':>5s}"
print("\nby function (innermost own frame)\n" + hdr)
for r, c in sorted(by_func.items(), key=lambda kv: -kv[1]["valu"]):
    print(f"{r[:44]:44s} {c['valu']:6d} {c['salu']:6d} {c['vmem']:5d} {c['lds']:5d} {c['smem']:5d} {c['branch']:5d} {c['scratch']:5d}")
print("\nby kernel-body line\n" + hdr)
for r, c in sorted(by_body.items(), key=lambda kv: -kv[1]["valu"])[:args.top]:
    print(f"{r[:44]:44s} {c['valu']:6d} {c['salu']:6d} {c['vmem']:5d} {c['lds']:5d} {c['smem']:5d} {c['branch']:5d} {c['scratch']:5d}")
