#!/usr/bin/env python3
"""Static VALU instruction mix of every gfx950 kernel in the product build,
priced with the issue costs tools/valu_probe.hip measured per opcode
(profiles/r01_valu_probe.txt, 4 waves per SIMD, independent streams).

usage: tools/isa_mix.py [--json profiles/isa_mix_r05.json]

The device code object is unbundled from each product object file
(cleisthenes_amd/csrc/*.o: .hip_fatbin -> clang-offload-bundler ->
llvm-objdump), and every VALU mnemonic of every kernel symbol is counted.
Classes (the probe's two issue classes on gfx950):
  A (~4.3-4.8 SIMD clk per wave64 instruction): v_alignbit, v_add3, v_perm, v_bfi
  B (~2.4-2.8): v_bitop3, v_xor, v_add, v_and, v_lshrrev (probed) and the
    other one- and two-operand ALU ops of the same encodings (v_mov, v_or,
    v_lshlrev, v_sub, v_not, v_cndmask, v_cmp, ...)
  U (not probed: v_mul_lo / v_mad_u64 / transcendental / readfirstlane /
    other three-operand VOP3): priced at class A's cost, their share reported
The static mix is the dynamic mix where a kernel is straight-line (the FFT
transforms) or dominated by one loop body (SHA, the GEMV); bench.py uses the
cost per instruction of each kernel to price the step's PMC VALU counts
(valu_step.issue_priced) instead of a flat 4 clocks.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
OBJS = ("kernels.o", "rs_fft.o", "gf_regen.o", "wire.o")
# w4 independent-stream cost (SIMD clk per wave64 instruction) from profiles/r01_valu_probe.txt
PROBED = {"v_alignbit_b32": 4.79, "v_add3_u32": 4.45, "v_perm_b32": 4.30, "v_bfi_b32": 4.29,
          "v_bitop3_b32": 2.78, "v_xor_b32": 2.62, "v_add_u32": 2.64, "v_lshrrev_b32": 2.44, "v_and_b32": 2.66,
          "v_fma_f32": 2.62}
COST_A, COST_B = 4.46, 2.63  # class means of the probed opcodes
CLASS_A = ("v_alignbit", "v_alignbyte", "v_add3", "v_perm", "v_bfi", "v_lshl_add", "v_add_lshl", "v_lshl_or",
           "v_and_or", "v_or3", "v_xad", "v_xor3", "v_mad_u32_u24", "v_bfe", "v_med3", "v_max3", "v_min3")
CLASS_B = ("v_bitop3", "v_xor", "v_add", "v_and", "v_lshrrev", "v_lshlrev", "v_ashrrev", "v_or", "v_mov",
           "v_sub", "v_subrev", "v_not", "v_cndmask", "v_cmp", "v_max_", "v_min_", "v_fma_f32", "v_mul_f32",
           "v_cvt_", "v_nop", "v_bfrev", "v_ffbh", "v_ffbl", "v_cmpx")


def opclass(m):
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", m)
    if base in PROBED:
        return ("A" if PROBED[base] > 3.5 else "B"), PROBED[base]
    if base.startswith(CLASS_A):
        return "A", COST_A
    if base.startswith(CLASS_B):
        return "B", COST_B
    return "U", COST_A


def disassemble(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fat")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                          text=True).stdout


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    return [o.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip() for o in out]


def mix(objs=OBJS):
    kernels = {}
    with tempfile.TemporaryDirectory() as tmp:
        for o in objs:
            path = os.path.join(ROOT, "cleisthenes_amd", "csrc", o)
            cur = None
            for line in disassemble(path, tmp).splitlines():
                h = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if h:
                    cur = h.group(1)
                    kernels.setdefault(cur, Counter())
                    continue
                t = line.split()
                if cur and t and t[0].startswith("v_"):
                    kernels[cur][t[0]] += 1
    names = list(kernels)
    res = {}
    for mangled, dem in zip(names, demangle(names)):
        c = kernels[mangled]
        n = sum(c.values())
        if not n:
            continue
        cls = Counter()
        clk = 0.0
        for m, k in c.items():
            cl, cost = opclass(m)
            cls[cl] += k
            clk += cost * k
        res[dem] = {"valu_static": n, "class_A": cls["A"], "class_B": cls["B"], "unprobed": cls["U"],
                    "clk_per_instr": round(clk / n, 3),
                    "top": dict(c.most_common(6))}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    a = ap.parse_args()
    res = mix()
    for k, v in sorted(res.items(), key=lambda x: -x[1]["valu_static"]):
        print(f"{k:60s} {v['valu_static']:7d}  A {v['class_A']:6d}  B {v['class_B']:6d}  U {v['unprobed']:5d}"
              f"  {v['clk_per_instr']:.2f} clk/instr")
    if a.json:
        json.dump({"source": "tools/isa_mix.py over cleisthenes_amd/csrc/{" + ",".join(OBJS) + "}",
                   "probe": "profiles/r01_valu_probe.txt (w4, independent streams)",
                   "kernels": res}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
