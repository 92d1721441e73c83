#!/usr/bin/env python3
"""Summarise a tools/profile.sh run per kernel ROLE (average per dispatch).

usage: tools/pmc_summary.py gpurun_out/prof_<tag> [--json out.json] [--traffic profiles/pmc_traffic_rNN.json --config c2]

Kernels that serve two roles in one bench step are split by dispatch order:
gf_rows_kernel<*> -> [encode] / [decode], sha_rows_kernel<false> ->
[leaves] / [regen].  HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE
(KiB) reads 1/2 of a wide streaming read on gfx950 -> x2; WRITE_SIZE (KiB)
is exact for 16-B-per-lane stores.
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROLES = {"gf_rows_kernel": ["encode", "decode"], "sha_rows_kernel<false>": ["leaves", "regen"]}
# FFT codec (rs_fft.hip): the encode and decode transforms are separate
# instantiations (last template argument = mode), and gf_rows_kernel only
# regenerates the missing data rows of interpolate
# SHA-256 compressions per launch of the bench's c2 step (I=1024, N=128,
# S=23832: 373 blocks per shard; verify adds 2 per branch level, d=7)
COMPRESSIONS = {("c2", "sha_rows_kernel<leaves>"): 1024 * 128 * 373,
                ("c2", "sha_rows_kernel<verify>"): 1024 * 128 * (373 + 14)}
FFT_ROLES = {"gf_rows_kernel": ["missing-data"], "sha_rows_kernel<false>": ["leaves", "regen"]}


def base(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def _fft_named(k):
    if k.startswith("rs_fft_kernel<"):
        return k + ("[encode]" if k.endswith(", 0>") else "[decode]")
    return None


FFT_MODE = False


def role_name(k, ordinal):
    f = _fft_named(k)
    if f:
        return f
    for prefix, roles in (FFT_ROLES if FFT_MODE else ROLES).items():
        if k.startswith(prefix):
            return f"{k}[{roles[ordinal % len(roles)]}]"
    return k


def dispatch_roles(rows):
    """Dispatch_Id -> role-qualified kernel name (by order of appearance)."""
    seen = defaultdict(int)
    out = {}
    for did, k in sorted({(int(r["Dispatch_Id"]), base(r["Kernel_Name"])) for r in rows}):
        out[did] = role_name(k, seen[k])
        seen[k] += 1
    return out


def load_pmc(d):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f) or sub == "trace":
            continue
        rows = list(csv.DictReader(open(f)))
        roles = dispatch_roles(rows)
        for r in rows:
            k = roles[int(r["Dispatch_Id"])]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    return {k: {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()} for k, cs in per.items()}


def load_trace(d):
    f = os.path.join(d, "trace", "run_kernel_trace.csv")
    res = defaultdict(list)
    if os.path.exists(f):
        rows = list(csv.DictReader(open(f)))
        seen = defaultdict(int)
        for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
            k = base(r["Kernel_Name"])
            res[role_name(k, seen[k])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            seen[k] += 1
    return {k: (len(v), sum(v) / len(v)) for k, v in res.items()}


def summarise(d):
    global FFT_MODE
    f = os.path.join(d, "trace", "run_kernel_trace.csv")
    FFT_MODE = os.path.exists(f) and "rs_fft_kernel" in open(f).read()
    pm, tr = load_pmc(d), load_trace(d)
    rows = {}
    for k in sorted(set(pm) | set(tr)):
        c = pm.get(k, {})
        calls, ns = tr.get(k, (0, 0.0))
        r = {"calls_traced": calls, "avg_us": round(ns / 1e3, 2)}
        r.update({kk: round(v) for kk, v in sorted(c.items())})
        if "FETCH_SIZE" in c:
            r["hbm_read_bytes"] = round(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            r["hbm_write_bytes"] = round(c["WRITE_SIZE"] * 1024)
        if "GRBM_GUI_ACTIVE" in c and ns:
            r["clock_GHz_est"] = round(c["GRBM_GUI_ACTIVE"] / 8 / ns, 3)
        if "SQ_INSTS_VALU" in c and ns:
            ghz = r.get("clock_GHz_est", 2.4)
            # integer VOP3 (alignbit/bitop3/perm/add3) issue one wave-instruction
            # per 4 clk per SIMD (16 lanes/clk); 1024 SIMDs
            r["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] / (ns * 1e-9) / (1024 * ghz * 1e9 / 4), 3)
        rows[k] = r
    return rows


if __name__ == "__main__":
    d = sys.argv[1]
    rows = summarise(d)
    for k, r in rows.items():
        print(k)
        for kk, v in r.items():
            print(f"    {kk:28s} {v}")
    if "--json" in sys.argv:
        json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    if "--traffic" in sys.argv:
        cfg = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "c2"
        bench_names = {"gf_rows_kernel": "gf_rows_kernel<encode>", "sha_rows_kernel<false>[leaves]":
                       "sha_rows_kernel<leaves>", "sha_rows_kernel<true>": "sha_rows_kernel<verify>"}
        out = {"config": cfg, "source": os.path.relpath(d), "kernels": {}}
        for k, r in rows.items():
            name = None
            if k.startswith("gf_rows_kernel") and k.endswith("[encode]"):
                name = "gf_rows_kernel<encode>"
            elif k.startswith("rs_fft_kernel") and k.endswith("[encode]"):
                name = "rs_fft_kernel<encode>"
            else:
                name = bench_names.get(k)
            if name and "hbm_read_bytes" in r and "hbm_write_bytes" in r:
                out["kernels"][name] = {"hbm_bytes_per_launch": r["hbm_read_bytes"] + r["hbm_write_bytes"],
                                        "hbm_read_bytes": r["hbm_read_bytes"], "hbm_write_bytes": r["hbm_write_bytes"],
                                        "avg_us_profiled": r["avg_us"], "SQ_INSTS_VALU": r.get("SQ_INSTS_VALU")}
                comp = COMPRESSIONS.get((cfg, name))
                if comp and r.get("SQ_INSTS_VALU"):
                    out["kernels"][name]["compressions_per_launch"] = comp
                    out["kernels"][name]["valu_per_compression"] = round(r["SQ_INSTS_VALU"] / comp, 3)
        json.dump(out, open(sys.argv[sys.argv.index("--traffic") + 1], "w"), indent=1)
