#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch).
usage: tools/pmc_summary.py gpurun_out/prof_<tag> [--json out.json]"""
import csv
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "")


def load(d):
    per = defaultdict(lambda: defaultdict(float))   # kernel -> counter -> sum
    disp = defaultdict(set)
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for k, cs in per.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    return out


def trace(d):
    f = os.path.join(d, "trace", "run_kernel_stats.csv")
    res = {}
    if os.path.exists(f):
        for r in csv.DictReader(open(f)):
            res[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    return res


if __name__ == "__main__":
    d = sys.argv[1]
    pm, tr = load(d), trace(d)
    rows = {}
    for k in sorted(set(pm) | set(tr)):
        c = pm.get(k, {})
        calls, ns = tr.get(k, (0, 0.0))
        r = {"calls": calls, "avg_us": round(ns / 1e3, 2)}
        r.update({kk: round(v) for kk, v in sorted(c.items())})
        if "FETCH_SIZE" in c:
            # gfx950: FETCH_SIZE (KB) reads half the bytes of a wide streaming read
            r["hbm_read_bytes_corr"] = round(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            r["hbm_write_bytes"] = round(c["WRITE_SIZE"] * 1024)
        if "GRBM_GUI_ACTIVE" in c and ns:
            r["clock_GHz_est"] = round(c["GRBM_GUI_ACTIVE"] / 8 / ns, 3)
        if "SQ_INSTS_VALU" in c and ns:
            # wave-instructions/s vs 256 CU x 4 SIMD x (1 wave-instr / 2 clk) at the estimated clock
            ghz = r.get("clock_GHz_est", 2.4)
            r["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] / (ns * 1e-9) / (1024 * ghz * 1e9 / 2), 3)
        rows[k] = r
    for k, r in rows.items():
        print(k)
        for kk, v in r.items():
            print(f"    {kk:28s} {v}")
    if "--json" in sys.argv:
        json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
