#!/usr/bin/env python3
"""Loaded clock and VALU issue per kernel role, from a serial-schedule run.

usage: tools/clock_summary.py gpurun_out/pmc_<tag> --config c2 [--instances 1024] [--last K] [--json out.json]

The directory is a tools/pmc_passes.sh run of `bench.py --pipeline 0` with at
least the sq2 pass (GRBM_GUI_ACTIVE, SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_ANY,
...) and sq1 (SQ_INSTS_VALU): under the serial schedule every kernel runs
alone, so its kernel-trace duration and its counters describe the same
execution (--pmc serialises dispatches anyway).

Per role (MI355X_MICROARCH.md, "DVFS give-back"): clock = GRBM_GUI_ACTIVE / 8
XCDs / duration.  SQ_ACTIVE_INST_VALU counts wave64 VALU instructions on
gfx950 (it equals SQ_INSTS_VALU to 0.1 %, profiles/r04b_*), not busy cycles:
no counter measures the VALU's busy fraction.  valu_at_4clk = 4 * VALU /
(1024 SIMDs * cycles) is only a flat-4-clock reference (v_bitop3, v_add and
shifts issue in ~2.5 clocks, v_perm / v_alignbit / v_add3 in ~4.4:
profiles/r01_valu_probe.txt); bench.py prices the counts per opcode instead
(tools/isa_mix.py, valu_step.issue_priced_ms / chain_priced_ms).
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_summary import CONFIGS, read_lines, role, summarize  # noqa: E402

SIMDS = 1024


def counters(d, sub, n, k, inst, last):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        return {}
    acc = defaultdict(float)
    for r in csv.DictReader(read_lines(f)):
        g = int(r["Grid_Size"])
        acc[(role(r["Kernel_Name"], g, n, k, inst), g, int(r["Dispatch_Id"]), r["Counter_Name"])] += float(
            r["Counter_Value"])
    biggest = defaultdict(int)
    for (rl, g, _, _) in acc:
        biggest[rl] = max(biggest[rl], g)
    per = defaultdict(lambda: defaultdict(list))
    for (rl, g, _, cn), v in sorted(acc.items(), key=lambda x: x[0][2]):
        per[rl if g == biggest[rl] else f"{rl}[grid {g}]"][cn].append(v)
    return {rl: {cn: sum(vs[-last:]) / len(vs[-last:]) for cn, vs in cs.items()} for rl, cs in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--instances", type=int, default=1024)
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--json")
    a = ap.parse_args()
    n, f = CONFIGS[a.config]
    k = n - 2 * f
    tr = summarize(os.path.join(a.dir, "trace", "run_kernel_trace.csv"), a.config, a.instances, a.last)
    c = {}
    for sub in ("sq1", "sq2"):
        for rl, cs in counters(a.dir, sub, n, k, a.instances, a.last).items():
            c.setdefault(rl, {}).update(cs)
    rows, cyc_sum, ms_sum = {}, 0.0, 0.0
    for rl in sorted(set(tr) & set(c)):
        cs, ms = c[rl], tr[rl]["avg_ms"]
        if "GRBM_GUI_ACTIVE" not in cs or ms < 0.3:  # the quotient reads high below ~0.3 ms (the guide)
            continue
        cyc = cs["GRBM_GUI_ACTIVE"] / 8
        r = {"alone_ms": ms, "clock_ghz": round(cyc / (ms * 1e-3) / 1e9, 3)}
        vi = cs.get("SQ_INSTS_VALU")
        if vi:
            r["valu_instr"] = int(vi)
            r["valu_at_4clk"] = round(4 * vi / (SIMDS * cyc), 3)
        if "SQ_ACTIVE_INST_VALU" in cs and vi:
            r["active_inst_valu_over_insts_valu"] = round(cs["SQ_ACTIVE_INST_VALU"] / vi, 4)
        rows[rl] = r
        cyc_sum += cyc
        ms_sum += ms
    out = {"config": a.config, "instances": a.instances, "source": os.path.relpath(a.dir),
           "schedule": "serial (--pipeline 0): each kernel alone", "kernels": rows,
           "clock_ghz_weighted": round(cyc_sum / (ms_sum * 1e-3) / 1e9, 3) if ms_sum else None}
    for rl, r in rows.items():
        print(f"{rl:44s} {r}")
    print("clock (duration-weighted):", out["clock_ghz_weighted"], "GHz")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
