#!/usr/bin/env python3
"""Summarise a tools/profile.sh run per kernel ROLE (average per dispatch).

usage: tools/pmc_summary.py gpurun_out/prof_<tag> [--config c2] [--instances 1024] [--last K]
       [--json out.json] [--traffic profiles/pmc_traffic_rNN.json]

Roles come from kernel name + grid size (tools/trace_summary.py: leaves vs
regen hashing, encode vs decode transform), averaged over the last K
dispatches of each role (the timed steps).  HBM bytes follow
MI355X_MICROARCH.md "HBM": FETCH_SIZE (KiB) reads 1/2 of a wide streaming
read on gfx950 -> x2; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_summary import CONFIGS, read_lines, role, shared_path, summarize  # noqa: E402


def blocks(S):
    return (S + 9 + 63) // 64


def load_pmc(d, n, k, inst, last, path=False):
    per = defaultdict(lambda: defaultdict(list))  # role -> counter -> [per-dispatch value]
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f) or sub == "trace":
            continue
        acc = defaultdict(float)  # (role, grid, dispatch, counter) -> summed value (over XCDs / instances)
        for r in csv.DictReader(read_lines(f)):
            g = int(r["Grid_Size"])
            rl = role(r["Kernel_Name"], g, n, k, inst, path)
            acc[(rl, g, int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        biggest = defaultdict(int)
        for (rl, g, _, _) in acc:
            biggest[rl] = max(biggest[rl], g)
        for (rl, g, did, cn), v in sorted(acc.items(), key=lambda x: x[0][2]):
            per[rl if g == biggest[rl] else f"{rl}[grid {g}]"][cn].append(v)
    out = {}
    for rl, cs in per.items():
        out[rl] = {cn: (sum(vs[-last:]) / len(vs[-last:]) if last else sum(vs) / len(vs)) for cn, vs in cs.items()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--instances", type=int, default=1024)
    ap.add_argument("--value-bytes", type=int, default=0, help="default: the config's (bench.py CONFIGS)")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--json")
    ap.add_argument("--traffic")
    ap.add_argument("--value-form", default="row view", choices=("row view", "joined"),
                    help="the bench's interpolate value form in the profiled run (bench.py --join: joined)")
    a = ap.parse_args()
    n, f = CONFIGS[a.config]
    k = n - 2 * f
    vb = a.value_bytes or {"c1": 1 << 20, "c2": 1 << 20, "c3": 4 << 20, "c4": 64 << 10}[a.config]
    S = (vb + k - 1) // k
    d = 0
    while (1 << d) < n:
        d += 1
    path = shared_path(a.config, vb)
    pm = load_pmc(a.dir, n, k, a.instances, a.last, path)
    tf = os.path.join(a.dir, "trace", "run_kernel_trace.csv")
    tr = summarize(tf, a.config, a.instances, a.last) if os.path.exists(tf) else {}
    # SHA-256 compressions per launch: leaves hash all N rows, ECHO verify the
    # N-f received rows (+2 per branch level)
    comp = {"sha_rows_kernel<leaves>": a.instances * n * blocks(S),
            "sha_rows_kernel<verify>": a.instances * (n - f) * (blocks(S) + 2 * d),
            # receive step: the received rows of t + the regenerated rows of t-1
            # (the f absent rows, plus the bench's one corrupted ECHO in 10 % of instances)
            "sha_rx_kernel<verify+regen>": a.instances * (n - f) * (blocks(S) + 2 * d)
            + (a.instances * f + a.instances // 10) * blocks(S),
            # C4: the receive step hashes leaves only; merkle_path_kernel walks the branches
            "sha_rx_kernel<leaves+regen>": a.instances * (n - f) * blocks(S)
            + (a.instances * f + a.instances // 10) * blocks(S)}
    rows = {}
    for rl in sorted(set(pm) | set(tr)):
        c = pm.get(rl, {})
        t = tr.get(rl, {})
        r = {"timed_launches": t.get("timed_launches", 0), "avg_ms_traced": t.get("avg_ms")}
        r.update({kk: round(v) for kk, v in sorted(c.items())})
        if "FETCH_SIZE" in c:
            r["hbm_read_bytes"] = round(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            r["hbm_write_bytes"] = round(c["WRITE_SIZE"] * 1024)
        if rl in comp and "SQ_INSTS_VALU" in c:
            r["compressions_per_launch"] = comp[rl]
            r["valu_per_compression"] = round(c["SQ_INSTS_VALU"] * 64 / comp[rl], 1)
        rows[rl] = r
    for rl, r in rows.items():
        print(rl)
        for kk, v in r.items():
            print(f"    {kk:28s} {v}")
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)
    if a.traffic:
        out = {"config": a.config, "instances": a.instances, "value_form": a.value_form,
               "source": os.path.relpath(a.dir), "kernels": {}}
        for rl, r in rows.items():
            if "hbm_read_bytes" in r and "hbm_write_bytes" in r:
                out["kernels"][rl] = {"hbm_bytes_per_launch": r["hbm_read_bytes"] + r["hbm_write_bytes"],
                                      "hbm_read_bytes": r["hbm_read_bytes"], "hbm_write_bytes": r["hbm_write_bytes"],
                                      "avg_ms_traced": r["avg_ms_traced"], "SQ_INSTS_VALU": r.get("SQ_INSTS_VALU"),
                                      "valu_per_compression": r.get("valu_per_compression")}
        # roofline_decode's unit (bench.py): the receive step's decode kernels together
        parts = [rl for rl in out["kernels"] if "[grid" not in rl and (
            rl.startswith(("decode_prepare", "gf_regen_kernel")) or rl == "rs_fft_kernel<decode>")]
        if len(parts) == 3:
            ks = [out["kernels"][p_] for p_ in parts]
            out["kernels"]["decode: prepare + gf_regen_kernel + rs_fft_kernel<decode>"] = {
                "hbm_bytes_per_launch": sum(x["hbm_bytes_per_launch"] for x in ks),
                "hbm_read_bytes": sum(x["hbm_read_bytes"] for x in ks),
                "hbm_write_bytes": sum(x["hbm_write_bytes"] for x in ks),
                "avg_ms_traced": round(sum(x["avg_ms_traced"] or 0 for x in ks), 4), "parts": parts}
        json.dump(out, open(a.traffic, "w"), indent=1)


if __name__ == "__main__":
    main()
