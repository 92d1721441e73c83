#!/usr/bin/env python3
"""Copy / kernel overlap inside a timed window of a rocprofv3 trace
(--kernel-trace --memory-copy-trace, CSV): how long host->device and
device->host copies (SDMA) and the zero-copy / blit kernels were active,
alone and together -- is the PCIe link carrying both directions at once?

usage: python tools/copy_overlap.py <trace dir> <t0_ns> <t1_ns>"""
import csv
import glob
import json
import os
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main(d, t0, t1):
    ev = []  # (start, end, class)
    for r in rows(d, "*memory_copy_trace.csv"):
        kind = r.get("Direction", r.get("Operation", ""))
        cls = "sdma_h2d" if "HOST_TO_DEVICE" in kind else ("sdma_d2h" if "DEVICE_TO_HOST" in kind else "sdma_other")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cls))
    for r in rows(d, "*kernel_trace.csv"):
        name = r["Kernel_Name"]
        cls = ("k_gather" if "gather" in name else "k_blit" if "__amd_rocclr" in name else "k_compute")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cls))
    ev = [(max(a, t0), min(b, t1), c) for a, b, c in ev if b > t0 and a < t1]
    classes = ("sdma_h2d", "sdma_d2h", "k_gather", "k_blit", "k_compute")
    edges = sorted([(a, 1, c) for a, b, c in ev] + [(b, -1, c) for a, b, c in ev])
    cnt = {c: 0 for c in classes + ("sdma_other",)}
    busy = {c: 0 for c in classes}
    combo = {}
    last = t0
    for t, delta, c in edges:  # sweep: between consecutive edges the active set is constant
        if t > last:
            act = tuple(x for x in classes if cnt[x] > 0)
            for x in act:
                busy[x] += t - last
            key = " + ".join(act) or "idle"
            combo[key] = combo.get(key, 0) + t - last
            last = t
        cnt[c] += delta
    if t1 > last:
        combo["idle"] = combo.get("idle", 0) + t1 - last
    tot = t1 - t0
    out = {"window_ms": round(tot / 1e6, 3), "busy_frac": {c: round(v / tot, 3) for c, v in busy.items()},
           "combinations_frac": {k: round(v / tot, 3) for k, v in sorted(combo.items(), key=lambda kv: -kv[1])[:12]}}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
