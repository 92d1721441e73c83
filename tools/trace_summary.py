#!/usr/bin/env python3
"""Per-kernel-role durations from a rocprofv3 --kernel-trace CSV of bench.py.

usage: tools/trace_summary.py <run_kernel_trace.csv> --config c2 [--instances 1024] [--last K]
       [--before join_kernel] [--json out.json]

Roles are told apart by kernel name plus grid size: sha_rows_kernel<false>
is the commit-side leaf hashing when its grid covers every row (I*N threads)
and interpolate's regen hashing when it covers the N-k regenerated slots per
instance; rs_fft_kernel<.., 0> is encode and <.., 1> the decode re-encode.
Only the last `K` launches of each role are averaged (the bench's K timed
steps; warmup launches come first, and launches on other batch sizes -- the
PCIe host-path measurement -- have other grids, hence other roles), so the
averages cover the same launches whose HIP-event spans bench.py reports as
stage_ms / roofline.avg_ms.  `--before KERNEL` drops every launch from the first
launch of KERNEL on: the default bench line's joined-value leg (join_kernel)
runs after the timed region and the guard, so its launches would otherwise be
the last ones.
"""
import argparse
import csv
import json
from collections import defaultdict

CONFIGS = {"c1": (64, 21), "c2": (128, 42), "c3": (128, 42), "c4": (256, 85)}
VALUE_BYTES = {"c1": 1 << 20, "c2": 1 << 20, "c3": 4 << 20, "c4": 64 << 10}


def read_lines(path, tries=5):
    """A CSV file's lines, read with os.read (retried: reads of freshly merged
    gpurun_out files have failed here with EBADF)."""
    import os
    import time
    for t in range(tries):
        try:
            fd = os.open(path, os.O_RDONLY)
            try:
                chunks = []
                while True:
                    b = os.read(fd, 1 << 20)
                    if not b:
                        break
                    chunks.append(b)
            finally:
                os.close(fd)
            return b"".join(chunks).decode().splitlines()
        except OSError:
            if t == tries - 1:
                raise
            time.sleep(0.2)


def shared_path(config, value_bytes=0):
    """The receive step's ECHO-verify form at a config: the C library's rule
    (csrc/capi.cpp shared_path_verify, rbc_ctx_verify_form): leaves + the
    shared-path verify where 16 d >= ceil((S + 9) / 64) and W <= 256."""
    n, f = CONFIGS[config]
    k = n - 2 * f
    S = ((value_bytes or VALUE_BYTES[config]) + k - 1) // k
    d = max(1, (n - 1).bit_length())
    return 16 * d >= (S + 9 + 63) // 64 and (1 << d) <= 256


def base(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()


def role(name, grid, n, k, inst, path=False):
    b = base(name)
    if b.startswith("rs_fft_kernel<"):
        return "rs_fft_kernel<encode>" if b.rstrip(">").endswith(", 0") else "rs_fft_kernel<decode>"
    if b == "sha_rows_kernel<false>":
        if grid == inst * n:
            return "sha_rows_kernel<leaves>"
        if grid == inst * (n - k):
            return "sha_rows_kernel<regen>"
        return f"sha_rows_kernel<false>[grid {grid}]"
    if b == "sha_rx_kernel":  # rbc_dev_receive_step: ECHO verify of t (C4: leaves only) + regen hashing of t-1
        return "sha_rx_kernel<leaves+regen>" if path else "sha_rx_kernel<verify+regen>"
    if b == "sha_rows_kernel<true>":
        return "sha_rows_kernel<verify>"
    return b


def summarize(path, config, inst, last, before=None):
    n, f = CONFIGS[config]
    k = n - 2 * f
    on_path = shared_path(config)
    durs = []
    rows = list(csv.DictReader(read_lines(path)))
    if before:
        cut = min((int(r["Start_Timestamp"]) for r in rows if base(r["Kernel_Name"]) == before), default=None)
        if cut is not None:
            rows = [r for r in rows if int(r["Start_Timestamp"]) < cut]
    for r in rows:
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # ms
        durs.append((int(r["Dispatch_Id"]), role(r["Kernel_Name"], grid, n, k, inst, on_path), grid, d))
    # one role may run on several batch sizes (the PCIe host-path measurement
    # uses small batches): the largest grid is the bench batch, others are
    # reported apart as role[grid G]
    biggest = defaultdict(int)
    for _, rl, grid, _ in durs:
        biggest[rl] = max(biggest[rl], grid)
    by_role = defaultdict(list)
    for _, rl, grid, d in sorted(durs):
        by_role[rl if grid == biggest[rl] else f"{rl}[grid {grid}]"].append(d)
    out = {}
    for rl, ds in by_role.items():
        kept = ds[-last:] if last else ds
        out[rl] = {"launches": len(ds), "timed_launches": len(kept), "avg_ms": round(sum(kept) / len(kept), 4),
                   "min_ms": round(min(kept), 4), "max_ms": round(max(kept), 4)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--instances", type=int, default=1024)
    ap.add_argument("--last", type=int, default=0, help="average only the last K launches per role (timed steps)")
    ap.add_argument("--before", help="ignore launches from the first launch of this kernel on")
    ap.add_argument("--json")
    a = ap.parse_args()
    res = summarize(a.trace, a.config, a.instances, a.last, a.before)
    for rl, v in sorted(res.items(), key=lambda x: -x[1]["avg_ms"] * x[1]["timed_launches"]):
        print(f"{rl:46s} {v['timed_launches']:4d} x {v['avg_ms']:8.4f} ms  (min {v['min_ms']:.4f}, max {v['max_ms']:.4f})")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"source": a.trace, "config": a.config, "instances": a.instances, "last": a.last,
                       "roles": res}, fh, indent=1)


if __name__ == "__main__":
    main()
