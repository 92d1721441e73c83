#!/usr/bin/env python3
"""Per-call latency of the synchronous single-call drop-ins (ticket NULL):
rbc_validate_message, rbc_interpolate and rbc_shard at C2 (N=128, f=42,
1 MiB), median / p10 / p90 over `reps` calls after a warm-up -- the
advisor's check that the blocking-sync slot events, which make
a waiter sleep instead of spin, do not slow the synchronous host API."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cleisthenes_amd as ca  # noqa: E402


def stats(fn, reps):
    for _ in range(5):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - t0) * 1e6)
    t = np.array(t)
    return {"median_us": round(float(np.median(t)), 1), "p10_us": round(float(np.percentile(t, 10)), 1),
            "p90_us": round(float(np.percentile(t, 90)), 1)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    n, f = 128, 42
    ctx = ca.Context(n, f)
    rng = np.random.default_rng(3)
    out = {"library": ca.rbc.library_path()}
    for B in (4096, 1 << 20):
        v = rng.integers(0, 256, B, dtype=np.uint8).tobytes()
        com = ctx.shard(v)
        j = 5
        shards = [s if i < n - f else None for i, s in enumerate(com["shards"])]
        out[f"B{B}"] = {
            "validate_message": stats(lambda: ctx.validate_message(com["root"], com["branches"][j], com["shards"][j], j),
                                      reps),
            "interpolate": stats(lambda: ctx.interpolate(com["root"], shards), max(20, reps // 4)),
            "shard": stats(lambda: ctx.shard(v), max(20, reps // 4))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
