#!/usr/bin/env python3
"""PMC evidence that rbc_interpolate_batch_verified hashes only the rows it
regenerates.

run:      python tools/pmc_interp_probe.py run [instances]
          (under rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES ...): one C2 batch
          committed on the GPU, its N-f received ECHOs (10 % of the instances
          with one corrupted ECHO) validated with rbc_validate_packed_leaves,
          then the same interpolate twice each way, alternating: the plain
          rbc_interpolate_batch (all N rows rehashed) and
          rbc_interpolate_batch_verified (the validate leaves reused).
summarise: python tools/pmc_interp_probe.py summary <counter_collection.csv> [instances]
          -> JSON: the last four sha_rows_kernel<false> dispatches are the
          interpolates (full, verified, full, verified); their VALU
          instructions per launch, the ratio, and the rows each form should
          hash (N per instance vs the regenerated ones) for comparison."""
import csv
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
N, F, B = 128, 42, 1 << 20


def run(instances):
    import cleisthenes_amd as ca
    from host_bench import _rx_messages
    ctx = ca.Context(N, F)
    k, d = ctx.k, ctx.depth
    S = (B + k - 1) // k
    pitch = (S + 63) // 64 * 64
    rng = np.random.default_rng(4)
    vals = ca.pinned_empty((instances, B))
    vals[:] = rng.integers(0, 256, (instances, B), dtype=np.uint8)
    com = ctx.shard_commit_submit(list(vals)).wait()
    present = np.zeros((instances, N), np.uint8)
    bad = np.full(instances, -1)
    for i in range(instances):
        rec = rng.permutation(N)[: N - F]
        present[i, rec] = 1
        if rng.random() < 0.10:
            bad[i] = int(rng.choice(rec))
    buf = ca.pinned_empty((instances, N, pitch))
    buf[:, :, :S] = com["shards"]
    buf[:, :, S:] = 0
    for i in np.flatnonzero(bad >= 0):
        buf[i, bad[i], 7] ^= 1
    inst, pos, offs = _rx_messages(present, N, pitch)
    ok, lv = ctx.validate_packed(buf, offs, np.full(len(inst), S, np.uint32), pos.astype(np.uint8),
                                 com["branches"][inst, pos].reshape(len(inst), -1), com["roots"][inst], leaves=True)
    valid = np.zeros((instances, N), np.uint8)
    valid[inst[ok], pos[ok]] = 1
    leaves = ca.pinned_empty((instances, N, 32))
    leaves[inst[ok], pos[ok]] = lv[ok]
    res = []
    for _ in range(2):
        res.append(ctx.interpolate_batch(buf, [S] * instances, valid, com["roots"]))
        res.append(ctx.interpolate_batch(buf, [S] * instances, valid, com["roots"], leaves=leaves))
    same = all(np.array_equal(r["values"], res[0]["values"]) and np.array_equal(r["digests"], res[0]["digests"])
               for r in res)
    # rows each form hashes: full = N per instance; verified = the absent positions + the rejected ECHO
    regen = int((valid == 0).sum())
    print(json.dumps({"instances": instances, "decoded": int((res[0]["status"] == 0).sum()), "same": bool(same),
                      "rows_full": instances * N, "rows_verified_expected": regen,
                      "valid_rows": int(valid.sum())}), flush=True)
    return 0 if same and (res[0]["status"] == 0).all() else 1


def summary(path, instances):
    rows = list(csv.DictReader(open(path)))
    by = {}
    for r in rows:
        if "sha_rows_kernel<false>" not in r["Kernel_Name"]:
            continue
        key = (int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
        by.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    disp = [by[k] for k in sorted(by)][-4:]
    valu = [x.get("SQ_INSTS_VALU") for x in disp]
    full = (valu[0] + valu[2]) / 2
    ver = (valu[1] + valu[3]) / 2
    return {"kernel": "sha_rows_kernel<false> (interpolate's row hashing)", "instances": instances,
            "valu_per_launch": {"full_rehash": full, "verified_leaves": ver}, "ratio": round(ver / full, 4),
            "dispatch_valu": valu, "source": os.path.relpath(path, ROOT) if path.startswith(ROOT) else path}


if __name__ == "__main__":
    if sys.argv[1] == "run":
        sys.exit(run(int(sys.argv[2]) if len(sys.argv) > 2 else 256))
    print(json.dumps(summary(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 256)))
