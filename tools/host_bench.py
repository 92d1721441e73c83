#!/usr/bin/env python3
"""Host-path (PCIe-inclusive) throughput of the C ABI's batch entry points.

The bench.py metric keeps inputs resident in HBM.  This measures what the Go
batcher would see: values in host memory -> rbc_shard_commit (pinned staging,
H2D, encode + leaves + tree, D2H of shards/roots/branches) and the ECHO side
rbc_interpolate_batch (shards H2D, decode + recheck, values D2H), with
`--inflight` submissions pipelined through the context's slots.

usage: python tools/host_bench.py [--config c2] [--batch 64] [--batches 8] [--inflight 2]
Prints one JSON line; GB/s counts committed shard bytes (N*S per instance).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG = {"c1": (64, 21, 1 << 20), "c2": (128, 42, 1 << 20), "c3": (128, 42, 4 << 20), "c4": (256, 85, 64 << 10)}


def measure(ca, n, f, B, batch=64, batches=8, inflight=2, pinned=True, device=0):
    """Host buffers in and out through rbc_shard_commit / rbc_interpolate_batch;
    returns GB/s of committed shard bytes (N*S per instance) for each side."""
    ctx = ca.Context(n, f, device=device)
    k = ctx.k
    S = (B + k - 1) // k
    rng = np.random.default_rng(1)
    pool = [[rng.integers(0, 256, B, dtype=np.uint8) for _ in range(batch)] for _ in range(2)]
    outsets = [None] * (inflight + 1)
    if pinned:
        for p_ in pool:
            for i, v in enumerate(p_):
                pv = ca.pinned_empty(B)
                pv[:] = v
                p_[i] = pv
        outsets = [{"shards": ca.pinned_empty((batch, n, S)), "roots": ca.pinned_empty((batch, 32)),
                    "branches": ca.pinned_empty((batch, n, max(ctx.depth, 1), 32))}
                   for _ in range(inflight + 1)]

    # shard + commit (proposer side)
    warm = [ctx.shard_commit_submit(pool[i % 2], out=outsets[i]) for i in range(inflight)]
    for w in warm:  # warm every slot's buffers
        w.wait()
    t0 = time.perf_counter()
    live, outs = [], []
    for b in range(batches):
        live.append(ctx.shard_commit_submit(pool[b % 2], out=outsets[b % len(outsets)]))
        if len(live) >= inflight:
            outs.append(live.pop(0).wait())
    while live:
        outs.append(live.pop(0).wait())
    t_enc = time.perf_counter() - t0

    # interpolate (receiver side) from N-f present shards of the last commit
    sh = outs[-1]["shards"]
    present = np.zeros((batch, n), np.uint8)
    for i in range(batch):
        present[i, rng.permutation(n)[: n - f]] = 1
    rx = sh * present[:, :, None]
    vout = None
    if pinned:
        prx = ca.pinned_empty(rx.shape)
        prx[:] = rx
        rx = prx
        vout = ca.pinned_empty((batch, ctx.k * S))
    lens = outs[-1]["shard_lens"]
    roots = outs[-1]["roots"].copy()
    vouts = [vout] + [ca.pinned_empty(vout.shape) if pinned else None for _ in range(inflight)]
    warm = [ctx.interpolate_submit(rx, lens, present, roots, values_out=vouts[i]) for i in range(inflight)]
    for w in warm:  # warm every slot's buffers
        w.wait()
    t0 = time.perf_counter()
    live, res = [], None
    for b in range(batches):
        live.append(ctx.interpolate_submit(rx, lens, present, roots, values_out=vouts[b % len(vouts)]))
        if len(live) >= inflight:
            res = live.pop(0).wait()
    while live:
        res = live.pop(0).wait()
    t_dec = time.perf_counter() - t0
    assert (res["status"] == 0).all()
    # proposer send path: shard + commit + per-recipient VAL marshal, one D2H of
    # the finished pb.Message bytes into a pinned ring (rbc_shard_commit_val)
    vrings = [None] * (inflight + 1)
    if pinned:
        need = max(ctx.val_message_size(S, 0, 0), ctx.val_message_size(S, n - 1, 0))
        vrings = [ca.pinned_empty((batch, n, (need + 15) // 16 * 16)) for _ in range(inflight + 1)]
    warm = [ctx.shard_commit_val_submit(pool[i % 2], ring=vrings[i]) for i in range(inflight)]
    for w in warm:
        w.wait()
    t0 = time.perf_counter()
    live = []
    for b in range(batches):
        live.append(ctx.shard_commit_val_submit(pool[b % 2], ring=vrings[b % len(vrings)]))
        if len(live) >= inflight:
            vo = live.pop(0).wait()
    while live:
        vo = live.pop(0).wait()
    t_val = time.perf_counter() - t0
    msg_bytes = int(vo["lens"].sum()) * batches
    ctx.close()
    shard_bytes = batch * n * S * batches
    return {"shard_commit_val_msg_GBps": round(msg_bytes / t_val / 1e9, 2),
            "shard_commit_val_ms_per_batch": round(t_val * 1e3 / batches, 3),
            "shard_commit_GBps": round(shard_bytes / t_enc / 1e9, 2),
            "interpolate_GBps": round(shard_bytes / t_dec / 1e9, 2),
            "shard_commit_ms_per_batch": round(t_enc * 1e3 / batches, 3),
            "interpolate_ms_per_batch": round(t_dec * 1e3 / batches, 3),
            "batch": batch, "batches": batches, "inflight": inflight, "pinned": pinned}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CFG))
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=2)
    ap.add_argument("--pinned", action="store_true",
                    help="values, shard/root/branch outputs and interpolate buffers in rbc_host_alloc memory "
                         "(the C ABI then copies to and from them directly, no staging memcpy)")
    args = ap.parse_args()
    import cleisthenes_amd as ca

    n, f, B = CFG[args.config]
    r = measure(ca, n, f, B, args.batch, args.batches, args.inflight, args.pinned)
    print(json.dumps({
        "metric": "host-path RBC shard GB/s (PCIe-inclusive, host buffers in and out)",
        "config": {"workload": args.config, "n": n, "f": f, "value_bytes": B, "batch": args.batch,
                   "batches": args.batches, "inflight": args.inflight, "pinned": args.pinned},
        **{k_: v for k_, v in r.items() if k_.endswith("GBps") or k_.endswith("batch")},
    }))


if __name__ == "__main__":
    main()
