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


def _rx_messages(present, n, pitch):
    """The received ECHOs of a sub-batch as rbc_validate_packed_leaves names
    them inside the receiver's [count][n][pitch] buffer."""
    inst, pos = np.nonzero(present)
    return inst, pos, ((inst * n + pos) * pitch).astype(np.uint64)


def epoch(ca, n, f, B, instances=1024, sub=128, ring=3, inflight=2, device=0, seed=20261018, tamper=0.10,
          phases=True, barrier=None, contexts=1):
    """One node's whole RBC epoch through the C ABI from pinned host memory
    (end-to-end with H2D / D2H).  Per
    sub-batch of `sub` instances, concurrently (`inflight` of each kind in
    flight through the context's host slots):
      proposer  rbc_shard_commit: values in, shards + roots + branches out;
      receiver  rbc_validate_packed_leaves of every received ECHO (N-f per
                instance, `tamper` of the instances carry one corrupted ECHO)
                straight out of the node's [sub][N][pitch] receive buffer
                (only the received rows cross PCIe), then
                rbc_interpolate_batch_verified of the ECHOs that validated,
                reusing their leaves (only the ~2f regenerated rows are
                hashed), values out.
    The receive side's inputs are a ring of `ring` committed sub-batches
    prepared before timing (the ECHOs other proposers would have sent).
    Every verdict, every decoded value and every proposer root is checked
    after timing.  `barrier` (callable) brackets the timed region when ranks
    run the leg together.  GB/s = instances x N x S committed shard bytes
    per second (the bench's unit); PCIe bytes are counted per direction.
    contexts=2: the proposer and the receiver side submit through contexts of
    their own (own host slots, streams and lock), as a node may.
    A third timed run (ABI 7, "kept") makes the same drop-in calls with the
    validated rows left on the device: rbc_validate_packed_keep into a device
    buffer per slot, then rbc_interpolate_batch_kept from it -- the ECHO rows
    cross PCIe once, as with the fused receive."""
    import time as _t
    ctx = ca.Context(n, f, device=device)
    pctx = ca.Context(n, f, device=device) if contexts == 2 else ctx  # the proposer side's
    k, d = ctx.k, ctx.depth
    S = (B + k - 1) // k
    pitch = (S + 63) // 64 * 64
    rng = np.random.default_rng(seed)
    nsub = (instances + sub - 1) // sub
    counts = [min(sub, instances - b * sub) for b in range(nsub)]
    # ---- inputs (untimed): `ring` distinct value sets, committed once for the receive side
    vals = []
    for r in range(ring):
        v = ca.pinned_empty((sub, B))
        v[:] = rng.integers(0, 256, (sub, B), dtype=np.uint8)
        vals.append(v)
    # the proposer's output rings at a 64-B row pitch: the shards come back in one D2H copy
    prop = [{"shards": ca.pinned_empty((sub, n, pitch)), "roots": ca.pinned_empty((sub, 32)),
             "branches": ca.pinned_empty((sub, n, max(d, 1), 32))} for _ in range(inflight + 1)]
    rx = []
    for r in range(ring):
        com = ctx.shard_commit_submit(list(vals[r]), out=prop[0]).wait()
        present = np.zeros((sub, n), np.uint8)
        bad = np.full(sub, -1)
        for i in range(sub):
            rec = rng.permutation(n)[: n - f]
            present[i, rec] = 1
            if rng.random() < tamper:
                bad[i] = int(rng.choice(rec))
        buf = ca.pinned_empty((sub, n, pitch))
        buf[:, :, :S] = com["shards"]
        buf[:, :, S:] = 0
        for i in np.flatnonzero(bad >= 0):
            buf[i, bad[i], S // 2] ^= 0x5A
        inst, pos, offs = _rx_messages(present, n, pitch)
        m = len(inst)
        br = ca.pinned_empty((m, max(d, 1) * 32))
        br[:] = com["branches"][inst, pos].reshape(m, -1)
        mroots = ca.pinned_empty((m, 32))
        mroots[:] = com["roots"][inst]
        meta = {"lens": np.full(m, S, np.uint32), "idx": pos.astype(np.uint8), "offs": offs}
        brall = ca.pinned_empty((sub, n, max(d, 1), 32))
        brall[:] = com["branches"].reshape(sub, n, max(d, 1), 32)
        want_valid = present.copy()
        want_valid[np.flatnonzero(bad >= 0), bad[bad >= 0]] = 0
        rx.append(dict(buf=buf, present=present, bad=bad, inst=inst, pos=pos, br=br, mroots=mroots, brall=brall,
                       roots=com["roots"].copy(), want=bad[inst] != pos, want_valid=want_valid, **meta))
    vout = ca.pinned_empty((instances, k * S))
    digests = np.zeros((instances, 32), np.uint8)
    status = np.full(instances, 99, np.int32)
    mmax = sub * (n - f)
    vres = [{"ok": ca.pinned_empty((mmax,)), "leaves": ca.pinned_empty((mmax, 32))} for _ in range(inflight + 1)]
    lvs = [ca.pinned_empty((sub, n, 32)) for _ in range(inflight + 1)]
    vmask = [np.zeros((sub, n), np.uint8) for _ in range(inflight + 1)]
    roots_out = np.zeros((instances, 32), np.uint8)
    verdict_bad = [0]
    keeps = [ca.DeviceBuffer(rx[0]["buf"].nbytes, device) for _ in range(inflight + 1)]

    def commit(b, slot):
        c = counts[b]
        o = {kk: v[:c] for kk, v in prop[slot].items()}
        return pctx.shard_commit_submit(list(vals[b % ring][:c]), out=o)

    def validate(b, slot, keep=False):
        """keep: the rows stay in keeps[slot] (free again: the interpolate that read them, of sub-batch
        b - inflight - 1, was waited before this submission)"""
        R = rx[b % ring]
        m = int(np.searchsorted(R["inst"], counts[b]))
        return ctx.validate_packed_submit(R["buf"], R["offs"][:m], R["lens"][:m], R["idx"][:m], R["br"][:m],
                                          R["mroots"][:m], leaves=True,
                                          out={"ok": vres[slot]["ok"], "leaves": vres[slot]["leaves"]},
                                          keep=keeps[slot] if keep else None)

    def interpolate(b, slot, ok, leaves, kept=False):
        R, c = rx[b % ring], counts[b]
        m = len(ok)
        if not np.array_equal(ok, R["want"][:m]):
            verdict_bad[0] += int((ok != R["want"][:m]).sum())
        valid = np.zeros((c, n), np.uint8)
        iv, pv = R["inst"][:m][ok], R["pos"][:m][ok]
        valid[iv, pv] = 1
        lv = lvs[slot][:c]
        lv[iv, pv] = leaves[ok]
        lo = b * sub
        if kept:  # the valid rows where the validate left them on the device
            rows = np.zeros((c, n), np.uint64)
            rows[iv, pv] = keeps[slot].value + R["offs"][:m][ok]
            return ctx.interpolate_kept_submit(rows, [S] * c, R["roots"][:c], leaves=lv, values_out=vout[lo:lo + c],
                                               digests_out=digests[lo:lo + c], status_out=status[lo:lo + c])
        return ctx.interpolate_submit(R["buf"][:c], [S] * c, valid, R["roots"][:c], values_out=vout[lo:lo + c],
                                      leaves=lv, digests_out=digests[lo:lo + c], status_out=status[lo:lo + c])

    def receive(b, slot):
        """rbc_receive_batch: verify + interpolate in one submission, the ECHO rows crossing PCIe once."""
        R, c = rx[b % ring], counts[b]
        lo = b * sub
        return ctx.receive_submit(R["buf"][:c], [S] * c, R["present"][:c], R["brall"][:c], R["roots"][:c],
                                  values_out=vout[lo:lo + c], valid_out=vmask[slot][:c],
                                  digests_out=digests[lo:lo + c], status_out=status[lo:lo + c])

    def run(kinds):
        """One epoch, the given sides concurrently; returns wall seconds."""
        live = {"c": [], "v": [], "i": [], "r": []}
        t0 = _t.perf_counter()
        for b in range(nsub + 1):
            if b < nsub:
                if "c" in kinds:
                    live["c"].append((b, commit(b, b % (inflight + 1))))
                if "v" in kinds:
                    live["v"].append((b, validate(b, b % (inflight + 1), keep="k" in kinds)))
                if "r" in kinds:
                    live["r"].append((b, receive(b, b % (inflight + 1))))
            # the receive side: interpolate a sub-batch once its validate is back
            while live["v"] and (len(live["v"]) > inflight - 1 or b == nsub):
                bv, tv = live["v"].pop(0)
                ok, leaves = tv.wait()
                if "i" in kinds or "k" in kinds:
                    live["i"].append((bv, interpolate(bv, bv % (inflight + 1), ok, leaves, kept="k" in kinds)))
                if b < nsub:
                    break
            for kd in ("c", "i", "r"):
                while live[kd] and (len(live[kd]) >= inflight or b == nsub):
                    bb, tt = live[kd].pop(0)
                    res = tt.wait()
                    if kd == "c":
                        roots_out[bb * sub: bb * sub + counts[bb]] = res["roots"]
                    elif kd == "r":  # the fused receive's verdicts
                        R, c = rx[bb % ring], counts[bb]
                        verdict_bad[0] += int((res["valid"] != R["want_valid"][:c]).sum())
        return _t.perf_counter() - t0

    marks = []

    def timed(kinds):
        """warm every slot's buffers, then time one epoch of `kinds` (all ranks together) and check it:
        verdicts, every value, statuses, proposer roots"""
        run(kinds)
        status[:] = 99
        vout[:] = 0
        roots_out[:] = 0
        verdict_bad[0] = 0
        if barrier:
            barrier()
        marks.append([kinds, _t.monotonic_ns()])
        el = run(kinds)
        marks[-1].append(_t.monotonic_ns())  # CLOCK_MONOTONIC, the clock of rocprofv3's timestamps
        if barrier:
            barrier()
        vals_ok = all(np.array_equal(vout[b * sub: b * sub + counts[b], :B], vals[b % ring][:counts[b]])
                      for b in range(nsub))
        roots_ok = all(np.array_equal(roots_out[b * sub: b * sub + counts[b]], rx[b % ring]["roots"][:counts[b]])
                       for b in range(nsub))
        chk = {"verdict_mismatches": verdict_bad[0], "values_ok": bool(vals_ok), "decoded": int((status == 0).sum()),
               "roots_ok": bool(roots_ok)}
        return el, chk, bool(vals_ok and roots_ok and verdict_bad[0] == 0 and (status == 0).all())

    el, checks, ok = timed("cvi")  # the drop-in's calls: shard_commit || validate -> interpolate
    el_f, checks_f, ok_f = timed("cr")  # shard_commit || the fused receive
    el_k, checks_k, ok_k = timed("cvk")  # the drop-in's calls, the validated rows kept on the device
    shard_bytes = instances * n * S
    echo = sum(int((rx[b % ring]["inst"] < counts[b]).sum()) for b in range(nsub))
    h2d = instances * B + 2 * echo * S  # values, ECHO rows for validate, the valid ECHO rows for interpolate
    d2h = shard_bytes + instances * n * d * 32 + instances * k * S
    h2d_f = instances * B + echo * S  # the fused receive moves the ECHO rows once
    out = {"GBps": round(shard_bytes / el / 1e9, 3), "seconds": round(el, 6), "instances": instances,
           "sub_batch": sub, "inflight": inflight, "echo_messages": echo,
           "pcie_GBps": {"h2d": round(h2d / el / 1e9, 2), "d2h": round(d2h / el / 1e9, 2)},
           "checks": checks, "ok": ok and ok_f and ok_k,
           "timed_windows_ns": marks,
           "fused": {"GBps": round(shard_bytes / el_f / 1e9, 3), "seconds": round(el_f, 6), "checks": checks_f,
                     "ok": ok_f, "pcie_GBps": {"h2d": round(h2d_f / el_f / 1e9, 2), "d2h": round(d2h / el_f / 1e9, 2)},
                     "path": "rbc_shard_commit || rbc_receive_batch (ECHO rows cross PCIe once, verified on the "
                             "device, interpolate reusing the leaves)"},
           "kept": {"GBps": round(shard_bytes / el_k / 1e9, 3), "seconds": round(el_k, 6), "checks": checks_k,
                    "ok": ok_k, "pcie_GBps": {"h2d": round(h2d_f / el_k / 1e9, 2), "d2h": round(d2h / el_k / 1e9, 2)},
                    "path": "rbc_shard_commit || rbc_validate_packed_keep -> rbc_interpolate_batch_kept (the drop-in's "
                            "calls; the validated ECHO rows stay on the device, crossing PCIe once)"}}
    if phases:  # each side alone over the same epoch: which one binds
        alone = {}
        for name, kinds in (("shard_commit", "c"), ("validate", "v"), ("validate+interpolate", "vi"),
                            ("receive_fused", "r"), ("validate+interpolate_kept", "vk")):
            alone[name] = round(shard_bytes / run(kinds) / 1e9, 3)
        out["alone_GBps"] = alone
    out["contexts"] = contexts
    if pctx is not ctx:
        pctx.close()
    ctx.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CFG))
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=2)
    ap.add_argument("--epoch", type=int, default=0,
                    help="instead: one host-fed epoch of this many instances (the bench's pcie_inclusive leg)")
    ap.add_argument("--sub", type=int, default=0, help="epoch sub-batch (default: ~400 MB of shards)")
    ap.add_argument("--contexts", type=int, default=1, choices=(1, 2),
                    help="epoch: 2 = the proposer and the receiver side on contexts of their own")
    ap.add_argument("--pinned", action="store_true",
                    help="values, shard/root/branch outputs and interpolate buffers in rbc_host_alloc memory "
                         "(the C ABI then copies to and from them directly, no staging memcpy)")
    args = ap.parse_args()
    import cleisthenes_amd as ca

    n, f, B = CFG[args.config]
    if args.epoch:
        k = n - 2 * f
        S = (B + k - 1) // k
        sub = args.sub or max(1, min(args.epoch, int(400e6 // (n * S))))
        r = epoch(ca, n, f, B, instances=args.epoch, sub=sub, inflight=args.inflight, contexts=args.contexts)
        print(json.dumps({"config": args.config, "library": ca.rbc.library_path(), **r}))
        return
    r = measure(ca, n, f, B, args.batch, args.batches, args.inflight, args.pinned)
    print(json.dumps({
        "metric": "host-path RBC shard GB/s (PCIe-inclusive, host buffers in and out)",
        "config": {"workload": args.config, "n": n, "f": f, "value_bytes": B, "batch": args.batch,
                   "batches": args.batches, "inflight": args.inflight, "pinned": args.pinned},
        **{k_: v for k_, v in r.items() if k_.endswith("GBps") or k_.endswith("batch")},
    }))


if __name__ == "__main__":
    main()
