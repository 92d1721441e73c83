#!/usr/bin/env python3
"""RBC data-path benchmark (BASELINE.json metric: "RBC shard GB/s (RS
encode+decode + Merkle verify) per GPU & node, N=128").

One step = one full RBC round of the data path over a batch of I instances
resident in HBM (default C2: N=128, f=42, 1 MiB values, I=1024 per GPU):
  1. shard+commit   rbc_dev_encode (Split+Encode), rbc_dev_leaves (SHA-256 of
                    every shard), rbc_dev_merkle_build (root + N branches)
  2. Byzantine input: 10 % of instances get one corrupted ECHO shard
  3. ECHO verify    rbc_dev_verify: validateMessage for all N shards of every
                    instance (hash shard + walk branch + compare root)
  4. interpolate    rbc_dev_interpolate: first k valid of a seeded N-f
                    present set -> regenerate the other N-k positions,
                    re-hash them, recheck the root, emit value + digest
  5. (N GPUs > 1)   RCCL all-gather of {root, digest} over xGMI (ACS set)
value = I * N * S bytes of committed shard output per step, summed over all
ranks, / (max over ranks of the timed wall time).

Default schedule: the stages in order on one HIP stream, so the per-kernel
event spans behind `roofline` match a rocprofv3 trace of the same command.
--pipeline 1 commits batch t on one stream while batch t-1 is verified and
interpolated on a second (K full commits + K full decodes still inside the
timed region); it measured +2.8 % (421 vs 409 GB/s, 3 runs each).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU).  Host-side coordination uses
torch.distributed with the gloo backend (CPU tensors); all GPU work, including
the RCCL all-gather, goes through librbc_gpu.so.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (N, f, value bytes, instances per GPU, description)
    "c1": (64, 21, 1 << 20, 1024, "N=64 f=21 1MiB x1024"),
    "c2": (128, 42, 1 << 20, 1024, "N=128 f=42 1MiB x1024"),
    "c3": (128, 42, 4 << 20, 1024, "N=128 f=42 4MiB x1024 per GPU (8192 over 8 GPUs)"),
    "c4": (256, 85, 64 << 10, 16384, "N=256 f=85 64KiB x16384"),
}
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
# SHA-256 VALU roof.  Issue cost per wave64 instruction on one SIMD, measured
# (profiles/r01_valu_probe.txt): v_alignbit / v_add3 / v_perm / v_bfi 4 clk,
# v_bitop3 / v_add / v_xor / v_and / shifts 2 clk (with >= 4 waves per SIMD).
# The compression loop of sha_rows_kernel (ISA) issues
# 833 four-clock + 576 two-clock instructions = 4484 SIMD clocks per
# wave-compression (64 rows): peak = 1024 SIMDs x 2.4 GHz / 4484 x 64.
SHA_CLK_PER_WAVE_COMPRESSION = 833 * 4 + 576 * 2
SHA_PEAK_CPS = 1024 * 2.4e9 / SHA_CLK_PER_WAVE_COMPRESSION * 64
# attainable: the same compression register-resident at 8 waves/SIMD
# (profiles/r01_sha_probe.txt, 5782 clk at the nominal 2.4 GHz)
SHA_PROBE_CPS = 1024 * 2.4e9 / 5782 * 64


def round_up(x, a):
    return (x + a - 1) // a * a


def main():
    # ONE JSON line on stdout: keep a private handle on the real stdout and
    # point fd 1 at stderr, so banners that native libraries print with
    # printf (RCCL's version block, gloo's peer count) cannot precede it
    out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--instances", type=int, default=0, help="override instances per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-instances", type=int, default=2048)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--streams", type=int, default=1,
                    help="split the batch over S HIP streams (one context each) so stages of different "
                         "instance groups overlap")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1: overlap batch t's commit (proposer stream) with batch t-1's verify + "
                         "interpolate (receiver stream), two shard buffer sets; 0 (default): one stream, "
                         "stages in order, so each kernel's event span is its own")
    ap.add_argument("--shard-align", type=int, default=128,
                    help="shard row pitch alignment in bytes (multiple of 64; the C ABI needs 64)")
    ap.add_argument("--force-gather", action="store_true",
                    help="run the RCCL all-gather even with one rank (exercises rbc_comm_*)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or "RANK" in os.environ:  # launched by torch.distributed.run
        import torch.distributed as dist  # host-side coordination only (gloo, CPU tensors)
        dist.init_process_group("gloo")

    import cleisthenes_amd as ca

    n, f, B, inst, desc = CONFIGS[args.config]
    if args.instances:
        inst = args.instances
    dev = local_rank
    ctx = ca.Context(n, f, device=dev)
    k, d = ctx.k, ctx.depth
    S = (B + k - 1) // k
    spitch = round_up(S, args.shard_align)  # row starts on whole 128-B lines: full-line HBM writes
    vpitch = round_up(k * S + 32, 64)
    opitch = round_up(k * S, 16)
    I = inst

    # ---- synthetic inputs (seeded per rank), uploaded once ----------------
    rng = np.random.default_rng(20261015 + rank)
    values_h = rng.integers(0, 256, size=(I, vpitch), dtype=np.uint8)
    present_h = np.zeros((I, n), dtype=np.uint8)
    corrupt_h = np.full(I, -1, dtype=np.int32)
    for i in range(I):
        pres = rng.permutation(n)[: n - f]
        present_h[i, pres] = 1
        if rng.random() < 0.10:
            corrupt_h[i] = int(rng.choice(pres))

    mb = lambda x: ca.DeviceBuffer(x, device=dev)  # noqa: E731
    d_values = mb(I * vpitch)
    d_values.upload(values_h)
    del values_h
    pipe = bool(args.pipeline) and args.streams == 1  # --streams > 1 is its own (serial) schedule
    nsets = 2 if pipe else 1
    sets = [dict(shards=mb(I * n * spitch), leaves=mb(I * n * 32), roots=mb(I * 32),
                 branches=mb(I * n * max(d, 1) * 32)) for _ in range(nsets)]
    d_shards, d_leaves_p, d_roots, d_branches = (sets[0][x] for x in ("shards", "leaves", "roots", "branches"))
    d_present = mb(I * n)
    d_present.upload(present_h)
    d_corrupt = mb(I * 4)
    d_corrupt.upload(corrupt_h)
    d_valid = mb(I * n)
    d_leaves_r = mb(I * n * 32)
    d_out = mb(I * opitch)
    d_digests = mb(I * 32)
    d_status = mb(I * 4)
    gather = world > 1 or args.force_gather
    d_gather = mb(world * I * 64) if gather else None

    if dist is None and gather:
        ctx.comm_init(1, 0, ca.Context.comm_unique_id())
    if dist is not None and gather:
        import torch
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid = torch.frombuffer(bytearray(ca.Context.comm_unique_id()), dtype=torch.uint8).clone()
        dist.broadcast(uid, 0)
        ctx.comm_init(world, rank, bytes(uid.numpy().tobytes()))

    nstreams = max(1, min(args.streams, I))
    streams = [ca.Stream(dev) for _ in range(nstreams)]
    ctxs = [ctx] + [ca.Context(n, f, device=dev) for _ in range(nstreams - 1)]  # own decode workspace each
    bounds = [(g * I // nstreams, (g + 1) * I // nstreams) for g in range(nstreams)]
    stream = streams[0]
    stage_names = ("t0", "enc", "leaf", "tree", "fault", "verify", "interp", "gather")
    # one event set per timed step: stage times are read after the closing
    # barrier, so the timed loop never waits on the host between steps
    ev_sets = [{name: ca.Event() for name in stage_names} for _ in range(max(args.steps, 3))]

    def at(buf, i0, per):
        return buf.value + i0 * per

    def step(ev):
        timed = ev is not None
        for g, (i0, i1) in enumerate(bounds):
            st, cx, cnt = streams[g].ptr, ctxs[g], i1 - i0
            rec = timed and g == 0  # per-stage events on stream 0 (group 0)
            if rec:
                ev["t0"].record(stream)
            cx.dev_encode(st, cnt, at(d_values, i0, vpitch), vpitch, None, B, at(d_shards, i0, n * spitch), spitch)
            if rec:
                ev["enc"].record(stream)
            cx.dev_leaves(st, cnt, at(d_shards, i0, n * spitch), spitch, None, S, at(d_leaves_p, i0, n * 32))
            if rec:
                ev["leaf"].record(stream)
            cx.dev_merkle_build(st, cnt, at(d_leaves_p, i0, n * 32), at(d_roots, i0, 32),
                                at(d_branches, i0, n * max(d, 1) * 32))
            if rec:
                ev["tree"].record(stream)
            cx.dev_inject_faults(st, cnt, at(d_shards, i0, n * spitch), spitch, at(d_corrupt, i0, 4))
            if rec:
                ev["fault"].record(stream)
            cx.dev_verify(st, cnt, at(d_shards, i0, n * spitch), spitch, None, S,
                          at(d_branches, i0, n * max(d, 1) * 32), at(d_roots, i0, 32), at(d_present, i0, n),
                          at(d_valid, i0, n), at(d_leaves_r, i0, n * 32))
            if rec:
                ev["verify"].record(stream)
            cx.dev_interpolate(st, cnt, at(d_shards, i0, n * spitch), spitch, None, S, at(d_valid, i0, n),
                               at(d_leaves_r, i0, n * 32), 1, at(d_roots, i0, 32), at(d_out, i0, opitch), opitch,
                               at(d_digests, i0, 32), at(d_status, i0, 4))
            if rec:
                ev["interp"].record(stream)
        if gather:
            for s_ in streams[1:]:
                s_.sync()
            ctx.dev_allgather_roots(stream.ptr, I, d_roots, d_digests, d_gather)
        if timed:
            ev["gather"].record(stream)

    # --pipeline: proposer stream P commits batch t into set t%2 while the
    # receiver stream R verifies + interpolates batch t-1 from the other set.
    # A set is reused only after R has finished with it (evR), and R starts a
    # batch only after P committed it (evP): K timed steps = K commits + K
    # decodes, all inside the timed region.
    rstream = ca.Stream(dev) if pipe else None
    evP = [ca.Event() for _ in range(nsets)]
    evR = [ca.Event() for _ in range(nsets)]
    for e in evP + evR:
        e.record(stream)  # recorded once, so every wait below is well defined

    def pstep(t):
        P, R = stream, rstream
        sp = sets[t % 2]
        P.wait(evR[t % 2])
        ctx.dev_encode(P.ptr, I, d_values.value, vpitch, None, B, sp["shards"].value, spitch)
        ctx.dev_leaves(P.ptr, I, sp["shards"].value, spitch, None, S, sp["leaves"].value)
        ctx.dev_merkle_build(P.ptr, I, sp["leaves"].value, sp["roots"].value, sp["branches"].value)
        ctx.dev_inject_faults(P.ptr, I, sp["shards"].value, spitch, d_corrupt.value)
        evP[t % 2].record(P)
        if t == 0:
            return
        sr = sets[(t - 1) % 2]
        R.wait(evP[(t - 1) % 2])
        ctx.dev_verify(R.ptr, I, sr["shards"].value, spitch, None, S, sr["branches"].value, sr["roots"].value,
                       d_present.value, d_valid.value, d_leaves_r.value)
        ctx.dev_interpolate(R.ptr, I, sr["shards"].value, spitch, None, S, d_valid.value, d_leaves_r.value, 1,
                            sr["roots"].value, d_out.value, opitch, d_digests.value, d_status.value)
        if gather:
            ctx.dev_allgather_roots(R.ptr, I, sr["roots"].value, d_digests.value, d_gather)
        evR[(t - 1) % 2].record(R)

    def barrier():
        if rstream is not None:
            rstream.sync()
        for s_ in streams:
            s_.sync()
        ca.rbc.lib.rbc_device_sync(dev)
        if dist is not None:
            dist.barrier()

    if pipe:
        args.warmup = max(args.warmup, 2)  # fill the pipeline: at least one decode before the guard
        for t in range(args.warmup):
            pstep(t)
        last_set = sets[(args.warmup - 2) % 2]
        d_roots = last_set["roots"]  # the set the last decode (and gather) read
    else:
        for _ in range(args.warmup):
            step(None)
    barrier()
    # correctness guard on the warmed-up state: every instance must decode
    status = np.frombuffer(d_status.download().tobytes(), dtype=np.int32)
    n_ok = int((status == 0).sum())
    if gather:
        # the gathered ACS records of this rank must equal its own {root, digest}
        from cleisthenes_amd import acs
        g = d_gather.download().reshape(world, I, 64)
        mine = acs.pack_records(d_roots.download().reshape(I, 32), d_digests.download().reshape(I, 32), I)
        assert np.array_equal(g[rank], mine), "RCCL all-gather returned wrong records"

    stage_ms = {kk: 0.0 for kk in ("enc", "leaf", "tree", "fault", "verify", "interp", "gather")}
    order = ["t0", "enc", "leaf", "tree", "fault", "verify", "interp", "gather"]
    barrier()
    t0 = time.perf_counter()
    if pipe:
        for t in range(args.warmup, args.warmup + args.steps):
            pstep(t)
    else:
        for t in range(args.steps):
            step(ev_sets[t])
    barrier()
    elapsed = time.perf_counter() - t0
    if not pipe:
        for ev in ev_sets[: args.steps]:
            for a, b in zip(order[:-1], order[1:]):
                stage_ms[b] += ev[a].elapsed_ms(ev[b])
    if pipe:
        # per-stage (and roofline) timings from an isolated serial pass: under
        # the overlap, one kernel's event span includes the other stream's work
        d_shards, d_leaves_p, d_roots, d_branches = (sets[0][x] for x in ("shards", "leaves", "roots", "branches"))
        iso = 3
        for it in range(iso):
            ev = ev_sets[it]
            step(ev)
            stream.sync()
            for a, b in zip(order[:-1], order[1:]):
                stage_ms[b] += ev[a].elapsed_ms(ev[b]) * args.steps / iso
        barrier()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        okt = torch.tensor([n_ok], dtype=torch.int64)
        dist.all_reduce(okt)
        n_ok = int(okt.item())

    for kk in stage_ms:
        stage_ms[kk] /= args.steps
    ms_per_step = elapsed * 1000.0 / args.steps
    shard_bytes = I * n * S
    value = shard_bytes * world * args.steps / elapsed / 1e9

    # ---- roofline of the dominant kernel --------------------------------
    blocks_per_shard = (S + 9 + 63) // 64
    Ig = bounds[0][1] - bounds[0][0]  # instances per launch (group 0's stream when --streams > 1)
    enc_kernel = "rs_fft_kernel<encode>" if ctx.codec == "fft" else "gf_rows_kernel<encode>"
    kern = {
        # name: (avg ms, algorithmic HBM bytes per launch, sha compressions per launch)
        enc_kernel: (stage_ms["enc"], Ig * (k * S + n * S), 0),
        "sha_rows_kernel<leaves>": (stage_ms["leaf"], Ig * (n * S + n * 32), Ig * n * blocks_per_shard),
        "sha_rows_kernel<verify>": (stage_ms["verify"], Ig * (n * S + n * d * 32 + n * 33 + 32 + n),
                                    Ig * n * (blocks_per_shard + 2 * d)),
    }
    pm = {}
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic_r01.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if pm.get("config") != args.config:
                pm = {}
        except Exception:
            pm = {}

    def roofline(name):
        ms, nbytes, ncomp = kern[name]
        ach = nbytes / (ms / 1e3) / 1e9
        r = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "algorithmic_bytes_per_launch": int(nbytes),
             "avg_ms": round(ms, 4)}
        pk = pm.get("kernels", {}).get(name)
        if pk:
            r["traffic"] = pk["hbm_bytes_per_launch"]
            r["traffic_source"] = os.path.relpath(pmc_path, ROOT)
        if ncomp:
            # SHA-256 is integer-VALU bound (north_star: hashes/s against the VALU
            # peak): compressions/s against the issue-cost-weighted VALU peak, and
            # against the register-resident probe (what the instruction mix attains)
            cps = ncomp / (ms / 1e3)
            r["sha256_compressions_per_s"] = round(cps / 1e9, 3)
            r["sha256_compressions_per_s_unit"] = "G/s"
            r["valu"] = {"achieved": round(cps / 1e9, 3), "peak": round(SHA_PEAK_CPS / 1e9, 2),
                         "unit": "G compressions/s", "frac": round(cps / SHA_PEAK_CPS, 4),
                         "attainable_probe": round(SHA_PROBE_CPS / 1e9, 2),
                         "frac_of_attainable": round(cps / SHA_PROBE_CPS, 4),
                         "model": "4 clk alignbit/add3/perm, 2 clk bitop3/add/shift per wave64 instr; "
                                  "4484 SIMD clk per wave-compression @2.4 GHz"}
            if pk and pk.get("valu_per_compression"):
                r["valu"]["valu_instr_per_compression_pmc"] = pk["valu_per_compression"]
        return r

    dom = max(kern, key=lambda x: kern[x][0])
    roof = roofline(dom)
    codec_roof = roofline(enc_kernel)  # north_star: encode against the HBM peak
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(n, f, B, args.cpu_instances, args.cpu_threads)

    line = {
        "metric": "RBC shard GB/s (RS encode+decode + Merkle verify) per GPU & node, N=128",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded uniform bytes, 10% instances with one corrupted ECHO shard)",
        "config": {"workload": f"{args.config}: {desc}; shard+commit, ECHO verify all N, interpolate from N-f",
                   "n": n, "f": f, "value_bytes": B, "shard_bytes": S, "instances_per_gpu": I,
                   "parallelism": f"instances partitioned over {world} GPU(s), RCCL root all-gather",
                   "streams_per_gpu": nstreams, "gf_codec": ctx.codec,
                   "pipeline": "commit(t) || verify+interpolate(t-1) on two streams" if pipe else "serial"},
        "stage_ms": {kk: round(v, 4) for kk, v in stage_ms.items()},
        "decoded_ok": n_ok,
        "roofline": roof,
        "roofline_encode": codec_roof,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), file=out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(n, f, B, count, threads):
    """The C restatement (oracle/librbc_ref.so: AVX2 split-nibble GF +
    SHA-NI) running the same per-instance pipeline on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rbc_ref

    k = n - 2 * f
    S = (B + k - 1) // k
    rng = np.random.default_rng(7)
    values = rng.integers(0, 256, size=(min(count, 128), B), dtype=np.uint8)  # instance i uses i % 128
    present = np.zeros((count, n), dtype=np.uint8)
    corrupt = np.full(count, -1, dtype=np.int32)
    for i in range(count):
        pres = rng.permutation(n)[: n - f]
        present[i, pres] = 1
        if rng.random() < 0.10:
            corrupt[i] = int(rng.choice(pres))
    threads = max(1, min(threads, os.cpu_count() or 1))
    secs, st = rbc_ref.pipeline(n, f, count, B, threads, values, present, corrupt)
    # one core as well ("1 thread and all cores"), on a 1/16 sample
    c1 = max(1, count // 16)
    secs1, st1 = rbc_ref.pipeline(n, f, c1, B, 1, values, present[:c1], corrupt[:c1])
    feats = rbc_ref.lib().rbcref_cpu_features()
    return {"value": round(count * n * S / secs / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{count} instances x {B} B (N={n} f={f}), same per-instance pipeline as the GPU step, "
                      f"{secs:.2f} s wall on {threads} threads",
            "single_core": {"value": round(c1 * n * S / secs1 / 1e9, 3), "unit": "GB/s", "cores": 1,
                            "sample": f"{c1} instances, {secs1:.2f} s"},
            "simd": ("avx2 " if feats & 1 else "") + ("sha-ni" if feats & 2 else ""), "status_sum": st + st1}


if __name__ == "__main__":
    main()
