#!/usr/bin/env python3
"""RBC data-path benchmark (BASELINE.json metric: "RBC shard GB/s (RS
encode+decode + Merkle verify) per GPU & node, N=128").

One step = one full RBC round of the data path over the instances this rank
owns, resident in HBM (default C2: N=128, f=42, 1 MiB values, 1024 per GPU):
  1. shard+commit   rbc_dev_encode (Split+Encode), rbc_dev_leaves (SHA-256 of
                    every shard), rbc_dev_merkle_build (root + N branches)
  2. Byzantine input: 10 % of instances get one corrupted ECHO shard
  3. ECHO verify    rbc_dev_verify: validateMessage for all N shards of every
                    instance (hash shard + walk branch + compare root)
  4. interpolate    rbc_dev_interpolate: first k valid of a seeded N-f
                    present set -> regenerate the other N-k positions,
                    re-hash them, recheck the root, emit value + digest
  5. (N GPUs > 1)   RCCL all-gather of the {root, digest} records over xGMI
                    (rbc_dev_allgather_records, ragged shares padded)
value = instances x N x S bytes of committed shard output per step, summed
over all ranks, / (max over ranks of the timed wall time).

Scaling: by default every GPU owns `instances` (weak scaling, as the driver
runs N = 1, 2, 4, 8).  --total-instances T partitions T instances over the
ranks in contiguous blocks (strong scaling; BASELINE configs[3] is
`--config c3 --total-instances 8192`).

Launch: python bench.py [--gpus N --steps K --warmup W].  For N > 1 either
under torch.distributed.run (one process per GPU; RANK / LOCAL_RANK /
WORLD_SIZE from the env) or directly: without WORLD_SIZE the process spawns
its N ranks itself before touching any GPU and exits with their status.
Host coordination (RCCL id, barriers, max-over-ranks) is loopback TCP
(cleisthenes_amd.rendezvous), not torch: torch is never imported, so the HIP
runtime and RCCL that librbc_gpu.so links (/opt/rocm) are the ones mapped.
All GPU work, including the RCCL all-gather, goes through librbc_gpu.so.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time
import uuid

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (N, f, value bytes, instances per GPU, description)
    "c1": (64, 21, 1 << 20, 1024, "N=64 f=21 1MiB"),
    "c2": (128, 42, 1 << 20, 1024, "N=128 f=42 1MiB"),
    "c3": (128, 42, 4 << 20, 1024, "N=128 f=42 4MiB"),
    "c4": (256, 85, 64 << 10, 16384, "N=256 f=85 64KiB"),
}
METRIC = "RBC shard GB/s (RS encode+decode + Merkle verify) per GPU & node, N=128"
SEED = 20261015
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


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=150,
                    help="timed steps (the default keeps ~1 s of GPU work in the timed region at C2)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--instances", type=int, default=0, help="instances per GPU (weak scaling; default per config)")
    ap.add_argument("--total-instances", type=int, default=0,
                    help="partition this many instances over the ranks (strong scaling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-configs", default="c1,c2,c3,c4",
                    help="configs the CPU port is also timed on (the bench config always is)")
    ap.add_argument("--pipeline", type=int, default=7,
                    help="7 (default): as 1 with the receiver as rbc_dev_receive_step -- verify(t-1) and the "
                         "regen hashing of t-2 in one SHA launch; 1: overlap batch t's commit (proposer stream) with batch t-1's verify + "
                         "interpolate (receiver stream); 2: three streams -- commit(t) || verify(t-1) || "
                         "interpolate(t-2); 3: phase-aligned -- every step runs the SHA phases of three batches "
                         "together (leaves(t) || verify(t-1) || regen hashing(t-2)), then their GF/FFT/tree "
                         "phases together; 4: as 1 with verify(t-1) split by instances over both streams; "
                         "5: balanced two streams -- commit(t) then rehash+check(t-2) || verify+decode(t-1); "
                         "6: as 1, commit(t) starts when the receiver has DECODED t-2 (overlaps its rehash tail); "

                         "0: one stream, stages in order")
    ap.add_argument("--sets", type=int, default=0,
                    help="shard buffer sets of the pipelined schedule (0: the minimum, 2 for --pipeline 1, "
                         "3 for --pipeline 2; more let the proposer run further ahead)")
    ap.add_argument("--shard-align", type=int, default=128,
                    help="shard row pitch alignment in bytes (multiple of 64; the C ABI needs 64)")
    ap.add_argument("--force-gather", action="store_true",
                    help="run the RCCL all-gather even with one rank (exercises rbc_comm_*)")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the 5 serial steps before the warmup that time each kernel alone on the chip "
                         "(roofline.isolated)")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the PCIe-inclusive host-path measurement (a secondary key, never `value`)")
    ap.add_argument("--rehearse-on-one-gpu", action="store_true",
                    help="rehearsal of the N-rank path on a 1-GPU box: every rank uses device 0 and the "
                         "RCCL all-gather is skipped (RCCL needs one device per rank); everything else -- "
                         "spawn, rendezvous, partition, checks, max-over-ranks -- runs as on N GPUs")
    ap.add_argument("--oracle-samples", type=int, default=16,
                    help="instances whose root and digest are checked against the C oracle after timing")
    return ap.parse_args(argv)


# --------------------------------------------------------------------------
# launch: self-spawn of N ranks (no GPU is touched in the parent)
# --------------------------------------------------------------------------
def spawn_ranks(n, argv, script=None):
    """Start ranks 0..n-1 of `script` (this file) with the torch.distributed.run
    environment; return the first non-zero exit status (the other ranks are
    then terminated: they would wait at the rendezvous), else 0."""
    script = script or os.path.abspath(__file__)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    key = uuid.uuid4().hex
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RBC_RDZV_KEY=key)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # one rank failed: the others would wait at the rendezvous
                    q.terminate()
        time.sleep(0.05)
    return rc


# --------------------------------------------------------------------------
# host facts
# --------------------------------------------------------------------------
def host_info():
    info = {"logical_cpus": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity_cpus"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    info["cgroup_cpu_quota"] = quota
    try:
        info["nproc"] = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout)
    except Exception:
        info["nproc"] = None
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["cpu_model"] = model
    usable = info["affinity_cpus"]
    if quota:
        usable = min(usable, int(quota))
    info["usable_cores"] = max(1, usable)
    return info


def numa_place(ca, dev):
    """Bind this rank's host threads to the CPUs local to its GPU (best effort)."""
    try:
        bus = ca.rbc.pci_bus_id(dev)
        base = f"/sys/bus/pci/devices/{bus}"
        node = int(open(f"{base}/numa_node").read())
        cpus = set()
        for part in open(f"{base}/local_cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        allowed = os.sched_getaffinity(0) & cpus
        if allowed:
            os.sched_setaffinity(0, allowed)
        return {"pci_bus_id": bus, "numa_node": node, "cpus": len(allowed)}
    except Exception as e:  # noqa: BLE001 -- placement is an optimisation only
        return {"error": type(e).__name__}


# --------------------------------------------------------------------------
def main(argv):
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}")

    # ONE JSON line on stdout: keep a private handle on the real stdout and
    # point fd 1 at stderr, so banners that native libraries print with
    # printf (RCCL's version block) cannot precede it
    out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    from cleisthenes_amd.rendezvous import Rendezvous
    rdz = Rendezvous(world, rank)

    import cleisthenes_amd as ca
    from cleisthenes_amd import acs, synth

    n, f, B, inst_default, desc = CONFIGS[args.config]
    if args.total_instances:
        total = args.total_instances
        first, I = acs.partition(total, world, rank)
        scaling = "strong"
    else:
        I = args.instances or inst_default
        total = I * world
        first = rank * I
        scaling = "weak"
    if I < 1:
        raise SystemExit(f"bench: rank {rank} owns no instances ({total} over {world})")
    dev = 0 if args.rehearse_on_one_gpu else local_rank
    placement = numa_place(ca, dev) if world > 1 else None

    ctx = ca.Context(n, f, device=dev)
    k, d = ctx.k, ctx.depth
    S = (B + k - 1) // k
    spitch = round_up(S, args.shard_align)  # row starts on whole 128-B lines: full-line HBM writes
    vpitch = round_up(k * S + 32, 64)
    opitch = round_up(k * S, 16)

    # ---- synthetic inputs: values on the device (global instance id seeds
    # each row); present sets / corruptions from one seeded stream over all
    # `total` instances, this rank's slice taken
    stream = ca.Stream(dev)
    mb = lambda x: ca.DeviceBuffer(x, device=dev)  # noqa: E731
    d_values = mb(I * vpitch)
    ca.rbc.fill_random(dev, stream.ptr, d_values, first, I, vpitch, SEED)
    rng = np.random.default_rng(SEED)
    present_all = np.zeros((total, n), dtype=np.uint8)
    corrupt_all = np.full(total, -1, dtype=np.int32)
    for i in range(total):
        pres = rng.permutation(n)[: n - f]
        present_all[i, pres] = 1
        if rng.random() < 0.10:
            corrupt_all[i] = int(rng.choice(pres))
    present_h = present_all[first:first + I]
    corrupt_h = corrupt_all[first:first + I]

    pipe = bool(args.pipeline)
    pipe3 = args.pipeline in (2, 3, 5)  # per-set valid / verified leaves, >= 3 sets
    phased = args.pipeline in (3, 5)    # per-set value / digest / status
    bal = args.pipeline == 5
    # the pipeline holds two shard sets; when they do not fit the 288 GB of
    # HBM (C3 with all 8192 instances on one GPU: 2 x 100 GB + values) run
    # the serial schedule instead
    set_bytes = I * n * spitch + I * (n * 32 + 32 + n * max(d, 1) * 32)
    other_bytes = I * (vpitch + opitch + n * 34 + 64)
    if pipe3:
        set_bytes += I * (n + n * 32)  # per-set valid + verified leaves (verify and interpolate run apart)
    if phased:
        set_bytes += I * (opitch + 32 + 4)  # per-set value / digest / status (decode and check run apart)
    pdec = args.pipeline == 6  # commit(t) starts when the receiver finished DECODING t-2
    rxs = args.pipeline == 7   # receiver = rbc_dev_receive_step (verify(t) + rehash(t-1) in one SHA launch)
    nsets = max(3 if (pipe3 or pdec or rxs) else 2, args.sets) if pipe else 1
    if rxs:
        set_bytes += I * (n + n * 32 + opitch + 32 + 4) * 2 // 3  # per-parity receiver buffers
    # Wave issue priority (s_setprio) under the two-stream schedule: the
    # receiver stream (verify + interpolate, whose regen-hash tail is a
    # latency-bound dependent chain) at 2, the proposer at 0.  A/B on one box
    # (tools/gpu_runs/gpu_r02prio*.sh): 442-446 GB/s at 0/0, 447-451 at 0/2, 411 at 3/0.
    # RBC_TX_PRIO / RBC_RX_PRIO override.
    prio_tx = int(os.environ.get("RBC_TX_PRIO", "0"))
    prio_rx = int(os.environ.get("RBC_RX_PRIO", "2" if pipe else "0"))
    ctx.set_wave_priority(prio_tx, prio_rx)
    budget = float(os.environ.get("RBC_BENCH_HBM_BUDGET", 250e9))
    while pipe and nsets * set_bytes + other_bytes > budget:
        nsets -= 1
        if nsets < (3 if (pipe3 or rxs or pdec) else 2):
            pipe, pipe3, nsets = False, False, 1
            rxs = pdec = False
    sets = [dict(shards=mb(I * n * spitch), leaves=mb(I * n * 32), roots=mb(I * 32),
                 branches=mb(I * n * max(d, 1) * 32),
                 **({"valid": mb(I * n), "leaves_r": mb(I * n * 32)} if pipe3 else {}),
                 **({"out": mb(I * opitch), "digests": mb(I * 32), "status": mb(I * 4)} if phased else {}))
            for _ in range(nsets)]
    d_present = mb(I * n)
    d_present.upload(present_h)
    d_corrupt = mb(I * 4)
    d_corrupt.upload(corrupt_h)
    d_valid = mb(I * n)
    d_leaves_r = mb(I * n * 32)
    d_out = mb(I * opitch)
    d_digests = mb(I * 32)
    d_status = mb(I * 4)
    d_count = mb(16)
    # --pipeline 7: a batch's receiver buffers live across two receive steps
    rxb = [dict(valid=mb(I * n), leaves_r=mb(I * n * 32), out=mb(I * opitch), digests=mb(I * 32), status=mb(I * 4))
           for _ in range(2)] if rxs else None
    rx_pending = {}
    gather = (world > 1 or args.force_gather) and not args.rehearse_on_one_gpu
    slots = acs.max_share(total, world)
    d_gather = mb(world * slots * 64) if gather else None
    rccl = None
    if gather:
        uid = rdz.broadcast(ca.Context.comm_unique_id() if rank == 0 else None)
        ctx.comm_init(world, rank, uid)
        rccl = ctx.comm_info()
        if rccl["nranks"] != world:
            raise SystemExit(f"bench: RCCL reports {rccl['nranks']} ranks, expected {world}")

    stage_names = ("t0", "enc", "leaf", "tree", "fault", "verify", "interp", "gather")
    # pipelined schedule: P = proposer stream (t0 .. fault), R = receiver
    # stream (r0 .. gather); a stage's time is its own stream's event span
    pipe_spans = (("t0", "enc"), ("enc", "leaf"), ("leaf", "tree"), ("tree", "fault"), ("r0", "verify"),
                  ("verify", "interp"), ("interp", "gather"))
    if pipe3:  # verify on its own stream V: (v0, verify); interpolate on R: (r0, interp)
        pipe_spans = pipe_spans[:4] + (("v0", "verify"), ("r0", "interp"), ("interp", "gather"))
    # one event set per timed step: stage times are read after the closing
    # barrier, so the timed loop never waits on the host between steps
    ev_sets = [{name: ca.Event() for name in stage_names + ("r0", "v0", "l0", "g0", "regen", "t0b", "e0",
                                                            "d0", "decode", "c0", "check")}
               for _ in range(max(args.steps, 3))]

    def step(ev, sp=None):
        sp = sp or sets[0]
        rec = (lambda name: ev[name].record(stream)) if ev is not None else (lambda name: None)
        rec("t0")
        ctx.dev_encode(stream.ptr, I, d_values, vpitch, None, B, sp["shards"], spitch)
        rec("enc")
        ctx.dev_leaves(stream.ptr, I, sp["shards"], spitch, None, S, sp["leaves"])
        rec("leaf")
        ctx.dev_merkle_build(stream.ptr, I, sp["leaves"], sp["roots"], sp["branches"])
        rec("tree")
        ctx.dev_inject_faults(stream.ptr, I, sp["shards"], spitch, d_corrupt)
        rec("fault")
        ctx.dev_verify(stream.ptr, I, sp["shards"], spitch, None, S, sp["branches"], sp["roots"], d_present,
                       d_valid, d_leaves_r)
        rec("verify")
        ctx.dev_interpolate(stream.ptr, I, sp["shards"], spitch, None, S, d_valid, d_leaves_r, 1, sp["roots"],
                            d_out, opitch, d_digests, d_status)
        rec("interp")
        if gather:
            ctx.dev_allgather_records(stream.ptr, I, slots, sp["roots"], d_digests, d_status, d_gather)
        rec("gather")

    # --pipeline: proposer stream P commits batch t into set t%2 while the
    # receiver stream R verifies + interpolates batch t-1 from the other set.
    # A set is reused only after R has finished with it (evR), and R starts a
    # batch only after P committed it (evP): K timed steps = K commits + K
    # decodes, all inside the timed region.
    # RBC_BENCH_PRIO (A/B knob): "R" puts the receiver stream (verify +
    # interpolate, whose regen-hash tail is latency-bound) at high priority,
    # "P" the proposer stream
    prio = os.environ.get("RBC_BENCH_PRIO", "")
    if pipe and prio == "P":
        stream.sync()  # the input fill ran on the old stream
        stream = ca.Stream(dev, priority="high")
    rstream = ca.Stream(dev, priority="high" if prio == "R" else None) if pipe else None
    # RBC_BENCH_CU_SPLIT=a/b (A/B knob): the proposer stream gets CUs with
    # (cu % b) < a, the receiver stream the rest -- disjoint CUs instead of both
    # stages' kernels sharing every CU (and its instruction cache)
    split = os.environ.get("RBC_BENCH_CU_SPLIT", "")
    if pipe and split:
        a_, b_ = (int(x) for x in split.split("/"))
        ncu = ca.rbc.cu_count(dev)
        stream.sync()
        stream = ca.Stream(dev, cu_mask=[c for c in range(ncu) if c % b_ < a_])
        rstream = ca.Stream(dev, cu_mask=[c for c in range(ncu) if c % b_ >= a_])
    vstream = ca.Stream(dev) if pipe3 else None  # --pipeline 2: verify stream V; 3: stream Z
    ctxV = ca.Context(n, f, device=dev) if pipe3 else None  # own decode/verify workspace per stream
    evP = [ca.Event() for _ in range(nsets)]
    evR = [ca.Event() for _ in range(nsets)]
    evV = [ca.Event() for _ in range(nsets)]
    for e in evP + evR + evV:
        e.record(stream)  # recorded once, so every wait below is well defined

    def pstep3(t, ev=None):
        """commit(t) on P || verify(t-1) on V || interpolate(t-2) on R; a set
        is reused by commit(t) only after interpolate(t - nsets) read it."""
        P, V, R = stream, vstream, rstream
        rec = (lambda name, st: ev[name].record(st)) if ev is not None else (lambda name, st: None)
        sp = sets[t % nsets]
        P.wait(evR[t % nsets])
        rec("t0", P)
        ctx.dev_encode(P.ptr, I, d_values, vpitch, None, B, sp["shards"], spitch)
        rec("enc", P)
        ctx.dev_leaves(P.ptr, I, sp["shards"], spitch, None, S, sp["leaves"])
        rec("leaf", P)
        ctx.dev_merkle_build(P.ptr, I, sp["leaves"], sp["roots"], sp["branches"])
        rec("tree", P)
        ctx.dev_inject_faults(P.ptr, I, sp["shards"], spitch, d_corrupt)
        rec("fault", P)
        evP[t % nsets].record(P)
        if t >= 1:
            sv = sets[(t - 1) % nsets]
            V.wait(evP[(t - 1) % nsets])
            rec("v0", V)
            ctxV.dev_verify(V.ptr, I, sv["shards"], spitch, None, S, sv["branches"], sv["roots"], d_present,
                            sv["valid"], sv["leaves_r"])
            rec("verify", V)
            evV[(t - 1) % nsets].record(V)
        if t >= 2:
            sr = sets[(t - 2) % nsets]
            R.wait(evV[(t - 2) % nsets])
            rec("r0", R)
            ctx.dev_interpolate(R.ptr, I, sr["shards"], spitch, None, S, sr["valid"], sr["leaves_r"], 1,
                                sr["roots"], d_out, opitch, d_digests, d_status)
            rec("interp", R)
            if gather:
                ctx.dev_allgather_records(R.ptr, I, slots, sr["roots"], d_digests, d_status, d_gather)
            rec("gather", R)
            evR[(t - 2) % nsets].record(R)

    # RBC_BENCH_PWAIT=verify (A/B knob, needs >= 3 sets): commit(t) starts when
    # the receiver finished VERIFYING batch t-2 (which implies decode(t-3),
    # the last reader of set t % nsets, is done) instead of when it finished
    # decoding t-2: the commit then overlaps the decode's tail, not its head
    pwait_verify = os.environ.get("RBC_BENCH_PWAIT", "") == "verify" and nsets >= 3
    evRV = [ca.Event() for _ in range(nsets)]
    # --pipeline 6: interpolate(t-1) runs as DECODE (value join forked onto
    # the aux stream) then REHASH + CHECK; commit(t) waits for the DECODE of
    # t-2 (which implies batch t-3, the last reader of set t % 3, is done),
    # so the commit overlaps the latency-bound regen-hash tail instead of
    # starting when it ends
    evRD = [ca.Event() for _ in range(nsets)]
    for e in evRV + evRD:
        e.record(stream)

    def pstep(t, ev=None):
        P, R = stream, rstream
        recP = (lambda name: ev[name].record(P)) if ev is not None else (lambda name: None)
        recR = (lambda name: ev[name].record(R)) if ev is not None else (lambda name: None)
        sp = sets[t % nsets]
        if pwait_verify:
            if t >= 2:
                P.wait(evRV[(t - 2) % nsets])
        elif pdec:
            if t >= 2:
                P.wait(evRD[(t - 2) % nsets])
        else:
            P.wait(evR[t % nsets])
        recP("t0")
        ctx.dev_encode(P.ptr, I, d_values, vpitch, None, B, sp["shards"], spitch)
        recP("enc")
        ctx.dev_leaves(P.ptr, I, sp["shards"], spitch, None, S, sp["leaves"])
        recP("leaf")
        ctx.dev_merkle_build(P.ptr, I, sp["leaves"], sp["roots"], sp["branches"])
        recP("tree")
        ctx.dev_inject_faults(P.ptr, I, sp["shards"], spitch, d_corrupt)
        recP("fault")
        evP[t % nsets].record(P)
        if t == 0:
            return
        sr = sets[(t - 1) % nsets]
        R.wait(evP[(t - 1) % nsets])
        recR("r0")
        ctx.dev_verify(R.ptr, I, sr["shards"], spitch, None, S, sr["branches"], sr["roots"], d_present, d_valid,
                       d_leaves_r)
        recR("verify")
        evRV[(t - 1) % nsets].record(R)
        if pdec:
            iargs = (I, sr["shards"], spitch, None, S, d_valid, d_leaves_r, 1, sr["roots"], d_out, opitch,
                     d_digests, d_status)
            ctx.dev_interpolate_phases(R.ptr, ctx.INTERP_DECODE | ctx.INTERP_FORK, *iargs)
            evRD[(t - 1) % nsets].record(R)
            ctx.dev_interpolate_phases(R.ptr, ctx.INTERP_REHASH | ctx.INTERP_CHECK, *iargs)
        else:
            ctx.dev_interpolate(R.ptr, I, sr["shards"], spitch, None, S, d_valid, d_leaves_r, 1, sr["roots"],
                                d_out, opitch, d_digests, d_status)
        recR("interp")
        if gather:
            ctx.dev_allgather_records(R.ptr, I, slots, sr["roots"], d_digests, d_status, d_gather)
        recR("gather")
        evR[(t - 1) % nsets].record(R)

    # --pipeline 4 (A/B option): the two-stream schedule with ECHO verify of
    # batch t-1 split by instances over both streams, so that the proposer
    # stream P (encode + leaves + tree, the shorter one) takes half of the
    # receiver stream's SHA work: P verifies the first half of t-1 (its own
    # context's workspace) then commits t; R verifies the second half, waits
    # for P's half and interpolates t-1.
    def pstep_rx(t, ev=None):
        """--pipeline 7: P commits t into set t % 3 once batch t-3 is complete;
        R runs rbc_dev_receive_step(cur = t-1, prev = t-2): verify(t-1) and
        the regen hashing of t-2 in one SHA launch, t-2's recheck + digest,
        then t-1's decode; batch t-2 is complete when it returns."""
        P, R = stream, rstream
        recP = (lambda name: ev[name].record(P)) if ev is not None else (lambda name: None)
        recR = (lambda name: ev[name].record(R)) if ev is not None else (lambda name: None)
        sp = sets[t % nsets]
        P.wait(evR[t % nsets])
        recP("t0")
        ctx.dev_encode(P.ptr, I, d_values, vpitch, None, B, sp["shards"], spitch)
        recP("enc")
        ctx.dev_leaves(P.ptr, I, sp["shards"], spitch, None, S, sp["leaves"])
        recP("leaf")
        ctx.dev_merkle_build(P.ptr, I, sp["leaves"], sp["roots"], sp["branches"])
        recP("tree")
        ctx.dev_inject_faults(P.ptr, I, sp["shards"], spitch, d_corrupt)
        recP("fault")
        evP[t % nsets].record(P)
        if t == 0:
            return
        x = t - 1
        sr, rb = sets[x % nsets], rxb[x % 2]
        R.wait(evP[x % nsets])
        recR("r0")
        cur = ctx.rx_batch(I, sr["shards"], spitch, None, S, sr["branches"], sr["roots"], d_present, rb["valid"],
                           rb["leaves_r"], rb["out"], opitch, rb["digests"], rb["status"])
        prev = rx_pending.pop(x - 1, None)
        # "verify" = the step's hashing launch (verify(t-1) + regen hashing of t-2),
        # "interp" = the rest (recheck(t-2), decode(t-1))
        ctx.dev_receive_step(R.ptr, cur, prev, ev["verify"] if ev is not None else None)
        rx_pending[x] = cur
        recR("interp")
        if gather and prev is not None:
            pb = rxb[(x - 1) % 2]
            ctx.dev_allgather_records(R.ptr, I, slots, sets[(x - 1) % nsets]["roots"], pb["digests"], pb["status"],
                                      d_gather)
        recR("gather")
        if prev is not None:
            evR[(x - 1) % nsets].record(R)

    def rx_flush():
        """complete the batch the last receive step decoded (outside the timed region)"""
        if rxs and rx_pending:
            x, cur = rx_pending.popitem()
            ctx.dev_receive_step(rstream.ptr, None, cur)
            if gather:  # the guard checks the gathered records of this batch
                pb = rxb[x % 2]
                ctx.dev_allgather_records(rstream.ptr, I, slots, sets[x % nsets]["roots"], pb["digests"],
                                          pb["status"], d_gather)
            rstream.sync()
            return x
        return None

    vsplit = args.pipeline == 4
    if vsplit:
        h1 = I // 2
        ctxS = ca.Context(n, f, device=dev)
        evVa = [ca.Event() for _ in range(nsets)]
        for e in evVa:
            e.record(stream)

    def vhalf(c, st, sr, lo, hi):
        if hi <= lo:
            return
        c.dev_verify(st.ptr, hi - lo, sr["shards"].ptr.value + lo * n * spitch, spitch, None, S,
                     sr["branches"].ptr.value + lo * n * max(d, 1) * 32, sr["roots"].ptr.value + lo * 32,
                     d_present.ptr.value + lo * n, d_valid.ptr.value + lo * n, d_leaves_r.ptr.value + lo * n * 32)

    def pstep_split(t, ev=None):
        P, R = stream, rstream
        recP = (lambda name: ev[name].record(P)) if ev is not None else (lambda name: None)
        recR = (lambda name: ev[name].record(R)) if ev is not None else (lambda name: None)
        sp = sets[t % nsets]
        sr = sets[(t - 1) % nsets] if t >= 1 else None
        if t >= 1:  # P's half of verify(t-1): commit(t-1) ran on P already
            if t >= 2:
                P.wait(evR[(t - 2) % nsets])  # interpolate(t-2) is done with d_valid / d_leaves_r
            recP("v0")
            vhalf(ctxS, P, sr, 0, h1)
            evVa[(t - 1) % nsets].record(P)
        P.wait(evR[t % nsets])
        recP("t0")
        ctx.dev_encode(P.ptr, I, d_values, vpitch, None, B, sp["shards"], spitch)
        recP("enc")
        ctx.dev_leaves(P.ptr, I, sp["shards"], spitch, None, S, sp["leaves"])
        recP("leaf")
        ctx.dev_merkle_build(P.ptr, I, sp["leaves"], sp["roots"], sp["branches"])
        recP("tree")
        ctx.dev_inject_faults(P.ptr, I, sp["shards"], spitch, d_corrupt)
        recP("fault")
        evP[t % nsets].record(P)
        if t == 0:
            return
        R.wait(evP[(t - 1) % nsets])
        recR("r0")
        vhalf(ctx, R, sr, h1, I)
        recR("verify")
        R.wait(evVa[(t - 1) % nsets])
        ctx.dev_interpolate(R.ptr, I, sr["shards"], spitch, None, S, d_valid, d_leaves_r, 1, sr["roots"], d_out,
                            opitch, d_digests, d_status)
        recR("interp")
        if gather:
            ctx.dev_allgather_records(R.ptr, I, slots, sr["roots"], d_digests, d_status, d_gather)
        recR("gather")
        evR[(t - 1) % nsets].record(R)

    # --pipeline 5 (A/B option): balanced two-stream schedule.  P commits t,
    # then rehashes the regenerated rows of t-2 and checks its root; R
    # verifies and decodes t-1.  Isolated work per stream: P 4.0 ms (encode,
    # leaves, tree, regen hashing, root check), R 4.1 (verify, prepare, GF,
    # FFT, join) instead of 2.9 / 4.9.  The decode and rehash of one batch
    # share a context's regen list, so batches alternate between two contexts.
    if bal:
        evD = [ca.Event() for _ in range(nsets)]
        for e in evD:
            e.record(stream)

    def pstep_bal(t, ev=None):
        P, R = stream, rstream
        recP = (lambda name: ev[name].record(P)) if ev is not None else (lambda name: None)
        recR = (lambda name: ev[name].record(R)) if ev is not None else (lambda name: None)
        cxo = (ctx, ctxV)
        sp = sets[t % nsets]
        # set t % 3 last held batch t-3, whose check ran on P (step t-1) after
        # waiting for its decode on R: P's own order frees it
        recP("t0")
        ctx.dev_encode(P.ptr, I, d_values, vpitch, None, B, sp["shards"], spitch)
        recP("enc")
        ctx.dev_leaves(P.ptr, I, sp["shards"], spitch, None, S, sp["leaves"])
        recP("leaf")
        ctx.dev_merkle_build(P.ptr, I, sp["leaves"], sp["roots"], sp["branches"])
        recP("tree")
        ctx.dev_inject_faults(P.ptr, I, sp["shards"], spitch, d_corrupt)
        recP("fault")
        evP[t % nsets].record(P)
        if t >= 2:
            s2, c2 = sets[(t - 2) % nsets], cxo[(t - 2) % 2]
            P.wait(evD[(t - 2) % nsets])
            recP("g0")
            c2.dev_interpolate_phases(P.ptr, ctx.INTERP_REHASH, I, s2["shards"], spitch, None, S, s2["valid"],
                                      s2["leaves_r"], 1, s2["roots"], s2["out"], opitch, s2["digests"], s2["status"])
            recP("regen")
            c2.dev_interpolate_phases(P.ptr, ctx.INTERP_CHECK, I, s2["shards"], spitch, None, S, s2["valid"],
                                      s2["leaves_r"], 1, s2["roots"], s2["out"], opitch, s2["digests"], s2["status"])
            recP("check")
            if gather:
                ctx.dev_allgather_records(P.ptr, I, slots, s2["roots"], s2["digests"], s2["status"], d_gather)
            recP("gather")
        if t >= 1:
            s1, c1 = sets[(t - 1) % nsets], cxo[(t - 1) % 2]
            R.wait(evP[(t - 1) % nsets])
            recR("v0")
            c1.dev_verify(R.ptr, I, s1["shards"], spitch, None, S, s1["branches"], s1["roots"], d_present,
                          s1["valid"], s1["leaves_r"])
            recR("verify")
            c1.dev_interpolate_phases(R.ptr, ctx.INTERP_DECODE, I, s1["shards"], spitch, None, S, s1["valid"],
                                      s1["leaves_r"], 1, s1["roots"], s1["out"], opitch, s1["digests"], s1["status"])
            recR("decode")
            evD[(t - 1) % nsets].record(R)

    # --pipeline 3: phase-aligned schedule on three streams X, Y, Z.  Step k:
    #   SHA phase     X: leaves(k)        Y: verify(k-1)     Z: rehash(k-2)
    #   non-SHA phase X: tree+fault(k),   Y: decode(k-1)     Z: check(k-2)
    #                    encode(k+1)         (prepare, GF,       (+ gather)
    #                                         FFT, join)
    # Every stream waits for all three streams' previous phase, so the SHA
    # kernels of three batches (2048 + 1376 + 672 waves at C2: four per SIMD)
    # run together and the GF/FFT transforms run together -- two SHA kernels
    # share CUs well, a transform beside SHA does not.
    # Set k % nsets is rewritten by encode(k+1)'s set only after rehash(k-2).
    if phased and not bal:
        X, Y, Z = stream, rstream, vstream
        evA = {nm: ca.Event() for nm in ("X", "Y", "Z")}  # end of a SHA phase, per stream
        evB = {nm: ca.Event() for nm in ("X", "Y", "Z")}  # end of a non-SHA phase, per stream
        for e in list(evA.values()) + list(evB.values()):
            e.record(stream)
        # encode(0) before the first step
        ctx.dev_encode(X.ptr, I, d_values, vpitch, None, B, sets[0]["shards"], spitch)
        evB["X"].record(X)

    def phase_wait(st, evs):
        for e in evs.values():
            st.wait(e)

    def pstep_phased(k, ev=None):
        rec = (lambda name, st: ev[name].record(st)) if ev is not None else (lambda name, st: None)
        sk, s1, s2 = sets[k % nsets], sets[(k - 1) % nsets], sets[(k - 2) % nsets]
        # ---- SHA phase
        for st in (X, Y, Z):
            phase_wait(st, evB)
        rec("l0", X)
        ctx.dev_leaves(X.ptr, I, sk["shards"], spitch, None, S, sk["leaves"])
        rec("leaf", X)
        if k >= 1:
            rec("v0", Y)
            ctxV.dev_verify(Y.ptr, I, s1["shards"], spitch, None, S, s1["branches"], s1["roots"], d_present,
                            s1["valid"], s1["leaves_r"])
            rec("verify", Y)
        if k >= 2:
            rec("g0", Z)
            ctx.dev_interpolate_phases(Z.ptr, ctx.INTERP_REHASH, I, s2["shards"], spitch, None, S, s2["valid"],
                                       s2["leaves_r"], 1, s2["roots"], s2["out"], opitch, s2["digests"],
                                       s2["status"])
            rec("regen", Z)
        for nm, st in (("X", X), ("Y", Y), ("Z", Z)):
            evA[nm].record(st)
        # ---- non-SHA phase
        for st in (X, Y, Z):
            phase_wait(st, evA)
        rec("t0b", X)
        ctx.dev_merkle_build(X.ptr, I, sk["leaves"], sk["roots"], sk["branches"])
        rec("tree", X)
        ctx.dev_inject_faults(X.ptr, I, sk["shards"], spitch, d_corrupt)
        rec("fault", X)
        rec("e0", X)
        ctx.dev_encode(X.ptr, I, d_values, vpitch, None, B, sets[(k + 1) % nsets]["shards"], spitch)
        rec("enc", X)
        if k >= 1:
            rec("d0", Y)
            ctx.dev_interpolate_phases(Y.ptr, ctx.INTERP_DECODE, I, s1["shards"], spitch, None, S, s1["valid"],
                                       s1["leaves_r"], 1, s1["roots"], s1["out"], opitch, s1["digests"],
                                       s1["status"])
            rec("decode", Y)
        if k >= 2:
            rec("c0", Z)
            ctx.dev_interpolate_phases(Z.ptr, ctx.INTERP_CHECK, I, s2["shards"], spitch, None, S, s2["valid"],
                                       s2["leaves_r"], 1, s2["roots"], s2["out"], opitch, s2["digests"],
                                       s2["status"])
            rec("check", Z)
            if gather:
                ctx.dev_allgather_records(Z.ptr, I, slots, s2["roots"], s2["digests"], s2["status"], d_gather)
            rec("gather", Z)
        for nm, st in (("X", X), ("Y", Y), ("Z", Z)):
            evB[nm].record(st)

    def barrier():
        if rstream is not None:
            rstream.sync()
        if vstream is not None:
            vstream.sync()
        stream.sync()
        ca.rbc.lib.rbc_device_sync(dev)
        rdz.barrier()

    # the same kernels alone on the chip (serial schedule, events per stage),
    # BEFORE the warmup so that the timed launches stay the last ones a
    # rocprof trace holds: under the pipeline a kernel's span also holds the
    # other stream's work, so the roofline carries both figures
    iso_ms = None
    if pipe and not phased and not args.no_isolated:
        for _ in range(2):
            step(None)
        iso_ev = ev_sets[:3]
        for ev in iso_ev:
            step(ev)
        stream.sync()
        iso_ms = {b_: sum(ev[a_].elapsed_ms(ev[b_]) for ev in iso_ev) / len(iso_ev)
                  for a_, b_ in zip(stage_names[:-1], stage_names[1:])}

    # (the receiver alone as rbc_dev_receive_step, 8 back-to-back batches:
    # 5.65 ms per C2 batch with its one-wave blocks, 4.87 with 256-thread
    # blocks, against 4.77 for verify + interpolate as separate calls -- the
    # receive step pays off only beside the proposer's stream)
    rx_sha_iso_ms = None

    if pipe:
        args.warmup = max(args.warmup, 3 if (pipe3 or rxs) else 2)  # fill the pipeline: a decode before the guard
        for t in range(args.warmup):
            (pstep_rx if rxs else pstep_bal if bal else pstep_phased if phased else pstep3 if pipe3 else pstep_split if vsplit
             else pstep)(t)
    else:
        for _ in range(args.warmup):
            step(None)
    barrier()

    stage_ms = {kk: 0.0 for kk in stage_names[1:]}
    barrier()
    t0 = time.perf_counter()
    if pipe:
        for t in range(args.warmup, args.warmup + args.steps):
            (pstep_rx if rxs else pstep_bal if bal else pstep_phased if phased else pstep3 if pipe3 else pstep_split if vsplit
             else pstep)(t, ev_sets[t - args.warmup])
    else:
        for t in range(args.steps):
            step(ev_sets[t])
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = rdz.max(elapsed)
    # the set the last decode read
    last = sets[(args.warmup + args.steps - (3 if pipe3 else 2)) % nsets] if pipe else sets[0]
    x_last = rx_flush()
    if rxs:
        last = sets[x_last % nsets]
    if bal:
        pipe_spans = (("t0", "enc"), ("enc", "leaf"), ("leaf", "tree"), ("tree", "fault"), ("v0", "verify"),
                      ("verify", "decode"), ("g0", "regen"), ("regen", "check"), ("check", "gather"))
        stage_ms.update(decode=0.0, regen=0.0, check=0.0)
    elif phased:
        pipe_spans = (("e0", "enc"), ("l0", "leaf"), ("t0b", "tree"), ("tree", "fault"), ("v0", "verify"),
                      ("d0", "decode"), ("g0", "regen"), ("c0", "check"), ("check", "gather"))
        stage_ms.update(decode=0.0, regen=0.0, check=0.0)
    for ev in ev_sets[: args.steps]:
        spans = pipe_spans if pipe else zip(stage_names[:-1], stage_names[1:])
        for a, b in spans:
            stage_ms[b] += ev[a].elapsed_ms(ev[b]) / args.steps
    if phased:  # interpolate = its three phases
        stage_ms["interp"] = stage_ms.pop("decode") + stage_ms.pop("regen") + stage_ms.pop("check")

    # ---- correctness of the timed run's last round (outside the timed region)
    res_out, res_status, res_dig = ((last["out"], last["status"], last["digests"]) if phased
                                    else (rxb[x_last % 2]["out"], rxb[x_last % 2]["status"],
                                          rxb[x_last % 2]["digests"]) if rxs
                                    else (d_out, d_status, d_digests))
    checks = check_results(args, ca, acs, synth, rdz, ctx, dev, stream, world, rank, first, I, total, slots, n, f,
                           k, B, S, vpitch, opitch, d_values, res_out, res_status, res_dig, last["roots"],
                           d_gather, d_count, gather)

    ms_per_step = elapsed_max * 1000.0 / args.steps
    shard_bytes_all = total * n * S
    value = shard_bytes_all * args.steps / elapsed_max / 1e9

    # ---- roofline of the dominant kernel ---------------------------------
    blocks_per_shard = (S + 9 + 63) // 64
    R_rows = int(present_h.sum())  # received ECHO shards over this rank's instances
    enc_kernel = "rs_fft_kernel<encode>" if ctx.codec == "fft" else "gf_rows_kernel<encode>"
    kern = {
        # name: (avg ms, algorithmic HBM bytes per launch, sha compressions per launch)
        enc_kernel: (stage_ms["enc"], I * (k * S + n * S), 0),
        "sha_rows_kernel<leaves>": (stage_ms["leaf"], I * (n * S + n * 32), I * n * blocks_per_shard),
        # ECHO verify hashes the received shards only (R = N-f per instance)
        "sha_rows_kernel<verify>": (stage_ms["verify"], R_rows * (S + d * 32 + 32) + I * (32 + 2 * n),
                                    R_rows * (blocks_per_shard + 2 * d)),
    }
    regen_rows = int(I * n - present_h.sum() + (corrupt_h >= 0).sum())
    if rxs:  # --pipeline 7: ECHO verify of t and the regen hashing of t-1 are one launch
        del kern["sha_rows_kernel<verify>"]
        kern["sha_rx_kernel<verify+regen>"] = (
            stage_ms["verify"], R_rows * (S + d * 32 + 32) + I * (32 + 2 * n) + regen_rows * (S + 32),
            R_rows * (blocks_per_shard + 2 * d) + regen_rows * blocks_per_shard)
    # PMC-measured HBM traffic per launch (tools/profile.sh + tools/pmc_summary.py
    # on this bench's default command), newest round first
    pm, pmc_path = {}, None
    for cand in ("pmc_traffic_r02s8.json", "pmc_traffic_r02.json", "pmc_traffic_r01.json"):
        pth = os.path.join(ROOT, "profiles", cand)
        if os.path.exists(pth):
            try:
                pm = json.load(open(pth))
            except Exception:
                pm = {}
            if pm.get("config") == args.config and pm.get("instances", 1024) == I:
                pmc_path = pth
                break
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
            r["bound_note"] = ("SHA-256 is integer-VALU bound: HBM frac is not this kernel's roof (see valu and "
                               "isolated); avg_ms is its span beside the other stream's kernels")
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
                                  "4484 SIMD clk per wave-compression @2.4 GHz nominal (the chip runs ~2.1 GHz "
                                  "under this load, so 1.0 is not reachable)"}
            if pk and pk.get("valu_per_compression"):
                r["valu"]["valu_instr_per_compression_pmc"] = pk["valu_per_compression"]
        return r

    # chip-level SHA-256 rate of the whole step (all three hashing kernels,
    # both streams): under the pipelined schedule a kernel's own span also
    # holds the other stream's work, so this is the utilisation figure
    step_comp = I * n * blocks_per_shard + R_rows * (blocks_per_shard + 2 * d) + regen_rows * blocks_per_shard
    step_cps = step_comp / (elapsed_max / args.steps)  # per GPU
    sha_chip = {"compressions_per_step": int(step_comp), "achieved": round(step_cps / 1e9, 2),
                "unit": "G compressions/s per GPU", "attainable_probe": round(SHA_PROBE_CPS / 1e9, 2),
                "frac_of_attainable": round(step_cps / SHA_PROBE_CPS, 3),
                "note": "leaves (all N rows) + ECHO verify (received rows + branch walk) + interpolate's "
                        "regenerated rows, per ms_per_step"}

    dom = max(kern, key=lambda x: kern[x][0])
    roof = roofline(dom)
    codec_roof = roofline(enc_kernel)  # north_star: encode against the HBM peak
    if iso_ms is not None:
        stage_of = {enc_kernel: "enc", "sha_rows_kernel<leaves>": "leaf", "sha_rows_kernel<verify>": "verify",
                    "sha_rx_kernel<verify+regen>": "rx_sha"}
        iso_all = dict(iso_ms, rx_sha=rx_sha_iso_ms)
        for r in (roof, codec_roof):
            ms_i = iso_all[stage_of[r["kernel"]]]
            if not ms_i:
                continue
            _, nbytes, ncomp = kern[r["kernel"]]
            iso = {"avg_ms": round(ms_i, 4), "achieved": round(nbytes / (ms_i / 1e3) / 1e9, 1),
                   "frac": round(nbytes / (ms_i / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                   "note": "same kernel and batch alone on the chip (3 serial steps before the warmup); "
                           "avg_ms above is its span under the two-stream pipeline, shared with the other "
                           "stream's kernels"}
            if ncomp:
                cps = ncomp / (ms_i / 1e3)
                iso["valu_frac_of_attainable"] = round(cps / SHA_PROBE_CPS, 4)
            r["isolated"] = iso

    # BASELINE configs[1] measures RS encode + Merkle build alone: the same
    # kernels timed alone on the chip (the serial steps before the warmup, or
    # the serial schedule's own spans)
    commit_src = iso_ms if iso_ms is not None else (stage_ms if not pipe else None)
    commit_only = None
    if commit_src is not None:
        cms = commit_src["enc"] + commit_src["leaf"] + commit_src["tree"]
        commit_only = {"GBps": round(I * n * S / (cms / 1e3) / 1e9, 2), "ms_per_batch": round(cms, 4),
                       "unit": "GB/s of committed shard bytes (N*S per instance), per rank",
                       "note": "RS encode + Merkle build alone (BASELINE configs[1]'s stages): encode + leaf "
                               "hashing + tree spans of serial steps"}
    receive_only = None
    if commit_src is not None:
        rms = commit_src["verify"] + commit_src["interp"]
        receive_only = {"GBps": round(I * n * S / (rms / 1e3) / 1e9, 2), "ms_per_batch": round(rms, 4),
                        "unit": "GB/s of committed shard bytes (N*S per instance), per rank",
                        "note": "ECHO-side Merkle branch verify + RS reconstruct / re-encode / root recheck alone "
                                "(BASELINE configs[2]'s stages): verify + interpolate spans of serial steps"}

    # GPU phase rates (per rank, from the stage events): encode+commit =
    # N*S shard bytes per instance; verify+decode = k*S value bytes
    enc_ms = stage_ms["enc"] + stage_ms["leaf"] + stage_ms["tree"]
    dec_ms = stage_ms["verify"] + stage_ms["interp"]
    phases = {"encode_commit": {"gpu_gbs": round(I * n * S / (enc_ms / 1e3) / 1e9, 2), "bytes": "N*S per instance"},
              "verify_decode": {"gpu_gbs": round(I * k * S / (dec_ms / 1e3) / 1e9, 2), "bytes": "k*S per instance"}}

    cpu = None
    host = host_info()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, host)
        for ph in ("encode_commit", "verify_decode"):
            phases[ph]["cpu_gbs"] = cpu["phases"][ph]
            phases[ph]["gpu_over_cpu"] = round(phases[ph]["gpu_gbs"] / cpu["phases"][ph], 1)

    pcie = None
    if rank == 0 and world == 1 and not args.no_pcie:
        # what a Go batcher sees with host buffers in and out (pinned rings,
        # two submissions in flight): PCIe-bound, reported beside `value`
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import host_bench
        pcie = host_bench.measure(ca, n, f, B, batch=64, batches=8, inflight=2, pinned=True, device=dev)
        pcie["unit"] = "GB/s of committed shard bytes (N*S per instance), host memory in and out"

    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": round(value / cpu["value"], 2) if cpu else None,
        "vs_baseline_basis": ("GPU value / cpu_baseline.value: the C restatement of the Go CPU path on this "
                              "box's host cores, same config (BASELINE.md publishes no number)") if cpu else None,
        "dtype": "u8",
        "data": "synthetic (device-generated splitmix64 bytes per instance, seeded; 10% of instances with one "
                "corrupted ECHO shard)",
        "config": {"workload": f"{args.config}: {desc}, {total} instances ({I} on this rank); shard+commit, "
                               "ECHO verify all N, interpolate from N-f",
                   "n": n, "f": f, "value_bytes": B, "shard_bytes": S, "instances_total": total,
                   "instances_per_gpu": I,
                   "parallelism": f"instances partitioned over {world} GPU(s) in contiguous blocks"
                                  + (", RCCL all-gather of {root,digest} records" if gather else ""),
                   "gf_codec": ctx.codec,
                   "wave_priority": {"commit": prio_tx, "receive": prio_rx},
                   **({"rehearsal": "all ranks on device 0, no RCCL (not a multi-GPU measurement)"}
                      if args.rehearse_on_one_gpu else {}),
                   "pipeline": ((f"balanced: commit(t) then rehash+check(t-2) || verify+decode(t-1), two streams, "
                                 f"{nsets} shard sets") if bal else
                                (f"phase-aligned: SHA of leaves(t) || verify(t-1) || rehash(t-2), then tree/encode "
                                 f"|| decode(t-1) || check(t-2), three streams, {nsets} shard sets") if phased else
                                (f"commit(t) || verify(t-1) || interpolate(t-2) on three streams, {nsets} shard "
                                 "sets") if pipe3 else
                                (f"verify(t-1) first half || second half, then commit(t) || interpolate(t-1), "
                                 f"two streams, {nsets} shard sets") if vsplit else
                                (f"commit(t) || receive step: verify(t-1) + rehash(t-2) in one SHA launch, "
                                 f"recheck(t-2), decode(t-1) (rbc_dev_receive_step), two streams, {nsets} shard "
                                 "sets") if rxs else
                                (f"commit(t) from decode(t-2) on || verify+interpolate(t-1) (decode, then "
                                 f"rehash+check), two streams, {nsets} shard sets") if pdec else
                                (f"commit(t) || verify+interpolate(t-1) on two streams, {nsets} shard sets")
                                if pipe else "serial")},
        "stage_ms": {kk: round(v, 4) for kk, v in stage_ms.items()},
        "phases": phases,
        "commit_only": commit_only,
        "receive_only": receive_only,
        **checks,
        "roofline": roof,
        "roofline_encode": codec_roof,
        "sha256_chip": sha_chip,
        "cpu_baseline": cpu,
        "pcie_inclusive": pcie,
        "rccl": rccl,
        "host": {kk: host[kk] for kk in ("cpu_model", "nproc", "cgroup_cpu_quota", "affinity_cpus")},
    }
    if placement:
        line["numa"] = rdz.allgather(placement)
    if not all(checks[c] for c in ("values_ok", "oracle_sample_ok", "gather_ok")) or \
            checks["decoded_ok"] != total:
        print(json.dumps({"error": "correctness check failed", **checks}), file=sys.stderr, flush=True)
        rdz.close()
        return 3
    if rank == 0:
        print(json.dumps(line), file=out, flush=True)
    rdz.barrier()
    rdz.close()
    return 0


def check_results(args, ca, acs, synth, rdz, ctx, dev, stream, world, rank, first, I, total, slots, n, f, k, B, S,
                  vpitch, opitch, d_values, d_out, d_status, d_digests, d_roots, d_gather, d_count, gather):
    """After the timed loop: every instance decoded, every decoded value equals
    its input, the gathered records of every rank are what that rank holds,
    and sampled roots / digests equal the C oracle's (checker only: nothing
    here is timed or shipped)."""
    stream.sync()
    status = d_status.download(I * 4).view(np.int32)
    n_ok = rdz.sum(int((status == 0).sum()))
    ca.rbc.count_mismatch(dev, stream.ptr, d_out, opitch, d_values, vpitch, I, B, d_count)
    stream.sync()
    mism = int(d_count.download(4).view(np.uint32)[0])
    values_ok = rdz.all(mism == 0)
    roots = d_roots.download(I * 32).reshape(I, 32)
    digests = d_digests.download(I * 32).reshape(I, 32)
    gather_ok = True
    if gather:
        mine = acs.pack_records(roots, digests, slots, status)
        everyone = rdz.allgather(mine.tobytes())
        g = d_gather.download().reshape(world, slots, 64)
        gather_ok = all(np.array_equal(g[r], np.frombuffer(everyone[r], np.uint8).reshape(slots, 64))
                        for r in range(world))
        out_set = acs.assemble_output_set(g, total, world)
        gather_ok = gather_ok and [o["instance"] for o in out_set] == list(range(total))
        gather_ok = rdz.all(gather_ok)
    # oracle sample: evenly spaced global ids, each checked by its owner
    sample_ok, checked = True, 0
    if args.oracle_samples > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import rbc_ref
        ids = sorted(set(np.linspace(0, total - 1, min(args.oracle_samples, total)).astype(int).tolist()))
        for g_id in ids:
            if not (first <= g_id < first + I):
                continue
            i = g_id - first
            value = synth.row(SEED, g_id, vpitch, B)
            _, root, _, leaves = rbc_ref.encode_commit(n, f, value)
            dig = rbc_ref.sha256(np.ascontiguousarray(leaves[:k]).tobytes())
            sample_ok = sample_ok and bytes(roots[i]) == root and bytes(digests[i]) == dig and status[i] == 0
            checked += 1
        sample_ok = rdz.all(sample_ok)
        checked = rdz.sum(checked)
    return {"decoded_ok": n_ok, "values_ok": values_ok, "value_mismatch_chunks": mism, "gather_ok": gather_ok,
            "oracle_sample_ok": sample_ok, "oracle_samples_checked": checked}


def cpu_baseline(args, host):
    """The C restatement (oracle/librbc_ref.so: AVX2 split-nibble GF +
    SHA-NI) running the same per-instance pipeline on this box's host cores,
    on bounded samples: the bench config (~6 GB of shard output) and, more
    briefly, every other config."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rbc_ref

    threads = host["usable_cores"]
    feats = rbc_ref.lib().rbcref_cpu_features()

    def run(cfg, target_bytes, nthreads):
        n, f, B, _, _ = CONFIGS[cfg]
        k = n - 2 * f
        S = (B + k - 1) // k
        count = max(nthreads, int(target_bytes // (n * S)))
        rng = np.random.default_rng(7)
        nv = min(count, 64)
        values = rng.integers(0, 256, size=(nv, B), dtype=np.uint8)  # instance i uses values[i % nv]
        present = np.zeros((count, n), dtype=np.uint8)
        corrupt = np.full(count, -1, dtype=np.int32)
        for i in range(count):
            pres = rng.permutation(n)[: n - f]
            present[i, pres] = 1
            if rng.random() < 0.10:
                corrupt[i] = int(rng.choice(pres))
        secs, st, es, ds = rbc_ref.pipeline(n, f, count, B, nthreads, values, present, corrupt, phases=True)
        return {"value": round(count * n * S / secs / 1e9, 3), "unit": "GB/s",
                "phases": {"encode_commit": round(count * n * S / (es / nthreads) / 1e9, 3),
                           "verify_decode": round(count * k * S / (ds / nthreads) / 1e9, 3)},
                "sample": f"{count} instances x {B} B (N={n} f={f}), {secs:.2f} s wall on {nthreads} threads",
                "status_sum": st}

    main_cfg = args.config
    res = run(main_cfg, 6e9, threads)
    single = run(main_cfg, 6e9 / 16, 1)
    per_config, per_config_1 = {}, {}
    for cfg in [c.strip() for c in args.cpu_configs.split(",") if c.strip() in CONFIGS]:
        per_config[cfg] = res if cfg == main_cfg else run(cfg, 1.5e9, threads)
        # one core too (BASELINE.md's CPU table: 1 core and all cores per config)
        per_config_1[cfg] = single if cfg == main_cfg else run(cfg, 1.5e9 / 16, 1)
    return {"value": res["value"], "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": res["sample"] + "; same per-instance pipeline as the GPU step (verified leaves reused)",
            "phases": res["phases"],
            "single_core": {"value": single["value"], "unit": "GB/s", "cores": 1, "phases": single["phases"],
                            "sample": single["sample"]},
            "per_config": {c: {"value": r["value"], "phases": r["phases"], "sample": r["sample"],
                               "single_core": {"value": per_config_1[c]["value"],
                                               "phases": per_config_1[c]["phases"]}}
                           for c, r in per_config.items()},
            "host": host, "simd": ("avx2 " if feats & 1 else "") + ("sha-ni" if feats & 2 else ""),
            "status_sum": res["status_sum"] + single["status_sum"] +
            sum(r["status_sum"] for r in per_config.values()) +
            sum(r["status_sum"] for c, r in per_config_1.items() if c != main_cfg)}


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
