"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path:
instances partitioned per rank in contiguous (ragged) blocks with no
data-path collective, one all-gather of max_share padded {root, digest}
records (a failed instance carries a zero digest), ACS output-set assembly
through the C ABI (rbc_acs_assemble) -- checked against a single-process
computation.  The per-rank compute stands in with the CPU oracle here; on
GPUs bench.py runs the same partition with librbc_gpu.so and the RCCL
all-gather (rbc_dev_allgather_records, tests/test_gpu_rccl.py)."""
import os
import socket

import multiprocessing as mp

import numpy as np

# torch is imported inside the workers only: a pytest process that imported
# it would map torch's bundled libamdhip64 / librccl, and librbc_gpu.so
# (linked against /opt/rocm) would then bind to those in every GPU test of
# the same session (tests/test_gpu_rccl.py checks which runtime is mapped).


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _records(first, count, n, f, B):
    import rbc_ref
    roots, digs, status = [], [], []
    for i in range(first, first + count):
        rng = np.random.default_rng(1000 + i)
        value = rng.integers(0, 256, B, dtype=np.uint8)
        shards, root, br, leaves = rbc_ref.encode_commit(n, f, value)
        valid = np.zeros(n, dtype=np.uint8)
        valid[rng.permutation(n)[: n - f]] = 1
        if i % 4 == 3:  # a wrong committed root: interpolate fails, no output for i
            root = bytes(32 * [7])
        rc, v, dg = rbc_ref.interpolate(n, f, shards, valid, root)
        roots.append(np.frombuffer(root, np.uint8))
        digs.append(np.frombuffer(dg, np.uint8))
        status.append(rc)
    return np.array(roots).reshape(-1, 32), np.array(digs).reshape(-1, 32), status


def _worker(rank, world, port, total, out_q):
    import sys

    import torch
    import torch.distributed as dist
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root_dir, os.path.join(root_dir, "oracle")]
    from cleisthenes_amd import acs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, f, B = 16, 5, 777
    first, count = acs.partition(total, world, rank)
    roots, digs, status = _records(first, count, n, f, B)
    slots = acs.max_share(total, world)
    mine = torch.from_numpy(acs.pack_records(roots, digs, slots, status))
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    out = acs.assemble_output_set(torch.stack(gathered).numpy(), total, world)
    if rank == 0:
        out_q.put([(o["instance"], o["root"], o["digest"]) for o in out])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_partition_and_allgather():
    total = 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    roots, digs, status = _records(0, total, 16, 5, 777)
    want = [(i, bytes(roots[i]), bytes(digs[i])) for i in range(total) if status[i] == 0]
    assert got == want and len(want) == total - total // 4
