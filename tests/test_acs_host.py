"""Host side of the multi-GPU step, no GPU needed:
the ACS partition / record packing / output-set assembly of the C ABI
(rbc_acs_*) against a plain-Python restatement, the synthetic-input
restatement (cleisthenes_amd.synth) against splitmix64's published first
output, and the torch-free rendezvous bench.py coordinates ranks with."""
import multiprocessing as mp
import os

import numpy as np
import pytest


def py_partition(total, world, rank):
    return rank * total // world, (rank + 1) * total // world - rank * total // world


def py_assemble(gathered, total, world):
    """Plain restatement: contiguous shares, a zero digest = not in the set."""
    out = []
    for r in range(world):
        first, cnt = py_partition(total, world, r)
        for t in range(cnt):
            rec = gathered[r, t]
            if rec[32:].any():
                out.append((first + t, bytes(rec[:32]), bytes(rec[32:])))
    return out


@pytest.mark.parametrize("total,world", [(1, 1), (9, 2), (10, 3), (8192, 8), (8193, 8), (5, 8), (1000, 7)])
def test_assemble_matches_restatement_on_ragged_shares(total, world):
    from cleisthenes_amd import acs
    rng = np.random.default_rng(total * 31 + world)
    slots = acs.max_share(total, world)
    assert slots == max(py_partition(total, world, r)[1] for r in range(world))
    gathered = np.zeros((world, slots, 64), dtype=np.uint8)
    status_all = np.where(rng.random(total) < 0.2, -8, 0).astype(np.int32)
    for r in range(world):
        first, cnt = acs.partition(total, world, r)
        assert (first, cnt) == py_partition(total, world, r)
        roots = rng.integers(0, 256, (cnt, 32), dtype=np.uint8)
        digs = rng.integers(1, 256, (cnt, 32), dtype=np.uint8)  # never all-zero
        gathered[r] = acs.pack_records(roots, digs, slots, status_all[first:first + cnt])
        assert not gathered[r, cnt:].any()  # padding past the share is zero
    got = [(o["instance"], o["root"], o["digest"]) for o in acs.assemble_output_set(gathered, total, world)]
    want = py_assemble(gathered, total, world)
    assert got == want
    assert [g[0] for g in got] == [i for i in range(total) if status_all[i] == 0]


def test_assemble_rejects_short_gather_buffer():
    from cleisthenes_amd import acs
    with pytest.raises(ValueError):
        acs.assemble_output_set(np.zeros((2, 4, 64), np.uint8), 10, 2)  # shares of 5 > 4 slots
    with pytest.raises(ValueError):
        acs.partition(10, 2, 2)


def test_synth_restates_splitmix64():
    from cleisthenes_amd import synth
    # splitmix64 seeded with 0: first output = mix(0x9E3779B97F4A7C15)
    # = 0xE220A8397B1DCDAF (the generator's published first value)
    row = synth.row(seed=1, r=0, pitch=16, nbytes=16)
    assert int.from_bytes(row[:8].tobytes(), "little") == 0xE220A8397B1DCDAF
    # rows are disjoint windows of one counter stream: row r word w = counter r*pitch/8 + w
    a = synth.row(7, 3, 64, 64)
    b = synth.row(7, 0, 64 * 4, 64 * 4)  # row 0 of a 4x wider pitch covers rows 0..3 of pitch 64
    assert np.array_equal(a, b[192:256])
    assert len(synth.row(7, 5, 64, 13)) == 13


def _rdz_worker(world, rank, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from cleisthenes_amd.rendezvous import Rendezvous
    rdz = Rendezvous(world, rank)  # key from the shared parent process
    got = {
        "gather": rdz.allgather({"rank": rank, "blob": "x" * (rank * 1000 + 1)}),
        "raw": rdz.allgather_bytes(bytes([rank]) * (rank * 1000 + 1)),
        "bcast": rdz.broadcast_bytes(b"uid-from-rank0" if rank == 0 else None),
        "max": rdz.max(float(rank) * 1.5),
        "sum": rdz.sum(rank + 1),
        "all": rdz.all(rank != 1),
    }
    rdz.barrier()
    rdz.close()
    q.put((rank, got))


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_collectives(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rdz_worker, args=(world, r, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        g = res[r]
        assert [x["rank"] for x in g["gather"]] == list(range(world))
        assert [len(x["blob"]) for x in g["gather"]] == [q_ * 1000 + 1 for q_ in range(world)]
        assert g["raw"] == [bytes([q_]) * (q_ * 1000 + 1) for q_ in range(world)]
        assert g["bcast"] == b"uid-from-rank0"
        assert g["max"] == 1.5 * (world - 1)
        assert g["sum"] == world * (world + 1) // 2
        assert g["all"] is False


def test_rendezvous_single_rank_is_local():
    from cleisthenes_amd.rendezvous import Rendezvous
    rdz = Rendezvous(1, 0)
    assert rdz.allgather(5) == [5] and rdz.max(2.0) == 2.0 and rdz.all(True)
    rdz.barrier()


def _rdz_rank0(key, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from cleisthenes_amd.rendezvous import Rendezvous
    try:
        rdz = Rendezvous(2, 0, key=key, timeout=5, connect_timeout=20)
        q.put(("ok", rdz.allgather_bytes(b"r0")))
    except Exception as e:  # noqa: BLE001
        q.put(("err", repr(e)))


def test_rendezvous_refuses_unauthenticated_peers_and_names_a_vanished_peer(tmp_path):
    """A connection that does not present the launch's secret is dropped (it
    cannot claim a rank); the real rank then joins, and a peer that has
    exited makes the next collective raise at once, naming it."""
    import socket
    import struct
    import time
    import uuid
    from cleisthenes_amd import rendezvous as rv
    key = uuid.uuid4().hex
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rdz_rank0, args=(key, q))
    p.start()
    path = os.path.join(rv.private_dir(), key)
    deadline = time.monotonic() + 60
    while not os.path.exists(path):
        assert time.monotonic() < deadline
        time.sleep(0.05)
    st = os.stat(rv.private_dir())
    assert st.st_mode & 0o077 == 0 and os.stat(path).st_mode & 0o077 == 0
    port = int(open(path).read().split()[0])
    # an impostor: right rank id, wrong secret -> dropped, the rendezvous goes on
    imp = socket.create_connection(("127.0.0.1", port))
    imp.sendall(struct.pack("<i", 1) + b"0" * 64)
    imp.settimeout(5)
    assert imp.recv(1) == b""  # closed by rank 0
    rdz = rv.Rendezvous(2, 1, key=key, timeout=5)
    assert rdz.allgather_bytes(b"r1") == [b"r0", b"r1"]
    assert q.get(timeout=30) == ("ok", [b"r0", b"r1"])
    p.join(timeout=30)
    # rank 0 is gone: the next collective fails at once with a named peer
    with pytest.raises(ConnectionError, match="rank 0"):
        rdz.barrier()


def test_rendezvous_never_unpickles():
    import inspect
    from cleisthenes_amd import rendezvous as rv
    src = inspect.getsource(rv)
    assert "pickle" not in src.replace("nothing is unpickled", "")
