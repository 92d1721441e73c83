"""bench.py's own N-rank launch (no GPU): `python bench.py --gpus N` without
WORLD_SIZE spawns N ranks with the torch.distributed.run environment before
touching any GPU, they rendezvous over loopback TCP (no torch), and the first
failing rank's status is the launcher's exit status."""
import os
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(f"""
        import json, os, sys
        sys.path.insert(0, {ROOT!r})
        from cleisthenes_amd.rendezvous import Rendezvous
        world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
        assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["MASTER_ADDR"] == "127.0.0.1"
        rdz = Rendezvous(world, rank)
        out = sys.argv[1]
    """) + textwrap.dedent(body))
    return str(p)


def test_spawn_ranks_rendezvous_and_exit_status(tmp_path):
    import bench
    out = tmp_path / "out"
    out.mkdir()
    script = _script(tmp_path, """
        ranks = rdz.allgather(rank)
        t = rdz.max(0.5 * rank)
        with open(os.path.join(out, f"r{rank}.json"), "w") as f:
            json.dump({"ranks": ranks, "max": t, "world": world, "torch": "torch" in sys.modules}, f)
        rdz.barrier()
    """)
    assert bench.spawn_ranks(3, [str(out)], script=script) == 0
    import json
    res = [json.load(open(out / f"r{r}.json")) for r in range(3)]
    assert all(x == {"ranks": [0, 1, 2], "max": 1.0, "world": 3, "torch": False} for x in res)


def test_spawn_ranks_propagates_failure(tmp_path):
    import bench
    script = _script(tmp_path, """
        if rank == 1:
            sys.exit(7)
        rdz.barrier()  # rank 0 would wait forever: the launcher terminates it
    """)
    rc = bench.spawn_ranks(2, [str(tmp_path)], script=script)
    assert rc != 0  # 7, or rank 0's own failure when its peer vanished first


def test_world_must_match_gpus(tmp_path, monkeypatch):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    try:
        bench.main(["--gpus", "4"])
    except SystemExit as e:
        assert "WORLD_SIZE=2" in str(e)
    else:
        raise AssertionError("bench accepted WORLD_SIZE != --gpus")
