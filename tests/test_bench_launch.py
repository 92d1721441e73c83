"""The N-rank launch of bench.py, without a GPU: `python bench.py --gpus N`
without WORLD_SIZE spawns N ranks with the torch.distributed.run environment
before touching any GPU (cleisthenes_amd.launch.spawn_ranks), they rendezvous
over loopback TCP (no torch), and the first failing rank's status is the
launcher's exit status.  A rank that dies or hangs mid-run ends the whole job
within its deadline, and the surviving ranks name the stage they were in
(cleisthenes_amd.launch.Watchdog) -- the first multi-rank run on the 8-GPU
node must fail loudly, not hang."""
import json
import os
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cleisthenes_amd import launch  # noqa: E402


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(f"""
        import json, os, signal, sys, time
        sys.path.insert(0, {ROOT!r})
        from cleisthenes_amd.launch import Watchdog
        from cleisthenes_amd.rendezvous import Rendezvous
        world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
        assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["MASTER_ADDR"] == "127.0.0.1"
        rdz = Rendezvous(world, rank)
        out = sys.argv[1]
    """) + textwrap.dedent(body))
    return str(p)


def _launcher(tmp_path, script, n, extra_env=None):
    """Run spawn_ranks in a child process so the ranks' stderr is captured."""
    p = tmp_path / "launch.py"
    p.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        from cleisthenes_amd.launch import spawn_ranks
        sys.exit(spawn_ranks({n}, [{str(tmp_path)!r}], {script!r}, grace_s=3))
    """))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(p)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, **(extra_env or {})))
    # the ranks share the stderr pipe: a report (one atomic write) may land
    # inside another rank's traceback line, so decode from each occurrence
    dec, reports, pos = json.JSONDecoder(), [], 0
    while (pos := r.stderr.find('{"watchdog"', pos)) >= 0:
        obj, end = dec.raw_decode(r.stderr, pos)
        reports.append(obj)
        pos = end
    return r.returncode, time.monotonic() - t0, reports, r.stderr


def test_spawn_ranks_rendezvous_and_exit_status(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    script = _script(tmp_path, """
        ranks = rdz.allgather(rank)
        t = rdz.max(0.5 * rank)
        with open(os.path.join(out, "out", f"r{rank}.json"), "w") as f:
            json.dump({"ranks": ranks, "max": t, "world": world, "torch": "torch" in sys.modules}, f)
        rdz.barrier()
    """)
    assert launch.spawn_ranks(3, [str(tmp_path)], script) == 0
    res = [json.load(open(out / f"r{r}.json")) for r in range(3)]
    assert all(x == {"ranks": [0, 1, 2], "max": 1.0, "world": 3, "torch": False} for x in res)


def test_spawn_ranks_propagates_failure(tmp_path):
    script = _script(tmp_path, """
        if rank == 1:
            sys.exit(7)
        rdz.barrier()  # rank 0's peer is gone: it fails too, or the launcher terminates it
    """)
    assert launch.spawn_ranks(2, [str(tmp_path)], script) != 0


def test_killed_rank_ends_the_job_and_the_others_name_their_stage(tmp_path):
    """One rank is SIGKILLed in the middle of the timed loop: the job exits
    non-zero well within the deadline, and every surviving rank reports the
    stage it was in (its rendezvous peer vanished, or the launcher terminated
    it)."""
    script = _script(tmp_path, """
        wd = Watchdog(rank, world)
        with wd.stage("timed loop", 60):
            for it in range(50):
                if rank == 1 and it == 3:
                    os.kill(os.getpid(), signal.SIGKILL)
                rdz.barrier()
                time.sleep(0.05)
    """)
    rc, secs, reports, err = _launcher(tmp_path, script, 3)
    assert rc != 0 and secs < 40, (rc, secs, err[-2000:])
    survivors = {r["rank"] for r in reports}
    assert survivors == {0, 2}, err[-2000:]
    assert all(r["stage"] == "timed loop" for r in reports)


def test_hung_rank_hits_the_rendezvous_deadline(tmp_path):
    """A rank that stops answering (alive, but stuck) makes its peers'
    collective time out after RBC_RDZV_TIMEOUT seconds instead of hanging; the
    launcher then terminates the stuck rank, whose watchdog thread still
    reports its stage although its main thread never returns to Python."""
    script = _script(tmp_path, """
        import ctypes
        wd = Watchdog(rank, world)
        with wd.stage("timed loop", 60):
            rdz.barrier()
            if rank == 1:
                wd.enter("stuck in a device call", 60)
                ctypes.CDLL(None).sleep(100)  # a C call that never yields to the interpreter
            rdz.barrier()
    """)
    rc, secs, reports, err = _launcher(tmp_path, script, 2, {"RBC_RDZV_TIMEOUT": "3"})
    assert rc != 0 and secs < 40, (rc, secs, err[-2000:])
    by_rank = {r["rank"]: r for r in reports}
    assert by_rank[0]["stage"] == "timed loop" and "TimeoutError" in by_rank[0]["watchdog"], err[-2000:]
    assert by_rank[1]["stage"] == "stuck in a device call" and "terminated" in by_rank[1]["watchdog"]


def test_stage_deadline_exits_with_a_report(tmp_path):
    script = _script(tmp_path, """
        import ctypes
        wd = Watchdog(rank, world)
        wd.info["pci_bus_id"] = "0000:00:00.0"
        wd.enter("rccl init", 1.0)
        ctypes.CDLL(None).sleep(30)
    """)
    rc, secs, reports, err = _launcher(tmp_path, script, 1)
    assert rc == launch.EXIT_DEADLINE and secs < 20, (rc, secs, err[-2000:])
    assert reports[0]["stage"] == "rccl init" and reports[0]["pci_bus_id"] == "0000:00:00.0"


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


def test_hbm_plan_divides_free_memory_by_the_ranks_sharing_the_device():
    """C3 with 8,192 instances: the pipelined plan (3 shard sets) does not fit
    one 288 GB GPU and the serial one does; rehearsed as 2 ranks on one
    device, each rank plans with half the free memory."""
    import bench
    n, f, B = 128, 42, 4 << 20
    k = n - 2 * f
    S = (B + k - 1) // k
    sp, vp, op = bench.round_up(S, 128), bench.round_up(k * S + 32, 64), bench.round_up(k * S, 16)
    free = 280e9
    plan, need = bench.hbm_plan(8192, n, 7, sp, vp, op, False, 0, free, 1, 0)
    assert need["pipelined"] > plan["budget_bytes"] >= need["serial"]
    plan2, need2 = bench.hbm_plan(4096, n, 7, sp, vp, op, False, 0, free, 2, 0)
    assert plan2["budget_bytes"] == int(free / 2 * 0.97) and need2["serial"] <= plan2["budget_bytes"]
    assert 2 * need2["serial"] <= free
    # the row view needs no value buffer: the joined form costs k*S more per instance
    _, need3 = bench.hbm_plan(8192, n, 7, sp, vp, op, True, 0, free, 1, 0)
    assert need3["serial"] - need["serial"] == 8192 * op


def test_rank_timing_keys_for_a_three_rank_rehearsal(tmp_path):
    """bench.rank_timing over 3 ranks: every rank's record carries its own
    elapsed time, ms per step and stage spans, and the line's skew names the
    slowest and the fastest rank (what a multi-GPU SCALE run is diagnosed by)."""
    script = _script(tmp_path, """
        import bench
        me = {"rank": rank, "device": rank, "pci_bus_id": f"0000:{rank:02x}:00.0"}
        stage = {"enc": 1.0 + rank, "leaf": 2.0}
        ranks, skew = bench.rank_timing(rdz, me, 0.5 + 0.25 * rank, 10, stage)
        with open(os.path.join(out, f"r{rank}.json"), "w") as f:
            json.dump({"ranks": ranks, "skew": skew}, f)
        rdz.close()
    """)
    assert launch.spawn_ranks(3, [str(tmp_path)], script) == 0
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(3)]
    for x in res:
        assert x == res[0]
        for r, rec in enumerate(x["ranks"]):
            assert rec["rank"] == r and rec["device"] == r
            assert rec["elapsed_s"] == 0.5 + 0.25 * r
            assert rec["ms_per_step"] == round((0.5 + 0.25 * r) * 100.0, 4)
            assert rec["stage_ms"] == {"enc": 1.0 + r, "leaf": 2.0}
        assert x["skew"] == {"elapsed_min_s": 0.5, "elapsed_max_s": 1.0, "slowest_rank": 2, "fastest_rank": 0,
                             "max_over_min": 2.0}


class _Ctx:
    """What bench.report reads of a Context, without a GPU."""
    codec = "fft"

    def __init__(self, form):
        self._form = form

    def verify_form(self, S):
        return self._form


def _report(config, pipe=True):
    import argparse
    import numpy as np
    import bench
    n, f, B, I, _ = bench.CONFIGS[config]
    k, d = n - 2 * f, max(1, (n - 1).bit_length())
    S = (B + k - 1) // k
    rng = np.random.default_rng(0)
    present = np.zeros((I, n), np.uint8)
    corrupt = np.full(I, -1, np.int32)
    for i in range(I):
        present[i, rng.permutation(n)[: n - f]] = 1
        if rng.random() < 0.1:
            corrupt[i] = int(rng.choice(np.flatnonzero(present[i])))
    stage = {"enc": 2.5, "leaf": 2.9, "tree": 0.13, "fault": 0.03, "verify": 3.1, "verify_rows": 2.95,
             "verify_path": 1.8 if config == "c4" else 0.005, "check": 0.06, "decode": 2.6, "interp": 2.7,
             "gather": 0.005}
    if not pipe:
        stage = {kk: v for kk, v in stage.items() if kk not in ("verify_rows", "verify_path", "check", "decode")}
    args = argparse.Namespace(config=config, join=False, steps=10)
    form = "shared_path" if config == "c4" else "walk"
    return bench.report(args, _Ctx(form), I, n, k, d, S, present, corrupt, stage, None, 10 * 5.9e-3)


def test_report_attributes_each_verify_launch_to_its_own_kernel():
    """at C4 the receive step's verify span holds two
    launches; the line gives each its own roofline entry with its own
    algorithmic bytes, and where the committed PMC file of the config has the
    kernel, traffic covers the algorithmic bytes (tests/test_profiles.py
    checks the same on the committed bench lines)."""
    out = _report("c4")
    rv, rp = out["roofline_verify"], out["roofline_verify_path"]
    assert rv["kernel"] == "sha_rx_kernel<leaves+regen>" and rp["kernel"] == "merkle_path_kernel<4>"
    assert rv["avg_ms"] == 2.95 and rp["avg_ms"] == 1.8
    for r in (rv, rp, out["roofline_encode"], out["roofline_decode"]):
        if r["traffic"] is not None:
            assert r["traffic"] >= 0.98 * r["algorithmic_bytes_per_launch"], (r["kernel"], r["traffic"])
    c2 = _report("c2")
    assert c2["roofline_verify"]["kernel"] == "sha_rx_kernel<verify+regen>" and c2["roofline_verify_path"] is None
    serial = _report("c4", pipe=False)
    assert "verify: sha_rows_kernel<leaves> + merkle_path_kernel<4>" == serial["roofline"]["kernel"] or \
        serial["roofline"]["kernel"] in ("sha_rows_kernel<leaves>", "rs_fft_kernel<encode>")


def test_report_prices_the_step_per_opcode_not_at_four_clocks():
    """valu_step prices every kernel's PMC VALU count from its static ISA mix
    (tools/isa_mix.py, profiles/isa_mix_r05.json) and, for the SHA-256
    kernels, at the probe's dependency-limited rate; no 4-clock figure."""
    out = _report("c2")
    v = out["valu_step"]
    assert v is not None and "busy_4clk" not in v
    assert 0 < v["issue_priced_ms"] < v["chain_priced_ms"]
    assert not v["unpriced_kernels"], v["unpriced_kernels"]
    assert "priced" in out["roofline_verify"]["valu"] and "measured" not in out["roofline_verify"]["valu"]


def test_host_fed_aggregate_over_ranks():
    """the host-fed epoch runs on every rank at once; the
    job figure is every rank's committed shard bytes over the slowest rank's
    seconds, never a sum of per-rank rates, and one failing rank fails it."""
    import bench
    n, S = 128, 23832
    per = [{"GBps": round(1024 * n * S / t / 1e9, 3), "seconds": t, "instances": 1024, "ok": True}
           for t in (0.20, 0.25, 0.40, 0.22)]
    agg = bench.host_fed_aggregate(per, n, S)
    assert agg["ranks"] == 4 and agg["slowest_rank"] == 2
    assert agg["aggregate_GBps"] == round(4 * 1024 * n * S / 0.40 / 1e9, 3)
    assert agg["aggregate_GBps"] < sum(agg["per_rank_GBps"])
    assert agg["min_over_max"] == round(min(agg["per_rank_GBps"]) / max(agg["per_rank_GBps"]), 4)
    assert agg["ok"] and agg["rank0"] is per[0]
    per[3]["ok"] = False
    assert not bench.host_fed_aggregate(per, n, S)["ok"]


def test_value_form_defaults_to_the_joined_value():
    """`value` is timed on the joined form interpolate
    returns (rbc/rbc.go:88); --row-view selects the row view."""
    import bench
    assert bench.parse_args([]).join is True
    assert bench.parse_args(["--row-view"]).join is False
    assert bench.parse_args(["--no-joined-leg"]).no_second_form is True


def test_profile_files_are_taken_newest_run_first():
    """The bench takes PMC traffic and clock files from the newest run of a
    round: runs are lettered a..z, then aa, ab, ... (r06ae after r06h)."""
    import bench
    names = ["pmc_traffic_r06h_c2.json", "pmc_traffic_r06ae_c2.json", "pmc_traffic_r05b_c2.json",
             "pmc_traffic_r06z_c2.json", "pmc_traffic_r06_c2.json", "pmc_traffic_r10a_c2.json"]
    got = sorted(names, key=bench._run_key, reverse=True)
    assert got == ["pmc_traffic_r10a_c2.json", "pmc_traffic_r06ae_c2.json", "pmc_traffic_r06z_c2.json",
                   "pmc_traffic_r06h_c2.json", "pmc_traffic_r06_c2.json", "pmc_traffic_r05b_c2.json"]
