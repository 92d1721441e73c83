"""bench.py end to end on the GPU.  Every run must pass the bench's own
correctness guard (all instances decode, every decoded value equals its
input, sampled roots / digests equal the C oracle, gathered records equal
what each rank holds; the bench exits 3 otherwise) and print exactly one JSON
line with the contract keys.  Covered: both schedules (0 serial, 7 the
two-stream default) in both value forms, BASELINE configs[3] at its stated
size (C3, 8,192 x 4 MiB) on one GPU and partitioned over two ranks, C4 at
SURVEY section 8d's 16,384 instances, the 1-rank RCCL gather, the 3-rank
ragged rehearsal and the HBM-plan fallback."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUICK = ["--no-cpu-baseline", "--no-pcie", "--oracle-samples", "4"]


def _run(args, timeout=300, env=None):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("pipeline,join", [(0, False), (7, False), (7, True)])
def test_bench_schedules_pass_their_guard(pipeline, join):
    d = _run(["--steps", "3", "--warmup", "3", "--instances", "96", "--pipeline", str(pipeline)]
             + ([] if join else ["--row-view"]) + QUICK)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "ranks"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0
    assert d["decoded_ok"] == 96 and d["values_ok"] and d["oracle_sample_ok"] and d["oracle_samples_checked"] == 4
    g = d["guard"]  # the last timed batch AND a poisoned receive both decode every instance to its input
    assert g["timed_batch"] == {"decoded": 96, "value_mismatch_chunks": 0}
    assert g["poisoned_batch"]["decoded"] == 96 and g["poisoned_batch"]["value_mismatch_chunks"] == 0
    assert d["library"] == os.path.realpath(os.path.join(ROOT, "cleisthenes_amd", "librbc_gpu.so"))
    assert d["rank_skew"]["slowest_rank"] == 0 and d["ranks"][0]["ms_per_step"] > 0
    assert 0 < d["roofline"]["frac"] < 1 and d["roofline"]["avg_ms"] > 0
    assert d["config"]["hbm_plan"]["schedule"] == ("pipelined" if pipeline else "serial")
    assert d["config"]["value_form"].startswith("joined" if join else "row view")
    if pipeline:
        rd = d["roofline_decode"]
        assert rd["avg_ms"] > 0 and 0 < rd["frac"] < 1 and rd["algorithmic_bytes_per_launch"] > 0
        # C2 walks the branches inside the row hashing: one launch, no shared-path span
        assert d["roofline_verify"]["kernel"] == "sha_rx_kernel<verify+regen>" and d["roofline_verify_path"] is None


def test_bench_c3_8192_instances_on_one_gpu():
    """BASELINE configs[3] at its stated size on one GPU: 8,192 x 4 MiB.  The
    HBM plan (free device memory) cannot hold the pipeline's three shard sets
    and runs the serial schedule; every instance decodes."""
    d = _run(["--config", "c3", "--total-instances", "8192", "--steps", "2", "--warmup", "1"] + QUICK, timeout=600)
    assert d["decoded_ok"] == 8192 and d["values_ok"] and d["oracle_sample_ok"] and d["oracle_samples_checked"] == 4
    plan = d["config"]["hbm_plan"]
    assert plan["schedule"] == "serial" and plan["ranks_sharing_device"] == 1
    assert plan["need_bytes"]["pipelined"] > plan["budget_bytes"] >= plan["need_bytes"]["serial"]
    assert d["config"]["instances_total"] == 8192 and d["scaling"] == "strong"


def test_bench_c3_8192_partitioned_over_two_ranks():
    """configs[3]'s partition: 8,192 instances over 2 ranks (4,096 each),
    rehearsed on this one GPU -- both ranks plan with half the free memory,
    and the records of every rank are checked through the rendezvous."""
    d = _run(["--config", "c3", "--total-instances", "8192", "--gpus", "2", "--rehearse-on-one-gpu", "--steps", "2",
              "--warmup", "1", "--no-isolated"] + QUICK, timeout=900)
    assert d["n_gpus"] == 2 and d["config"]["instances_per_gpu"] == 4096
    assert d["decoded_ok"] == 8192 and d["values_ok"] and d["gather_ok"] and d["oracle_sample_ok"]
    assert d["config"]["hbm_plan"]["ranks_sharing_device"] == 2
    assert [r["rank"] for r in d["ranks"]] == [0, 1] and all(r["pci_bus_id"] for r in d["ranks"])


def test_bench_c4_16384_instances():
    """C4 (N=256, f=85, 64 KiB) at SURVEY section 8d's 16,384 instances:
    every instance decodes to its input under the default schedule."""
    d = _run(["--config", "c4", "--steps", "3", "--warmup", "3", "--no-isolated"] + QUICK)
    assert d["config"]["instances_per_gpu"] == 16384
    assert d["decoded_ok"] == 16384 and d["values_ok"] and d["value_mismatch_chunks"] == 0 and d["oracle_sample_ok"]
    # C4 verifies with the shared path: the row hashing and merkle_path_kernel each have their own span
    rv, rp = d["roofline_verify"], d["roofline_verify_path"]
    assert rv["kernel"] == "sha_rx_kernel<leaves+regen>" and rp["kernel"] == "merkle_path_kernel<4>"
    sm = d["stage_ms"]
    assert sm["verify_rows"] > 0 and sm["verify_path"] > 0 and sm["verify_rows"] + sm["verify_path"] <= sm["verify"]


def test_bench_multi_rank_rehearsal_ragged_strong_scaling():
    """The N-rank path on this one GPU: bench.py spawns 3 ranks itself (all on
    device 0, no RCCL), partitions 250 instances 83/83/84, and the guard checks
    every rank's decodes, values, gathered records (through the torch-free
    rendezvous) and oracle samples; the line reports the whole job."""
    d = _run(["--gpus", "3", "--rehearse-on-one-gpu", "--total-instances", "250", "--steps", "3", "--warmup", "3",
              "--no-isolated"] + QUICK)
    assert d["n_gpus"] == 3 and d["scaling"] == "strong"
    assert d["config"]["instances_total"] == 250 and "rehearsal" in d["config"]
    assert d["decoded_ok"] == 250 and d["values_ok"] and d["gather_ok"] and d["oracle_sample_ok"]
    assert [r["rank"] for r in d["ranks"]] == [0, 1, 2]


def test_bench_eight_rank_rehearsal():
    """The driver's first 8-GPU run, rehearsed on this one GPU (VERDICT r04
    item 5): bench.py spawns 8 ranks itself, all on device 0 with no RCCL, and
    partitions 1,000 instances 125 apiece.  Exercised: the self-spawn, the
    world-size-8 rendezvous, the per-stage watchdog, the HBM plan with 8 ranks
    sharing the device, the ragged-capable partition, the guard over every
    rank (decodes, values, gathered records through the rendezvous, oracle
    samples) and the 8-entry ranks / rank_skew keys.  Not a multi-GPU
    measurement: RCCL at nranks > 1 needs the driver's 8-GPU node."""
    d = _run(["--gpus", "8", "--rehearse-on-one-gpu", "--total-instances", "1000", "--steps", "3", "--warmup", "3",
              "--no-isolated", "--no-joined-leg"] + QUICK, timeout=600)
    assert d["n_gpus"] == 8 and d["scaling"] == "strong" and "rehearsal" in d["config"]
    assert d["config"]["instances_total"] == 1000 and d["config"]["instances_per_gpu"] == 125
    assert d["decoded_ok"] == 1000 and d["values_ok"] and d["gather_ok"] and d["oracle_sample_ok"]
    assert [r["rank"] for r in d["ranks"]] == list(range(8)) and all(r["ms_per_step"] > 0 for r in d["ranks"])
    assert d["config"]["hbm_plan"]["ranks_sharing_device"] == 8
    sk = d["rank_skew"]
    assert sk["slowest_rank"] in range(8) and sk["fastest_rank"] in range(8) and sk["max_over_min"] >= 1.0


def test_bench_one_rank_rccl_gather():
    """--force-gather runs the RCCL record all-gather in the timed step on one
    rank: the line names the ROCm 7.2 RCCL that was mapped and the guard
    checks the gathered records against the device results."""
    d = _run(["--force-gather", "--instances", "64", "--steps", "3", "--warmup", "3", "--no-isolated"] + QUICK)
    assert d["rccl"] is not None and d["rccl"]["nranks"] == 1 and d["ranks"][0]["rccl_nranks"] == 1
    assert "torch" not in d["rccl"]["lib"]
    assert d["decoded_ok"] == 64 and d["values_ok"] and d["gather_ok"]


def test_bench_falls_back_to_serial_when_the_shard_sets_do_not_fit():
    """With an HBM budget below the pipeline's three shard sets the default
    schedule falls back to the serial one and still passes its guard."""
    d = _run(["--instances", "64", "--steps", "3", "--warmup", "2", "--hbm-budget", "1.5e9"] + QUICK)
    assert d["config"]["pipeline"] == "serial" and d["config"]["hbm_plan"]["schedule"] == "serial"
    assert d["decoded_ok"] == 64 and d["values_ok"] and d["oracle_sample_ok"]


def _host_fed_ok(h, n, S):
    assert h["ok"] and h["checks"]["verdict_mismatches"] == 0 and h["checks"]["values_ok"] and h["checks"]["roots_ok"]
    assert h["checks"]["decoded"] == h["instances"] and h["echo_messages"] == h["instances"] * (n - 42)
    assert h["GBps"] > 0 and h["pcie_GBps"]["h2d"] > 0 and h["pcie_GBps"]["d2h"] > 0


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_host_fed_leg_on_every_rank(gpus):
    """the host-fed epoch (rbc_shard_commit ||
    rbc_validate_packed_leaves of every received ECHO -> rbc_interpolate_batch_verified,
    pinned host memory both ways) runs on EVERY rank at once -- here 1 rank and
    2 ranks rehearsed on this GPU -- and every rank's verdicts (10 % of the
    instances carry a corrupted ECHO), values and proposer roots are checked;
    each rank's record carries its own rate and the line the job aggregate."""
    extra = ["--gpus", "2", "--rehearse-on-one-gpu"] if gpus == 2 else []
    d = _run(["--instances", "256", "--steps", "3", "--warmup", "3", "--no-isolated", "--no-cpu-baseline",
              "--oracle-samples", "4", "--host-instances", "256"] + extra, timeout=600)
    p = d["pcie_inclusive"]
    n, S = 128, d["config"]["shard_bytes"]
    assert p["ok"] and p["ranks"] == gpus and len(p["per_rank_GBps"]) == gpus
    _host_fed_ok(p["rank0"], n, S)
    assert p["rank0"]["alone_GBps"]["validate+interpolate"] > 0
    assert p["kept"]["ok"] and p["kept"]["aggregate_GBps"] > 0 and p["rank0"]["kept"]["checks"]["values_ok"]
    for r in d["ranks"]:
        assert r["host_fed"]["ok"] and r["host_fed"]["instances"] == 256 and r["host_fed"]["GBps"] > 0
    assert p["aggregate_GBps"] <= sum(p["per_rank_GBps"]) * 1.001


MUTANT = os.path.join(ROOT, "tests", "mutants", "librbc_gpu_skip_regen.so")


@pytest.mark.parametrize("config,join", [("c2", False), ("c4", False), ("c2", True)])
def test_bench_guard_fails_a_build_that_never_regenerates(config, join):
    """The guard must not pass a no-op regeneration.  tests/mutants'
    librbc_gpu_skip_regen.so is the product with gf_regen_kernel never
    launched: the timed batches still hold the proposer's intact rows in the
    absent slots and pass, but the poisoned receive cannot, so bench.py exits
    3 with values_ok and decoded_ok false -- and names the mutant it mapped."""
    assert os.path.exists(MUTANT), "build() makes tests/mutants"
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", config, "--instances", "64", "--steps", "3",
            "--warmup", "3", "--no-isolated"] + QUICK + ([] if join else ["--row-view"])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=dict(os.environ, RBC_GPU_LIB=MUTANT))
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    err = [ln for ln in r.stderr.splitlines() if ln.startswith('{"error"')]
    assert len(err) == 1, r.stderr[-3000:]
    e = json.loads(err[0])
    timed, poisoned = e["guard"]["timed_batch"], e["guard"]["poisoned_batch"]
    # the timed batches' absent rows still hold the proposer's bytes: only the ~10 % of instances whose
    # corrupted ECHO is a data row can fail there; with every such row poisoned, (nearly) every one does
    assert timed["decoded"] >= 64 * 0.7, timed
    assert poisoned["decoded"] <= 64 * 0.1 and poisoned["value_mismatch_chunks"] > 10 * max(1, timed["value_mismatch_chunks"])
    assert not e["values_ok"] and e["decoded_ok"] <= poisoned["decoded"] and e["library"] == os.path.realpath(MUTANT)
