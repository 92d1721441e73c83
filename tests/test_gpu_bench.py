"""bench.py end to end on the GPU at a small batch: every schedule
(--pipeline 0 serial, 1 two-stream, 2 three-stream, 3 phase-aligned,
4 split verify, 5 balanced, 6 commit from the receiver's decode, 7 two-stream with
rbc_dev_receive_step, the default) must pass the bench's own correctness guard (all instances decode, every
decoded value equals its input, sampled roots / digests equal the C oracle;
the bench exits 3 otherwise) and print exactly one JSON line with the
contract keys."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("pipeline", [0, 1, 2, 3, 4, 5, 6, 7])
def test_bench_schedules_pass_their_guard(pipeline):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "3", "--instances", "96",
           "--pipeline", str(pipeline), "--no-cpu-baseline", "--no-pcie", "--oracle-samples", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0
    assert d["decoded_ok"] == 96 and d["values_ok"] and d["oracle_sample_ok"] and d["oracle_samples_checked"] == 4
    assert 0 < d["roofline"]["frac"] < 1 and d["roofline"]["avg_ms"] > 0


def _run(args, timeout=300, env=None):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_multi_rank_rehearsal_ragged_strong_scaling():
    """The N-rank path on this one GPU: bench.py spawns 3 ranks itself (all on
    device 0, no RCCL), partitions 250 instances 83/83/84, and the guard checks
    every rank's decodes, values, gathered records (through the torch-free
    rendezvous) and oracle samples; the line reports the whole job."""
    d = _run(["--gpus", "3", "--rehearse-on-one-gpu", "--total-instances", "250", "--steps", "3", "--warmup", "3",
              "--no-cpu-baseline", "--no-pcie", "--no-isolated", "--oracle-samples", "4"])
    assert d["n_gpus"] == 3 and d["scaling"] == "strong"
    assert d["config"]["instances_total"] == 250 and "rehearsal" in d["config"]
    assert d["decoded_ok"] == 250 and d["values_ok"] and d["gather_ok"] and d["oracle_sample_ok"]


def test_bench_one_rank_rccl_gather():
    """--force-gather runs the RCCL record all-gather in the timed step on one
    rank: the line names the ROCm 7.2 RCCL that was mapped and the guard
    checks the gathered records against the device results."""
    d = _run(["--force-gather", "--instances", "64", "--steps", "3", "--warmup", "3", "--no-cpu-baseline",
              "--no-pcie", "--no-isolated", "--oracle-samples", "4"])
    assert d["rccl"] is not None and d["rccl"]["nranks"] == 1
    assert "torch" not in d["rccl"]["lib"]
    assert d["decoded_ok"] == 64 and d["values_ok"] and d["gather_ok"]


def test_bench_falls_back_to_serial_when_the_shard_sets_do_not_fit():
    """C3 with all 8,192 instances on one GPU cannot hold the pipeline's shard
    sets: with an HBM budget below one set the default schedule must fall back
    to the serial one and still pass its guard."""
    env = dict(os.environ, RBC_BENCH_HBM_BUDGET="1e6")
    d = _run(["--instances", "64", "--steps", "3", "--warmup", "2", "--no-cpu-baseline", "--no-pcie",
              "--oracle-samples", "4"], env=env)
    assert d["config"]["pipeline"] == "serial"
    assert d["decoded_ok"] == 64 and d["values_ok"] and d["oracle_sample_ok"]
