"""The committed bench lines' rooflines follow from the committed profiles
(VERDICT r04, next-round item 1): every roofline entry that carries PMC
`traffic` names a kernel whose HBM bytes per launch are at least the
algorithmic bytes it is credited with (a kernel cannot do the stated work
moving less), its traffic source exists and holds that kernel, and a
profiled per-kernel trace of the same config agrees with the live span the
line divides by.  Lines from round 5 on are checked (earlier rounds' lines
are history; round 4's C4 line is the case that failed this)."""
import glob
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lines():
    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "*.json"))):
        m = re.match(r"r(\d+)", os.path.basename(os.path.dirname(p)))
        if not m or int(m.group(1)) < 5:
            continue
        try:
            j = json.load(open(p))
        except ValueError:
            continue
        if isinstance(j, dict) and j.get("metric") and j.get("roofline"):
            out.append((os.path.relpath(p, ROOT), j))
    return out


LINES = lines()


def entries(j):
    for key in ("roofline", "roofline_encode", "roofline_decode", "roofline_verify", "roofline_verify_path"):
        r = j.get(key)
        if isinstance(r, dict):
            yield key, r


def test_round5_lines_are_committed():
    assert LINES, "no profiles/r05*/ bench lines committed yet"


@pytest.mark.parametrize("path,line", LINES, ids=[p for p, _ in LINES])
def test_traffic_covers_algorithmic_bytes(path, line):
    checked = 0
    for key, r in entries(line):
        if r.get("traffic") is None:
            continue
        ratio = r["traffic"] / r["algorithmic_bytes_per_launch"]
        assert ratio >= 0.98, (path, key, r["kernel"], ratio)
        src = os.path.join(ROOT, r["traffic_source"])
        assert os.path.exists(src), (path, key, src)
        pm = json.load(open(src))["kernels"]
        assert pm[r["kernel"]]["hbm_bytes_per_launch"] == r["traffic"], (path, key)
        checked += 1
    assert checked >= 2, (path, "fewer than two roofline entries carry PMC traffic")


@pytest.mark.parametrize("path,line", LINES, ids=[p for p, _ in LINES])
def test_frac_is_achieved_over_peak(path, line):
    for key, r in entries(line):
        ach = r["algorithmic_bytes_per_launch"] / (r["avg_ms"] / 1e3) / 1e9
        assert abs(ach - r["achieved"]) <= 0.002 * ach + 0.1, (path, key)
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3, (path, key)


def _profiled_pairs():
    """(line, trace roles) pairs: a bench line of a run made under rocprofv3
    and the per-role trace summary of that same run (tools/trace_summary.py)."""
    out = []
    for tr in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "trace_roles.json"))):
        m = re.match(r"r(\d+)", os.path.basename(os.path.dirname(tr)))
        line = os.path.join(os.path.dirname(tr), "prof_default.json")
        if m and int(m.group(1)) >= 5 and os.path.exists(line):
            out.append((os.path.relpath(line, ROOT), json.load(open(line)), json.load(open(tr))["roles"]))
    return out


PAIRS = _profiled_pairs()


def test_a_profiled_round5_run_is_committed():
    assert PAIRS, "no profiles/r05*/prof_default.json + trace_roles.json pair"


@pytest.mark.parametrize("path,line,roles", PAIRS, ids=[p for p, _, _ in PAIRS])
def test_live_span_agrees_with_the_rocprof_average(path, line, roles):
    """The contract's check: the dominant kernel's live span (HIP events in
    bench.py) and rocprofv3's average duration of the same kernel over the
    same timed launches agree -- within 5 % (the event span also holds the
    launch's own enqueue and, under the pipeline, nothing else on its stream)."""
    for key in ("roofline", "roofline_encode"):
        r = line[key]
        tr = roles.get(r["kernel"])
        assert tr and tr["timed_launches"] >= 20, (path, key, r["kernel"])
        assert abs(tr["avg_ms"] - r["avg_ms"]) <= 0.05 * r["avg_ms"], (path, key, tr["avg_ms"], r["avg_ms"])
