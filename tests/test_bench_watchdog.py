"""bench.py's per-phase watchdog (the N > 1 hang guard): on a stalled phase it prints the JSON line
accumulated so far with an "error" field, dumps every thread's stack and exits non-zero; a run whose
phases all finish prints nothing extra. CPU only (the watchdog is host code)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import sys, time
sys.path.insert(0, {root!r})
import bench
out = {{"metric": "m", "value": 123.0, "nested": {{"a": [1, 2]}}}}
wd = bench.Watchdog(out, rank={rank}, enabled=True, scale=1.0, grace=0.5)
wd.phase("headline", 30)
out["ms_per_step"] = 4.5
wd.phase("k5_splitfed x2", {limit})
time.sleep({sleep})
wd.disarm()
print("finished")
"""


def _run(rank=0, limit=0.5, sleep=20.0, env=None):
    code = _SCRIPT.format(root=ROOT, rank=rank, limit=limit, sleep=sleep)
    e = dict(os.environ)
    e.pop("SLK_BENCH_STALL", None)
    e.update(env or {})
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, env=e)


def test_watchdog_prints_partial_json_and_exits_nonzero():
    r = _run()
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr[-2000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "finished" not in r.stdout
    d = json.loads(lines[0])
    assert d["error"] == "watchdog: k5_splitfed x2"
    assert d["value"] == 123.0 and d["ms_per_step"] == 4.5 and d["nested"] == {"a": [1, 2]}
    assert d["phases_completed"] == ["headline"]
    assert "Thread" in r.stderr and "watchdog" in r.stderr     # all-thread stack dump


def test_watchdog_quiet_when_phases_finish():
    r = _run(limit=30, sleep=0.5)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "finished"


def test_watchdog_nonzero_rank_prints_no_json():
    r = _run(rank=2, limit=0.3)
    assert r.returncode == 3
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_stall_knob_stalls_the_named_phase():
    # the phase itself would finish at once (sleep 0), but the knob parks rank 0 inside it
    r = _run(limit=0.5, sleep=0.0, env={"SLK_BENCH_STALL": "k5_splitfed", "SLK_BENCH_STALL_RANK": "0"})
    assert r.returncode == 3
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["error"] == "watchdog: k5_splitfed x2" and d["value"] == 123.0
