"""bench.py's companion measurement (the elasticity system inside the ONE JSON line of a Poisson run): a failure or a
hang of the companion never costs the metric line (host logic, CPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fem355 import dist  # noqa: E402


def test_companion_result_drops_line_keys():
    out = {"metric": "m", "value": 1.0}
    d = {"metric": "m", "value": 2.0, "n_gpus": 1, "dtype": "f64", "roofline": {"frac": 0.5}}
    res = dist.guarded_companion(out, "elasticity", lambda: d, timeout=30)
    assert res["value"] == 1.0
    assert res["elasticity"] == {"value": 2.0, "roofline": {"frac": 0.5}}


def test_companion_exception_is_reported():
    def boom():
        raise RuntimeError("no RCCL")
    res = dist.guarded_companion({"value": 1.0}, "elasticity", boom, timeout=30)
    assert res["value"] == 1.0 and "no RCCL" in res["elasticity"]["error"]


def test_companion_other_ranks_return_none():
    assert dist.guarded_companion(None, "elasticity", lambda: None, rank=1, timeout=30) is None


def test_companion_timeout_prints_metric_line_and_exits_cleanly():
    code = ("import sys, time; sys.path.insert(0, %r); from fem355 import dist; "
            "dist.guarded_companion({'value': 3.0}, 'elasticity', lambda: time.sleep(60), timeout=1.0); "
            "print('not reached')") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 3.0 and "timed out" in d["elasticity"]["error"]
