"""bench.py's companion measurement (the elasticity system inside the ONE JSON line of a Poisson run): a failure or a
hang of the companion -- or of the teardown after it -- never costs the metric line (host logic, CPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fem355 import dist  # noqa: E402


def test_companion_result_drops_line_keys(capsys):
    out = {"metric": "m", "value": 1.0}
    d = {"metric": "m", "value": 2.0, "n_gpus": 1, "dtype": "f64", "roofline": {"frac": 0.5}}
    g = dist.CompanionGuard(out, "elasticity", timeout=30)
    res = g.run(lambda: d)
    g.emit()
    g.emit()   # printed once
    g.close()
    assert res["value"] == 1.0
    assert res["elasticity"] == {"value": 2.0, "roofline": {"frac": 0.5}}
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0])["elasticity"]["value"] == 2.0


def test_companion_exception_is_reported():
    def boom():
        raise RuntimeError("no RCCL")
    g = dist.CompanionGuard({"value": 1.0}, "elasticity", timeout=30)
    res = g.run(boom)
    g.close()
    assert res["value"] == 1.0 and "no RCCL" in res["elasticity"]["error"]


def test_companion_other_ranks_print_nothing(capsys):
    g = dist.CompanionGuard(None, "elasticity", rank=1, timeout=30)
    assert g.run(lambda: None) is None
    g.emit()
    g.close()
    assert capsys.readouterr().out == ""


def _run(code):
    p = subprocess.run([sys.executable, "-c", "import sys, time; sys.path.insert(0, %r); from fem355 import dist; "
                        % ROOT + code], capture_output=True, text=True, timeout=120)
    return p.returncode, [ln for ln in p.stdout.splitlines() if ln.strip()], p.stderr


def test_companion_timeout_prints_metric_line_and_exits_cleanly():
    rc, lines, err = _run("g = dist.CompanionGuard({'value': 3.0}, 'elasticity', timeout=1.0); "
                          "g.run(lambda: time.sleep(60)); print('not reached')")
    assert rc == 0, err
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["value"] == 3.0 and "timed out" in d["elasticity"]["error"]


def test_hang_after_the_line_exits_without_a_second_line():
    rc, lines, err = _run("g = dist.CompanionGuard({'value': 3.0}, 'elasticity', timeout=1.0); "
                          "g.run(lambda: {'value': 5.0}); g.emit(); time.sleep(60); print('not reached')")
    assert rc == 0, err
    assert len(lines) == 1, lines
    assert json.loads(lines[0])["elasticity"] == {"value": 5.0}
