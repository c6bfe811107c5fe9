"""GPU: bench.py end to end on short runs (a child process each, as the
driver runs it): the default line carries the roofline, the per-rank fields
and a passing parity check; --flags inplace,iphdr (the TX drop-in's mode,
checks written into the frames, no result array) carries its own in-place
ceiling probe and passes the parity check of the frame bytes."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def run_bench(*args):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "1",
           "--reps", "2", "--ramp-ms", "0", "--no-cpu-baseline", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_default_line():
    line = run_bench()
    assert line["parity_ok"] is True and line["parity_digest"]["ok"] is True
    assert line["per_rank"]["ranks"] == 1
    roof = line["roofline"]
    assert roof["bound"] == "hbm" and 0 < roof["frac"] < 1
    assert "ceiling_measured" in roof and len(line["lib_sha16"]) == 16
    # same-run visiting-order A/B and the layout's own bound
    ab = roof["order_ab"]
    assert set(ab["orders"]) == {"auto", "0,0", "3,4", "4,4", "2,5"}
    assert all(0 < v["frac_vs_ceiling"] < 1.2 for v in ab["orders"].values())
    assert 0 < roof["layout_bound_frac"] <= 1 and 0 < roof["frac_of_layout_bound"] < 1.2


def test_config3_layout_bound():
    """Config 3 (64-B payloads): the line states the layout's bound -- a
    106-B frame in 112 B + a 16-B descriptor per 82 algorithmic bytes -- so
    its fraction of 8 TB/s reads against what the layout allows."""
    line = run_bench("--config", "3")
    roof = line["roofline"]
    assert 0.5 < roof["layout_alg_over_real"] < 0.75
    assert roof["layout_bound_frac"] < 0.6 and roof["frac_of_layout_bound"] > 0.5


@pytest.mark.parametrize("cid", [2, 4])
def test_inplace_line(cid):
    line = run_bench("--config", str(cid), "--flags", "inplace,iphdr")
    assert line["parity_ok"] is True and line["parity_spot_check"] is True
    assert line["parity_digest"]["ok"] is True
    assert line["config"]["flags"] == "inplace,iphdr" and line["config"]["result_array"] is False
    roof = line["roofline"]
    assert roof["inplace_probe_ms"] > 0 and 0 < roof["frac_vs_inplace_probe"] < 2
