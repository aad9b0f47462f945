"""bench.py's live counter leg (`roofline.traffic` and the VALU issue were
looked up in committed PMC files): at N = 1 rank 0 re-runs the timed layout under
`rocprofv3 --pmc` children after the timed region, and the line's `roofline.traffic` is that
run's FETCH_SIZE x 2 + WRITE_SIZE.  Run the way the driver runs bench.py.  Needs an MI355X: -m gpu."""
import json
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "2", "--skeletons", "1024", "--steps", "3",
           "--warmup", "1", "--no-cpu-baseline", "--no-parity", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(shutil.which("rocprofv3") is None, reason="rocprofv3 not on PATH")
def test_bench_traffic_is_measured_in_the_run():
    line = run_bench("--layout", "4:16:1:1:0:1:1", "--pmc", "on")
    live = line["pmc_live"]
    assert "error" not in live, live
    rf = line["roofline"]
    assert rf["traffic_source"].startswith("pmc")
    assert rf["traffic"] == live["hbm_bytes_per_launch"]
    # at least the algorithmic bytes (poses in and out, targets, setup tables), and not absurdly more
    assert rf["algorithmic_bytes_per_launch"] * 0.5 < rf["traffic"] < rf["algorithmic_bytes_per_launch"] * 50
    assert live["child_layout_keys"] == ["c2_1024_" + rf["traffic_key"].split("c2_1024_")[1]]
    pw = live["per_wave"]
    assert pw["waves"] > 0 and 0 < pw["issue_frac"] < 1 and 0 <= pw["wait_any_frac"] < 1


def test_bench_pmc_off_reports_its_source():
    line = run_bench("--layout", "4:16:1:1:0:1:1", "--pmc", "off")
    assert "pmc_live" not in line
    rf = line["roofline"]
    assert rf["traffic"] is None or rf["traffic_source"].startswith("profiles/traffic.json")


@pytest.mark.skipif(shutil.which("rocprofv3") is None, reason="rocprofv3 not on PATH")
def test_bench_issue_is_measured_for_one_wave_layouts():
    """A layout with one kind of wave per block takes `issue` from the run's own counters; the
    helper-wave layout keeps the committed replay figure of its solving wave (and says so)."""
    line = run_bench("--layout", "4:16:1:1:0:1:0", "--pmc", "on")
    assert "error" not in line["pmc_live"], line["pmc_live"]
    assert line["issue"]["source"] == "pmc_live (this run)"
    assert line["issue"]["frac"] == line["pmc_live"]["per_wave"]["issue_frac"]
    helper = run_bench("--layout", "4:16:1:1:0:1:1", "--pmc", "on")
    assert helper["issue"] is None or helper["issue"]["source"].startswith("profiles/valu_mix.json")
