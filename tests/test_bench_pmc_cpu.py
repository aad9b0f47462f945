"""bench.py's live counter leg, host side (no GPU): when it runs, and how it reads rocprofv3's
counter CSVs (tests/test_gpu_bench_pmc.py runs it for real on an MI355X)."""
import argparse
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def write_csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(w.fieldnames, r)))


def test_counter_means_last_dispatches(tmp_path):
    b = load_bench()
    rows = []
    # an autotune-candidate dispatch first, then three timed ones; FETCH_SIZE split over two
    # counter instances (rows are summed per dispatch); another kernel in between is ignored
    rows.append((1, "void mbik_solve_kernel<...>", "FETCH_SIZE", 999.0))
    for d, v in ((5, 10.0), (7, 20.0), (9, 30.0)):
        rows.append((d, "void (anonymous namespace)::mbik_solve_kernel_rw<4, 2, 103>(...)", "FETCH_SIZE", v / 2))
        rows.append((d, "void (anonymous namespace)::mbik_solve_kernel_rw<4, 2, 103>(...)", "FETCH_SIZE", v / 2))
        rows.append((d + 1, "void mbik_tile_rows(...)", "FETCH_SIZE", 1e9))
    p = tmp_path / "run_counter_collection.csv"
    write_csv(p, rows)
    m = b.counter_means([str(p)], "mbik_solve_kernel", ["FETCH_SIZE"])
    assert m == {"FETCH_SIZE": 20.0}
    assert b.counter_means([str(p)], "mbik_cmode_kernel", ["FETCH_SIZE"]) is None


def test_pmc_enabled_rules(monkeypatch):
    b = load_bench()
    ns = argparse.Namespace
    monkeypatch.delenv("LD_PRELOAD", raising=False)
    for k in list(os.environ):
        if k.startswith("ROCPROF"):
            monkeypatch.delenv(k)
    assert not b.pmc_enabled(ns(pmc="off"), 1)
    assert not b.pmc_enabled(ns(pmc="child"), 1)
    assert not b.pmc_enabled(ns(pmc="on"), 2)          # never at N > 1
    assert b.pmc_enabled(ns(pmc="on"), 1)
    monkeypatch.setattr("shutil.which", lambda name: "/opt/rocm/bin/rocprofv3")
    assert b.pmc_enabled(ns(pmc="auto"), 1)
    monkeypatch.setenv("ROCPROF_COUNTERS", "SQ_WAVES")  # already under a profiler
    assert not b.pmc_enabled(ns(pmc="auto"), 1)
    monkeypatch.delenv("ROCPROF_COUNTERS")
    monkeypatch.setattr("shutil.which", lambda name: None)
    assert not b.pmc_enabled(ns(pmc="auto"), 1)


def test_layout_fields_round_trip():
    """The child's --layout string is the timed plan's mbik_plan_info layout, in bench.py's
    --layout field order (K:spw:interval:staging:placement:waves:helper:roles)."""
    b = load_bench()
    info = {"lanes_per_skeleton": 4, "skeletons_per_block": 64, "checkpoint_interval": 2, "heading_staging": 0,
            "state_placement": 2, "waves_per_simd": 2, "helper_wave": 0, "wave_roles": 1}
    assert ":".join(str(int(info[k])) for k in b.LAYOUT_FIELDS) == "4:64:2:0:2:2:0:1"
    assert b.layout_key(info) == "K4_s64_i2_st0_pl2_w2_rw"
