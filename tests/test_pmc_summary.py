"""scripts/pmc_summary.py: per-launch HBM bytes from rocprofv3 PMC passes.

The bench's `roofline.traffic` comes from these summaries, so the averaging
rules are pinned here on synthetic counter CSVs shaped like rocprofv3's:
FETCH_SIZE is doubled (gfx950 reports half of a wide streaming read), the
DP classes of one rf_realign are summed, and only full-size launches count
(the bench's trailing scorer launch without a DP before it, and c5's 16-read
parity launch, must not dilute the means)."""
import csv
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(REPO, "scripts", "pmc_summary.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, name, v in rows:
            w.writerow({"Dispatch_Id": d, "Kernel_Name": name, "Counter_Name": "X", "Counter_Value": v})


DP1 = "void k_dpr<1, true, 11, 16, true>(DPTask const*, int)"
DP2 = "void k_dpr<2, true, 33, 16, false>(DPTask const*, int)"
WS = "void k_score_ws<19, 256>(WorkItem const*)"
SCAT = "k_scatter(Segment const*)"


def _run(tmp_path, fetch_rows, write_rows):
    run = str(tmp_path / "run")
    _write(os.path.join(run, "pmc_FETCH_SIZE", "p_counter_collection.csv"), fetch_rows)
    _write(os.path.join(run, "pmc_WRITE_SIZE", "p_counter_collection.csv"), write_rows)
    mod = _load()
    f_tot, f_cnt = mod.per_launch(os.path.join(run, "pmc_FETCH_SIZE", "p_counter_collection.csv"))
    w_tot, w_cnt = mod.per_launch(os.path.join(run, "pmc_WRITE_SIZE", "p_counter_collection.csv"))
    return f_tot, f_cnt, w_tot, w_cnt


def test_dp_groups_and_trailing_scorer_launch(tmp_path):
    # three steps: two DP classes + scatter + scorer; then one scorer launch
    # with no DP before it (the bench's parity pass)
    rows = []
    d = 0
    for _ in range(3):
        rows += [(d, DP1, 100.0), (d + 1, DP2, 20.0), (d + 2, SCAT, 1.0), (d + 3, WS, 300.0)]
        d += 4
    rows.append((d, WS, 300.0))
    f_tot, f_cnt, w_tot, w_cnt = _run(tmp_path, rows, rows)
    # k_dp: mean over the three real groups (120 each), not diluted by the 4th launch
    assert f_cnt["k_dp"] == 3
    assert f_tot["k_dp"] / f_cnt["k_dp"] == pytest.approx(120.0)
    assert f_tot["k_score"] / f_cnt["k_score"] == pytest.approx(300.0)


def test_small_parity_launch_excluded(tmp_path):
    rows = []
    for s in range(4):
        rows += [(3 * s, DP1, 50.0), (3 * s + 1, WS, 1000.0)]
    rows.append((99, WS, 2.0))          # 16-read parity launch
    f_tot, f_cnt, _, _ = _run(tmp_path, rows, rows)
    assert f_cnt["k_score"] == 4
    assert f_tot["k_score"] / f_cnt["k_score"] == pytest.approx(1000.0)


def test_main_doubles_fetch(tmp_path):
    rows = [(0, DP1, 10.0), (1, WS, 40.0)]
    run = str(tmp_path / "run")
    _write(os.path.join(run, "pmc_FETCH_SIZE", "p_counter_collection.csv"), rows)
    _write(os.path.join(run, "pmc_WRITE_SIZE", "p_counter_collection.csv"), rows)
    mod = _load()
    import json
    import sys
    out = str(tmp_path / "out.json")
    argv = sys.argv
    try:
        sys.argv = ["pmc_summary.py", run, out, "1"]
        mod.main()
    finally:
        sys.argv = argv
    res = json.load(open(out))["kernels"]
    assert res["k_score"]["fetch_bytes"] == 2 * 1024 * 40.0     # KiB -> bytes, x2 (gfx950)
    assert res["k_score"]["write_bytes"] == 1024 * 40.0
    assert res["k_dp"]["hbm_bytes_per_launch"] == 2 * 1024 * 10.0 + 1024 * 10.0


def test_bench_quotes_traffic_at_the_profiled_size():
    """bench.py's roofline.traffic comes from profiles/pmc_<config>.json only
    when that profile was taken at the run's size: clusters per rank (c4),
    reads per rank (c5; round 3 compared 5000 reads with 'clusters': 1)."""
    import json
    import sys
    sys.path.insert(0, REPO)
    import bench
    for cfg, key in (("c4", "clusters"), ("c5", "reads")):
        pm = json.load(open(os.path.join(REPO, "profiles", f"pmc_{cfg}.json")))
        size = pm[key]
        got = bench.pmc_traffic(cfg, size, "k_score")
        assert got == pm["kernels"]["k_score"]["hbm_bytes_per_launch"]
        assert bench.pmc_traffic(cfg, size + 1, "k_score") is None
