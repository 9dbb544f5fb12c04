"""The committed bench line keeps the driver's contract (bench.py's JSON schema, roofline and
cpu_baseline objects) and agrees with the rocprofv3 summary committed beside it.  CPU only:
reads files under profiles/, runs nothing."""
import csv
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
BENCH = ROOT / "profiles" / "r02_final/bench.json"
STATS = ROOT / "profiles" / "r02_final/kernel_stats.csv"

REQUIRED = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
            "roofline", "cpu_baseline"]


def _line():
    return json.loads(BENCH.read_text().strip().splitlines()[-1])


def test_bench_line_schema():
    b = _line()
    for k in REQUIRED:
        assert k in b, k
    assert b["n_gpus"] == 1 and b["scaling"] == "weak" and b["higher_is_better"] is True
    assert "workload" in b["config"]
    # value = W*H*64 ray-samples per frame / ms_per_step
    assert abs(b["value"] - 800 * 800 * 64 / (b["ms_per_step"] / 1e3)) / b["value"] < 1e-6


def test_roofline_consistent():
    r = _line()["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["unit"] == "TFLOP/s" and r["peak"] == 2500.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    assert abs(r["achieved"] - r["flop_per_launch"] / (r["avg_kernel_ms"] / 1e3) / 1e12) \
        / r["achieved"] < 1e-6
    c = _line()["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0


def test_rocprof_agrees_with_live_timing():
    r = _line()["roofline"]
    with STATS.open() as f:
        rows = [row for row in csv.DictReader(f) if "k_march16" in row["Name"]]
    assert rows, "k_march16 missing from the rocprof summary"
    avg_ms = float(rows[0]["AverageNs"]) / 1e6
    assert abs(avg_ms - r["avg_kernel_ms"]) / avg_ms < 0.05
