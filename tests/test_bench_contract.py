"""The committed bench line keeps the driver's contract (bench.py's JSON schema, roofline and
cpu_baseline objects) and agrees with the rocprofv3 summary committed beside it.  CPU only:
reads files under profiles/, runs nothing."""
import csv
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
# the round's final line (bench.py with the CPU baseline) and the rocprofv3 --kernel-trace --stats
# summary of the same frame (bench.py --no-cpu-baseline --no-extra-legs)
BENCH = ROOT / "profiles" / "r05" / "final" / "bench.json"
STATS = ROOT / "profiles" / "r05" / "final" / "kernel_stats.csv"
PEAK = {"fp32": 157.3, "fp16": 2500.0, "fp32-split": 2500.0, "mixed": 2500.0}

REQUIRED = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
            "roofline", "cpu_baseline"]


def _line():
    import pytest
    if not BENCH.exists():
        pytest.skip("the round's final bench line is not committed yet (tools/run_gpu_round.sh)")
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
    b = _line()
    r = b["roofline"]
    # the headline is the reference's precision: FP32 on the FP32 MFMA peak
    assert b["dtype"] == "fp32"
    assert r["bound"] in ("hbm", "mfma") and r["unit"] == "TFLOP/s" and r["peak"] == PEAK[b["dtype"]]
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    assert abs(r["achieved"] - r["flop_per_launch"] / (r["avg_kernel_ms"] / 1e3) / 1e12) \
        / r["achieved"] < 1e-6
    c = _line()["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0


def test_rocprof_agrees_with_live_timing():
    r = _line()["roofline"]
    with STATS.open() as f:
        rows = [row for row in csv.DictReader(f) if f"{r['kernel']}<" in row["Name"]]
    assert rows, f"{r['kernel']} missing from the rocprof summary"
    avg_ms = float(rows[0]["AverageNs"]) / 1e6
    assert abs(avg_ms - r["avg_kernel_ms"]) / avg_ms < 0.05
