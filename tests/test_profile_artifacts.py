"""The committed round-6 measurement artifacts agree with each other (CPU; reads files only):
the profiled bench line's event-timed product launch against the rocprofv3 kernel trace of the same command
(the roofline's `achieved` must match the committed summary), its traffic against the PMC passes
(profiles/pmc_traffic.json, which bench.py reports), and the headline lines' contract fields."""
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles", "r06", "prof")
KERNEL = "gemm_i8_persistent_pg_kernel<false, 1, 0>"


def _load(*parts):
    with open(os.path.join(ROOT, *parts)) as f:
        return json.load(f)


def test_rocprof_average_matches_the_line():
    line = _load("profiles", "r06", "prof", "bench.json")
    rows = [r for r in csv.reader(open(os.path.join(PROF, "kernel_stats.csv"))) if KERNEL in r[0]]
    assert len(rows) == 1, rows
    avg_ms = float(rows[0][3]) / 1e6  # AverageNs
    events_ms = line["roofline"]["avg_launch_ms"]
    # rocprof averages every launch of the command (warm-up and the accuracy call included), the line the timed ones
    assert abs(avg_ms - events_ms) / events_ms < 0.05, (avg_ms, events_ms)
    assert line["roofline"]["kernel"].startswith("gemm_i8_persistent_pg_kernel")


def test_traffic_matches_the_pmc_summary():
    summ = _load("profiles", "r06", "prof", "summary.json")

    def find(d):
        if isinstance(d, dict):
            for k, v in d.items():
                if KERNEL in str(k) and isinstance(v, dict) and "hbm_read_bytes" in v:
                    return v
                r = find(v)
                if r:
                    return r
        return None

    k = find(summ)
    assert k is not None
    traffic = _load("profiles", "pmc_traffic.json")
    assert abs(k["hbm_read_bytes"] - traffic["hbm_read_bytes"]) / traffic["hbm_read_bytes"] < 0.01
    assert abs(k["hbm_write_bytes"] - traffic["hbm_write_bytes"]) / traffic["hbm_write_bytes"] < 0.01
    line = _load("profiles", "r06", "prof", "bench.json")
    assert line["roofline"]["traffic"] == traffic["gemm_hbm_bytes_per_launch"]


def test_headline_lines_keep_the_contract():
    for name in ("bench_cfg2_final.json", "bench_cfg4.json", "bench_cfg5.json"):
        line = _load("profiles", "r06", "lines", name)
        for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                    "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
            assert key in line, (name, key)
        rf = line["roofline"]
        assert rf["bound"] == "mfma" and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3, (name, rf)
        assert line["n_gpus"] == 1 and line["value"] > 0
    cfg2 = _load("profiles", "r06", "lines", "bench_cfg2_final.json")
    assert "cpu_baseline" in cfg2 and cfg2["cpu_baseline"]["value"] > 0
    assert cfg2["config"]["workload"].startswith("cfg2")
