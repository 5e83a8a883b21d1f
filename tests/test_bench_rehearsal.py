"""ARTIFACT CHECK (it parses a committed file; it does not run bench.py or gemmul8.dist, so it stays green whatever
they become -- tests/test_bench_cli.py and tests/test_dist.py test the code).  CPU check of the committed 8-rank
rehearsal of the driver's multi-GPU bench:
`GEMMUL8_BENCH_BACKEND=gloo python bench.py --gpus 8 --size 2048` on one GPU (8 ranks sharing the device, so its
timings mean nothing) must produce ONE complete line: the cfg3-style sharded step, the single-GPU baseline, the
accuracy check and every partition variant timed, nothing marked incomplete or failed.  The line is the one
`tools/gpu_session.sh <tag> gloo8=--size 2048` wrote (profiles/r06/gloo8.json); its source_sha16 field names the
bench.py / gemmul8.dist / gemmul8 binding revision that produced it (test_line_matches_sources)."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = os.path.join(ROOT, "profiles", "r06", "gloo8.json")

VARIANTS = ["moduli_columns", "moduli_columns_gathered", "moduli_whole_planes_to_root", "row_blocks_all_moduli",
            "output_blocks_2x4_all_moduli", "moduli_grid_2x4", "moduli_partial_sums_reduce"]


@pytest.fixture(scope="module")
def line():
    if not os.path.exists(LINE):
        pytest.skip("no committed rehearsal line")
    with open(LINE) as f:
        lines = [x for x in f.read().splitlines() if x.strip()]
    assert len(lines) == 1, "rank 0 prints exactly one JSON line"
    return json.loads(lines[0])


def test_contract_fields(line):
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in line, key
    assert line["n_gpus"] == 8 and line["config"]["world_size"] == 8
    assert line["scaling"] == "strong" and line["higher_is_better"] is True
    assert line["config"]["parallelism"] == "row blocks 2 x (moduli x column blocks) x4 x8"
    assert line["config"]["partition"] == "grid"
    assert line["cpu_baseline"] is None  # rank 0 at N = 1 only
    assert "incomplete" not in line


def test_every_phase_measured(line):
    assert line["value"] > 0 and line["ms_per_step"] > 0
    r = line["roofline"]
    assert r["bound"] == "mfma" and r["achieved"] > 0 and "aggregate" in r and "composite" in r
    assert set(line["step_phases_ms_rank0"]) == {"shifts", "encode", "products", "exchange", "crt"}
    assert line["single_gpu_ms"] > 0 and line["strong_scaling_efficiency"] > 0
    assert 0 < line["relerr_max"] < 1e-6  # the sharded C checked against the double-double GEMM on every rank
    assert [list(u) for u in line["launches_rank0"]]


def test_every_variant_timed(line):
    v = line["variants"]
    assert sorted(v) == sorted(VARIANTS)
    for name in VARIANTS:
        assert isinstance(v[name], dict), (name, v[name])  # a string would be "failed: ..."
        assert v[name]["ms_per_step"] > 0


def test_line_matches_sources(line):
    """the committed line was produced by the sources under test (else it is a stale artifact: regenerate it)"""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_for_sha", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    now = b.source_sha16()
    if line.get("source_sha16") != now:
        pytest.skip(f"stale artifact: line from {line.get('source_sha16')}, sources now {now}")
