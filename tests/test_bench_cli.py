"""bench.py's host logic on the CPU: the --gpus launcher and the workload / metric selection
(BASELINE.json: cfg2 on one GPU, the moduli-sharded cfg3 on more)."""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launcher_spawns_ranks_only_outside_torchrun(monkeypatch):
    b = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert b.launch_command(b.parse([]), []) is None
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd = b.launch_command(b.parse(argv), argv)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv
    monkeypatch.setenv("WORLD_SIZE", "8")  # under torchrun: the ranks are already there
    assert b.launch_command(b.parse(argv), argv) is None


def test_workload_selection_and_labels():
    b = _bench()
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    W = b.select_workload(b.parse([]), 1)
    assert (W["name"], W["m"], W["N"], W["fast"], W["custom"]) == ("cfg2", 8192, 14, True, False)
    wl, metric = b.labels(W)
    assert metric == base["metric"] and wl.startswith("cfg2")
    W = b.select_workload(b.parse(["--gpus", "8"]), 8)
    assert (W["name"], W["m"], W["N"], W["fast"], W["custom"]) == ("cfg3", 16384, 14, True, False)
    wl, metric = b.labels(W)
    assert "16384" in metric and "cfg3" in metric and metric != base["metric"] and "sharded" in wl
    W = b.select_workload(b.parse(["--gpus", "4", "--partition", "rows"]), 4)
    assert W["name"] == "cfg2"
    W = b.select_workload(b.parse(["--size", "4096"]), 1)
    wl, metric = b.labels(W)
    assert W["custom"] and "4096" in metric and metric != base["metric"] and not wl.startswith("cfg")
    W = b.select_workload(b.parse(["--workload", "cfg4"]), 1)
    assert (W["m"], W["N"], W["fast"], W["kind"], W["custom"]) == (8192, 10, False, "dfd", False)
    assert "accurate" in b.labels(W)[1]
    W = b.select_workload(b.parse(["--workload", "cfg5"]), 1)
    assert (W["m"], W["N"], W["kind"]) == (4096, 12, "z") and "ZGEMM" in b.labels(W)[1]


def test_headline_partition(monkeypatch):
    """--partition auto: the 2-D unit grid at an even W >= 4 in fast mode (measured faster than the moduli units on
    the cfg3 replay, profiles/r06/cfg3_partitions/), the (modulus, column block) units otherwise; an explicit
    --partition wins; sub-groups that failed at setup (GEMMUL8_BENCH_NO_GRID) fall back to moduli"""
    b = _bench()
    monkeypatch.delenv("GEMMUL8_BENCH_NO_GRID", raising=False)
    assert b.resolve_partition(b.parse(["--gpus", "8"]), 8, True) == "grid"
    assert b.resolve_partition(b.parse(["--gpus", "4"]), 4, True) == "grid"
    assert b.resolve_partition(b.parse(["--gpus", "2"]), 2, True) == "moduli"
    assert b.resolve_partition(b.parse(["--gpus", "6"]), 6, True) == "grid"
    assert b.resolve_partition(b.parse(["--gpus", "8", "--accurate"]), 8, False) == "moduli"
    assert b.resolve_partition(b.parse(["--gpus", "8", "--partition", "moduli"]), 8, True) == "moduli"
    assert b.resolve_partition(b.parse(["--gpus", "8", "--partition", "rows"]), 8, True) == "rows"
    assert b.resolve_partition(b.parse([]), 1, True) == "single"
    monkeypatch.setenv("GEMMUL8_BENCH_NO_GRID", "1")
    assert b.resolve_partition(b.parse(["--gpus", "8"]), 8, True) == "moduli"
    assert b.select_workload(b.parse(["--gpus", "8"]), 8)["name"] == "cfg3"


def test_algorithmic_work_and_composite_roofline():
    """cfg2's fused-minimum bytes (operands once, slices and residues written and read once,
    C once) and the composite fraction; the per-phase GB/s follow from phase_ms"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
    import gemmul8 as G
    b = _bench()
    L = G.layout(8192, 8192, 8192, 14, G.REAL_DEFAULT)
    w = b.algorithmic_work(8192, 8192, 8192, 14, "d", True, L)
    mk = 8192 * 8192
    assert w["int8_ops"] == 2.0 * mk * 8192 * 14
    assert w["bytes"]["split"] == 2 * 8 * mk + 14 * 2 * mk
    assert w["bytes"]["products"] == 14 * 2 * mk + 14 * mk
    assert w["bytes"]["crt"] == 14 * mk + 8 * mk
    assert abs(w["bytes"]["total"] - 7.248e9) < 0.01e9  # 7.28 GB with the reference's k' = 8256
    c = b.composite_roofline(w, 6.0, {"scaling": 0.7, "inverse_scaling": 0.27})
    t_m, t_h = w["int8_ops"] / (b.INT8_PEAK_TOPS * 1e12), w["bytes"]["total"] / (b.HBM_PEAK_GBS * 1e9)
    assert abs(c["frac"] - (t_m + t_h) / 6e-3) < 1e-4
    assert abs(c["phases"]["split"]["GBps"] - w["bytes"]["split"] / 0.7e-3 / 1e9) < 0.1
    assert abs(c["phases"]["crt"]["GBps"] - w["bytes"]["crt"] / 0.27e-3 / 1e9) < 0.1
    # over W GPUs the same work is priced against W peaks
    c8 = b.composite_roofline(w, 6.0 / 8, None, 8)
    assert abs(c8["frac"] - c["frac"]) < 1e-3 and "phases" not in c8
    # accurate mode: the bound plane and its magnitude slices on top
    La = G.layout(8192, 8192, 8192, 10, G.REAL_DEFAULT)
    wa = b.algorithmic_work(8192, 8192, 8192, 10, "dfd", False, La)
    assert wa["int8_ops"] == 2.0 * mk * 8192 * 11
    assert wa["bytes"]["split"] == 8 * mk + 4 * mk + 10 * 2 * mk + 2 * mk


def test_new_bench_options():
    b = _bench()
    a = b.parse(["--gpus", "2", "--order", "columns", "--no-single-gpu"])
    assert a.order == "columns" and a.no_single_gpu
    assert b.parse([]).order == "moduli" and not b.parse([]).no_single_gpu


def test_physical_core_count_from_cpuinfo(monkeypatch, tmp_path):
    """cpu_baseline's all-core bound counts distinct (physical id, core id) pairs, not SMT siblings"""
    b = _bench()
    text = "".join(f"processor\t: {i}\nphysical id\t: {i // 4 % 2}\ncore id\t\t: {i % 2}\n\n" for i in range(8))
    f = tmp_path / "cpuinfo"
    f.write_text(text)
    real_open = open
    monkeypatch.setattr("builtins.open", lambda p, *a, **k: real_open(f if p == "/proc/cpuinfo" else p, *a, **k))
    assert b._physical_cores() == 4  # 2 sockets x 2 cores, each core listed twice


def test_step_power_sampler_fields(monkeypatch):
    """bench.StepPower (the N = 1 line's power_steady_state) against a stand-in amdsmi: energy per step from the
    settled window's accumulator readings, clocks averaged over the 8 XCDs, PPT residency from the accumulators"""
    import time
    import types
    t0 = time.perf_counter()
    tick = lambda: time.perf_counter() - t0
    fake = types.SimpleNamespace(
        amdsmi_init=lambda: None, amdsmi_shut_down=lambda: None,
        amdsmi_get_power_cap_info=lambda d: {"power_cap": 1400000000},
        # 1400 W: 1400 J/s = 1400e6 uJ/s at 15.3 uJ per count
        amdsmi_get_energy_count=lambda d: {"energy_accumulator": int(tick() * 1400e6 / 15.3),
                                           "counter_resolution": 15.3},
        amdsmi_get_gpu_metrics_info=lambda d: {
            "current_socket_power": 1400, "current_gfxclks": [1600] * 8, "temperature_hotspot": 60,
            "energy_accumulator": int(tick() * 1400e6 / 15.3), "ppt_residency_acc": int(tick() * 1e6),
            "accumulation_counter": int(tick() * 1e6)})
    monkeypatch.setitem(sys.modules, "amdsmi", fake)
    b = _bench()
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import power_trace
    monkeypatch.setattr(power_trace, "find_device", lambda smi: ("dev", "bdf"))
    sp = b.StepPower(period=0.002)
    sp.begin()
    time.sleep(0.2)
    out = sp.end(100, settle=0.3)  # 100 steps in 0.2 s: 2 ms and 2.8 J per step at 1400 W
    assert out["power_cap_W"] == 1400 and out["gfxclk_MHz_mean_8xcd"] == 1600 and out["socket_power_W_mean"] == 1400
    assert abs(out["power_from_energy_W"] - 1400) < 50 and abs(out["energy_per_step_J"] - 2.8) < 0.2
    assert out["ppt_limiter_residency"] == 1.0 and out["samples"] > 10 and abs(out["loop_ms_per_step"] - 2.0) < 0.3
