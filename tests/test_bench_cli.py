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
