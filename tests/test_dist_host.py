"""Host-side logic of gemmul8.dist on the CPU: the unit orders of ShardPlan, the workspace cache bound, the
side-stream knob and the stage watchdog (no GPU, no process group)."""
import io
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
from gemmul8 import dist as GD  # noqa: E402


@pytest.mark.parametrize("order", ["moduli", "columns"])
@pytest.mark.parametrize("m,n,N,W", [(16384, 16384, 14, 8), (16384, 16384, 14, 4), (16384, 16384, 14, 2),
                                     (1000, 3000, 9, 6), (700, 2600, 5, 3), (512, 4096, 3, 7), (256, 2560, 20, 8)])
def test_plan_covers_every_residue_column_once(order, m, n, N, W):
    p = GD.ShardPlan(m, n, N, W, order=order)
    cover = {}
    for r in range(W):
        got = set()
        for j0, j1, c0, c1 in p.launches[r]:
            assert c0 % 256 == 0 and (c1 % 256 == 0 or c1 == n)
            for j in range(j0, j1):
                got.add((j, c0, c1))
                for c in range(c0, c1, 256):
                    assert (j, c) not in cover
                    cover[(j, c)] = r
        # the moduli a rank encodes are one contiguous range holding every modulus its launches use
        j0, j1 = p.mods[r]
        assert all(j0 <= j < j1 for j, _, _ in got)
    assert set(cover) == {(j, c) for j in range(N) for c in range(0, n, 256)}
    # every unit is sent to (or kept by) the owner of its columns, once
    for r in range(W):
        s0, s1 = p.cols[r]
        recv = sorted((j, a) for t in range(p.stages) for (_, j, a, b) in p.recvs(r, t))
        own = sorted((j, c) for (j, c), q in cover.items() if q == r and s0 <= c < s1)
        need = sorted((j, c) for j in range(N) for c in range(s0, s1, 256))
        got = sorted(set((j, c) for (j, a) in recv for c in [a]) | set(own))
        assert {x[0] for x in got} <= set(range(N)) and len(need) >= len(own)
    # equal MACs per rank when the column blocks come out equal (ragged n: the last block is shorter)
    macs = [sum((c1 - c0) * (j1 - j0) for j0, j1, c0, c1 in p.launches[r]) for r in range(W)]
    if n % (256 * p.col_blocks) == 0:
        assert max(macs) == min(macs)
    assert sum(macs) == N * n


def test_columns_order_cfg3_encodes_a_quarter_of_b():
    """cfg3 at W = 8: column-major units give each rank 7 moduli of one quarter of the columns; the
    modulus-major plan gives 2 moduli of (almost) all columns, and spreads the transfers over 7 peers"""
    pc = GD.ShardPlan(16384, 16384, 14, 8, order="columns")
    pm = GD.ShardPlan(16384, 16384, 14, 8, order="moduli")
    for r in range(8):
        assert pc.mods[r][1] - pc.mods[r][0] == 7
        assert {(c0, c1) for _, c0, c1 in pc.units[r]} == {GD.blocks(16384, 4)[r // 2]}
        assert len({s for t in range(pc.stages) for s, *_ in pc.sends(r, t)}) == 1
        assert pm.mods[r][1] - pm.mods[r][0] <= 3
    assert max(len({s for t in range(pm.stages) for s, *_ in pm.sends(r, t)}) for r in range(8)) == 7
    with pytest.raises(ValueError):
        GD.ShardPlan(64, 64, 4, 2, order="rows")


def test_workspace_cache_is_bounded():
    c = GD._WorkCache(cap=2)
    made = []
    mk = lambda tag: (lambda: made.append(tag) or tag)
    assert c.get(("work", 1), mk("a")) == "a"
    assert c.get(("work", 2), mk("b")) == "b"
    assert c.get(("work", 1), mk("x")) == "a"  # hit: becomes the most recent
    assert c.get(("side", 0), mk("s")) == "s"  # other entries do not count
    assert c.get(("work", 3), mk("c")) == "c"  # evicts ("work", 2), the least recently used workspace
    assert [k for k in c.keys() if k[0] == "work"] == [("work", 1), ("work", 3)]
    assert made == ["a", "b", "s", "c"]
    c.clear()
    assert c.keys() == []


def test_default_ops_are_per_thread_and_releasable():
    import threading
    mine = GD._shard_ops()
    assert GD._shard_ops() is mine
    other = []
    t = threading.Thread(target=lambda: other.append(GD._shard_ops()))
    t.start()
    t.join()
    assert other[0] is not mine
    mine.cache.get(("work", 9), lambda: "w")
    extra = GD.HipShardOps()
    extra.cache.get(("work", 1), lambda: "v")
    GD.release_workspaces(extra)
    assert mine.cache.keys() == [] and extra.cache.keys() == []


def test_side_stream_knob(monkeypatch):
    monkeypatch.delenv("GEMMUL8_DIST_SIDE_STREAM", raising=False)
    assert GD.side_stream_enabled()
    monkeypatch.setenv("GEMMUL8_DIST_SIDE_STREAM", "0")
    assert not GD.side_stream_enabled()


def test_watchdog_reports_the_stage_in_flight():
    out = io.StringIO()
    wd = GD.StageWatchdog(0.3, rank=5, out=out, exit=False)
    try:
        wd.arm("quick")
        time.sleep(0.05)
        wd.disarm()
        time.sleep(0.4)
        assert wd.fired is None  # a phase that ended in time reports nothing
        GD.progress("exchange stage 3", "sends to [1, 2], receives from [4] (side stream)")
        wd.arm("timed steps")
        deadline = time.time() + 5
        while wd.fired is None and time.time() < deadline:
            time.sleep(0.05)
        assert wd.fired is not None
        for part in ("rank 5", "timed steps", "exchange stage 3", "receives from [4]"):
            assert part in out.getvalue()
    finally:
        wd.close()


def test_watchdog_optional_phase_reports_and_exits_zero():
    """a phase armed with on_fire (bench.py: the work after the timed region) hands the message to the
    callback (rank 0 prints the line measured so far) and exits with status 0, not 3"""
    out, got = io.StringIO(), []
    wd = GD.StageWatchdog(0.2, rank=0, out=out, exit=False)
    try:
        wd.arm("variants: moduli_columns_gathered", got.append)
        deadline = time.time() + 5
        while wd.fired is None and time.time() < deadline:
            time.sleep(0.05)
        assert wd.fired is not None and wd.exit_status == 0
        assert got == [wd.fired] and "variants: moduli_columns_gathered" in got[0]
        # a failing callback is reported and does not stop the exit
        wd.arm("report", lambda msg: 1 / 0)
        deadline = time.time() + 5
        while "report failed" not in out.getvalue() and time.time() < deadline:
            time.sleep(0.05)
        assert "ZeroDivisionError" in out.getvalue() and wd.exit_status == 0
        wd.arm("timed steps")  # a measured phase stays fatal
        deadline = time.time() + 5
        while wd.exit_status != 3 and time.time() < deadline:
            time.sleep(0.05)
        assert wd.exit_status == 3
    finally:
        wd.close()
