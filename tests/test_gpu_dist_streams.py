"""GPU: gemmul8.dist's NCCL branch -- stream-ordered transfers, receive-only stages on a side stream, no host
synchronisation -- run with 2 or 3 ranks as threads on one GPU through tests/fake_nccl.py, a stand-in for
ProcessGroupNCCL's stream semantics (a one-GPU box cannot run RCCL with more than one rank).  The gloo tests
cover the host-synchronised branch only.  Every rank runs the real native steps on its own compute stream with its
own workspace; several calls follow each other through the same workspaces without a host sync, so a missing
stream dependency (a transfer reading residues before their product launch, a receive overwriting columns the
previous call's CRT still reads, the CRT starting before the last receive) shows up as wrong bits against the
single gemmul8_gemm call.
"""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fake_nccl import FakeNcclWorld, run_ranks  # noqa: E402
from test_gpu_phases import _rand, _same, _single  # noqa: E402


DELAY = 200_000  # GPU cycles of spin before every received copy (~0.1 ms): transfers always land late


def _world(W, monkeypatch, delay=DELAY):
    from gemmul8 import dist as GD
    world = FakeNcclWorld(W, delay_cycles=delay)
    monkeypatch.setattr(GD, "dist", world.module)
    return world


def _inputs(m, n, k, seeds, dtype):
    import torch
    data = [(_rand(m, k, s, dtype), _rand(k, n, s + 1, dtype) * (10.0 ** (s % 3))) for s in seeds]
    torch.cuda.synchronize()
    return data


def _on_own_stream(fn):
    """fn() on a fresh compute stream of the calling rank thread; waits for it before returning"""
    import torch
    comp = torch.cuda.Stream()
    with torch.cuda.stream(comp):
        out = fn()
    comp.synchronize()
    return out


@pytest.mark.parametrize("W,side", [(2, True), (3, True), (3, False)])
def test_exchange_stream_ordered_back_to_back(W, side, monkeypatch):
    """three calls with different operands per rank, back to back on one compute stream: each rank's column block
    equals the single call's, bit for bit; with and without the side stream for receive-only stages"""
    import torch
    from gemmul8 import dist as GD
    if not side:
        monkeypatch.setenv("GEMMUL8_DIST_SIDE_STREAM", "0")
    world = _world(W, monkeypatch)
    m, n, k, N = 1000, 1536, 1100, 14
    data = _inputs(m, n, k, (1, 3, 5), torch.float64)
    refs = [_single(A, B, N, True, torch.float64) for A, B in data]
    plan = GD.ShardPlan(m, n, N, W)

    def rank(r):
        ops = GD.HipShardOps()
        return _on_own_stream(lambda: [GD.matmul_moduli(A, B, N, True, gather=False, ops=ops) for A, B in data])

    res = run_ranks(world, rank)
    for r in range(W):
        c0, c1 = plan.cols[r]
        for i in range(len(data)):
            assert _same(res[r][i], refs[i][:, c0:c1]), (r, i)
    assert world.calls["batch_isend_irecv"] >= W * plan.stages // 2 and world.calls["all_gather"] == 3 * W


def test_gather_accurate_and_complex(monkeypatch):
    """C gathered on the root (the blocks received concurrently), accurate mode (the bound maxima MAX-combined
    on the communication streams), complex Karatsuba operands (three residue sub-planes per transfer)"""
    import torch
    import gemmul8 as G
    from gemmul8 import dist as GD
    W = 3
    world = _world(W, monkeypatch)
    m, n, k, N = 520, 768, 700, 14  # (every rank owns columns: blocks of 256)
    (A, B), (A2, B2) = _inputs(m, n, k, (7, 9), torch.float64)
    mc, nc, kc, Nc = 1024, 768, 3072, 12
    (Ac, Bc), = _inputs(mc, nc, kc, (11,), torch.complex128)
    assert G.layout(mc, nc, kc, Nc, G.COMPLEX_BIG_MATRIX_ENCODE)["nsub"] == 3
    ref_f = _single(A, B, N, True, torch.float64)
    ref_a = _single(A2, B2, N, False, torch.float64)
    ref_c = _single(Ac, Bc, Nc, True, torch.complex128)
    plan_c = GD.ShardPlan(mc, nc, Nc, W)

    def rank(r):
        ops = GD.HipShardOps()

        def calls():
            return (GD.matmul_moduli(A, B, N, True, gather=True, ops=ops),
                    GD.matmul_moduli(A2, B2, N, False, gather=True, ops=ops),
                    GD.matmul_moduli(A2, B2, N, False, gather=False, ops=ops),
                    GD.matmul_moduli(Ac, Bc, Nc, True, gather=False, ops=ops))
        return _on_own_stream(calls)

    res = run_ranks(world, rank)
    assert _same(res[0][0], ref_f) and _same(res[0][1], ref_a)
    assert all(res[r][0] is None and res[r][1] is None for r in range(1, W))
    plan = GD.ShardPlan(m, n, N, W)
    for r in range(W):
        c0, c1 = plan.cols[r]
        assert _same(res[r][2], ref_a[:, c0:c1]), r
        c0, c1 = plan_c.cols[r]
        assert _same(res[r][3], ref_c[:, c0:c1]), r
    assert world.calls["all_reduce"] == 2 * W  # the two accurate calls


def test_planes_to_root_and_partial_sums_reduce(monkeypatch):
    """the two comparison partitions bench.py times: whole residue planes sent to the root (bit-identical C) and
    the north star's sum-reduce of partial CRT sums (C1 exact, C2 reordered: within 2^-40 of max |C|)"""
    import torch
    import gemmul8 as G
    from gemmul8 import dist as GD
    W = 3
    world = _world(W, monkeypatch)
    m, n, k, N = 700, 600, 900, 14
    data = _inputs(m, n, k, (13, 15), torch.float64)
    refs = [_single(A, B, N, True, torch.float64) for A, B in data]

    def rank(r):
        ops = GD.HipShardOps()

        def calls():
            out = []
            for A, B in data:
                out.append(GD.gemm_moduli_planes_to_root(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, True, ops=ops))
                out.append(GD.gemm_moduli_reduce(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, True, ops=ops))
            return out
        return _on_own_stream(calls)

    res = run_ranks(world, rank)
    for i, ref in enumerate(refs):
        planes, red = res[0][2 * i], res[0][2 * i + 1]
        assert _same(planes.t(), ref)
        err = (red.t() - ref).abs().max().item()
        assert err <= 2.0 ** -40 * ref.abs().max().item(), (i, err)
    assert all(x is None for r in range(1, W) for x in res[r])
    assert world.calls["reduce"] == 2 * W


@pytest.mark.parametrize("order,op", [("moduli", "T"), ("columns", "T"), ("moduli", "N")])
def test_grid_over_sub_groups(order, op, monkeypatch):
    """gemm_moduli_grid under the NCCL branch: 4 ranks in 2 row blocks, each a gemm_moduli over its own sub-group
    (its own P2P channels and collective sequence), two calls back to back without a host sync: every rank's block
    and the gathered C (sub-roots to the root over the parent group) equal the single call bit for bit.  op N is
    the path bench.py times: the row block of op(A) is then a strided column range A[:, r0:r1] of the (k, m)
    storage, passed with the parent's lda = m"""
    import torch
    import gemmul8 as G
    from gemmul8 import dist as GD
    W, H = 4, 2
    monkeypatch.setattr(GD, "_GRID_GROUPS", {})
    world = _world(W, monkeypatch)
    m, n, k, N = 1000, 1536, 1100, 14
    data = _inputs(m, n, k, (21, 23), torch.float64)
    refs = [_single(A, B, N, True, torch.float64) for A, B in data]
    if op == "N":  # column-major m x k / k x n storage of the same matrices
        data = [(A.t().contiguous(), B.t().contiguous()) for A, B in data]
        torch.cuda.synchronize()
    gop, lda, ldb = (G.OP_N, m, k) if op == "N" else (G.OP_T, k, n)

    def rank(r):
        ops = GD.HipShardOps()

        def calls():
            out = []
            for A, B in data:
                out.append(GD.gemm_moduli_grid(gop, gop, m, n, k, A, lda, B, ldb, N, True, ops=ops, row_blocks=H,
                                               order=order))
                out.append(GD.gemm_moduli_grid(gop, gop, m, n, k, A, lda, B, ldb, N, True, ops=ops, row_blocks=H,
                                               gather=True, order=order))
            return out
        return _on_own_stream(calls)

    res = run_ranks(world, rank)
    Gs = W // H
    for i, ref in enumerate(refs):
        for r in range(W):
            h, sub = divmod(r, Gs)
            r0, r1 = GD.blocks(m, H)[h]
            c0, c1 = GD.ShardPlan(r1 - r0, n, N, Gs, GD.TILE, order).cols[sub]
            blk = res[r][2 * i]
            assert tuple(blk.shape) == (c1 - c0, r1 - r0), (i, r)
            assert _same(blk.t(), ref[r0:r1, c0:c1]), (i, r)
        assert _same(res[0][2 * i + 1].t(), ref), i
        assert all(res[r][2 * i + 1] is None for r in range(1, W))
    assert len(world._groups) == H  # the sub-groups were created once, not per call


def test_grid_over_non_world_parent(monkeypatch):
    """gemm_moduli_grid over a parent group smaller than the world: 6 processes, the call runs on
    the 4 ranks of a sub-group only.  new_group is collective over the WHOLE world unless it synchronises
    locally (tests/fake_nccl.py enforces it), so the row-block sub-groups must be created with local
    synchronization, else ranks 0-3 wait for 4 and 5 forever (a hang under RCCL).  Blocks bit-identical to
    the single call"""
    import torch
    import gemmul8 as G
    from gemmul8 import dist as GD
    W, H = 6, 2
    monkeypatch.setattr(GD, "_GRID_GROUPS", {})
    world = FakeNcclWorld(W, timeout_s=60.0, delay_cycles=DELAY)
    monkeypatch.setattr(GD, "dist", world.module)
    m, n, k, N = 700, 900, 650, 12
    (A, B), = _inputs(m, n, k, (31,), torch.float64)
    ref = _single(A, B, N, True, torch.float64)

    def rank(r):
        parent = world.module.new_group([0, 1, 2, 3])  # every process enters (world-collective creation)
        if r >= 4:
            return None
        ops = GD.HipShardOps()
        return _on_own_stream(lambda: GD.gemm_moduli_grid(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, True, ops=ops,
                                                          group=parent, row_blocks=H))

    res = run_ranks(world, rank)
    Gs = 4 // H
    for r in range(4):
        h, sub = divmod(r, Gs)
        r0, r1 = GD.blocks(m, H)[h]
        c0, c1 = GD.ShardPlan(r1 - r0, n, N, Gs, GD.TILE, "moduli").cols[sub]
        assert _same(res[r].t(), ref[r0:r1, c0:c1]), r
    assert res[4] is None and res[5] is None


def test_negative_control_dropped_transfers(monkeypatch):
    """the comparison depends on the exchanged data: with every receive completed without its copy, the owners'
    blocks differ from the single call (operands no other test uses, so a recycled workspace cannot already hold
    their residues).  A missing stream dependency, by contrast, is caught with high probability only: streams
    that share a hardware queue run in order (tests/fake_nccl.py)"""
    import torch
    from gemmul8 import dist as GD
    W = 2
    world = FakeNcclWorld(W, drop_receives=True)
    monkeypatch.setattr(GD, "dist", world.module)
    m, n, k, N = 1000, 1536, 1100, 14
    (A, B), = _inputs(m, n, k, (31,), torch.float64)
    ref = _single(A, B, N, True, torch.float64)
    plan = GD.ShardPlan(m, n, N, W)
    res = run_ranks(world, lambda r: _on_own_stream(
        lambda: GD.matmul_moduli(A, B, N, True, gather=False, ops=GD.HipShardOps())))
    bad = [r for r in range(W) if not _same(res[r], ref[:, plan.cols[r][0]:plan.cols[r][1]])]
    assert bad == list(range(W)), bad


def test_row_blocks_accurate_gathered(monkeypatch):
    """matmul_rows under the NCCL branch: accurate mode MAX-combines the bound product's column maxima, the root
    gathers the row blocks; equal to the single call over all rows, bit for bit"""
    import torch
    from gemmul8 import dist as GD
    W = 3
    world = _world(W, monkeypatch)
    m, n, k, N = 900, 500, 800, 12
    (A, B), = _inputs(m, n, k, (21,), torch.float64)
    ref = _single(A, B, N, False, torch.float64)
    bl = GD.blocks(m, W)
    res = run_ranks(world, lambda r: _on_own_stream(
        lambda: GD.matmul_rows(A[bl[r][0]:bl[r][1]].contiguous(), B, N, False, gather=True, ops=GD.HipOps())))
    assert _same(res[0], ref)
    assert res[1] is None and res[2] is None
    assert world.calls["all_reduce"] == W



def test_random_cases():
    """40 random cases of the NCCL branch (tests/dist_soak.py; its command line runs hundreds)"""
    from dist_soak import soak
    n, fails = soak(40, 2024)
    assert n == 0, fails[:3]
