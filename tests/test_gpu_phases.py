"""GPU: the phase entry points (gemmul8_split / _split_bound / _products / _recombine) and the
multi-GPU partitions of gemmul8.dist, run through the native library.

Every composition must reproduce the single gemmul8_gemm call (itself bit-exact against the
oracle, test_gpu_parity.py) bit for bit:
  * moduli computed in separate ranges (the modulus-sharded layout),
  * accurate-mode row blocks whose bound-product column maxima are MAX-combined,
  * gemmul8.dist.matmul_rows / matmul_moduli in a one-rank RCCL group.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rand(m, n, seed, dtype):
    import torch
    g = torch.Generator().manual_seed(seed)
    def one():
        return (torch.rand((m, n), generator=g, dtype=torch.float64) - 0.5) * torch.exp(
            torch.randn((m, n), generator=g, dtype=torch.float64))
    x = one()
    if dtype.is_complex:
        x = torch.complex(x, one())
    return x.to(dtype).cuda()


def _single(A, B, N, fast, out_dtype):
    import torch
    import gemmul8 as G
    m, k = A.shape
    n = B.shape[1]
    Ct = torch.empty((n, m), dtype=out_dtype, device="cuda")
    ct = G.COMPLEX_BIG_MATRIX_ENCODE if A.is_complex() else G.REAL_DEFAULT
    work = G.alloc_work(m, n, k, N, ct)
    G.gemm(G.OP_T, G.OP_T, m, n, k, 1.0, A, k, B, n, 0.0, Ct, m, N, fast, work, ct)
    torch.cuda.synchronize()
    return Ct.t().contiguous()


def _same(a, b):
    import torch
    # (flattened first: a one-column block of a column-major buffer counts as contiguous with a stride of m)
    flat = lambda x: x.reshape(-1).contiguous().view(torch.uint8)
    return a.shape == b.shape and torch.equal(flat(a), flat(b))


@pytest.mark.parametrize("m,n,k,N,fast,dt", [
    (300, 260, 500, 14, True, "f64"),
    (257, 190, 333, 9, False, "f64"),
    (200, 128, 256, 6, True, "f32"),
    # (m + n) k >= 2^25: the phase entry points fork operand B's split onto the second stream
    (2048, 1900, 8400, 14, True, "f64"),
    (1900, 2048, 8400, 11, False, "f64"),
])
def test_moduli_ranges_compose(m, n, k, N, fast, dt):
    import torch
    import gemmul8 as G
    tdt = torch.float64 if dt == "f64" else torch.float32
    A, B = _rand(m, k, 1, tdt), _rand(k, n, 2, tdt)
    ref = _single(A, B, N, fast, tdt)
    work = G.alloc_work(m, n, k, N)
    for j0, j1 in ((0, 1), (1, N // 2), (N // 2, N)):
        G.split(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, fast, work, tdt, j0, j1)
        G.products(m, n, k, N, work, j0, j1)
    Ct = torch.empty((n, m), dtype=tdt, device="cuda")
    G.recombine(m, n, k, N, 1.0, 0.0, Ct, m, work)
    torch.cuda.synchronize()
    assert _same(Ct.t(), ref)


@pytest.mark.parametrize("m,n,k,N,fast,dt", [
    (300, 260, 500, 14, True, "f64"), (257, 190, 333, 20, False, "f64"), (200, 128, 256, 6, True, "f64"),
    (210, 140, 300, 8, True, "f64"), (200, 128, 256, 7, True, "f32"), (180, 100, 200, 12, False, "f32"),
])
def test_partial_crt_sums(m, n, k, N, fast, dt):
    """gemmul8_crt_partial / _finish (the north star's reduce of FP64 partial CRT sums, gemm_moduli_reduce):
    over the full moduli range the finish reproduces the single call bit for bit; over a partition, the summed
    C1 planes equal the full range's exactly and C is within a few ulp (C2's summation order differs)."""
    import torch
    import gemmul8 as G
    tdt = torch.float64 if dt == "f64" else torch.float32
    A, B = _rand(m, k, 11, tdt), _rand(k, n, 12, tdt)
    ref = _single(A, B, N, fast, tdt)
    work = G.alloc_work(m, n, k, N)
    G.split(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, fast, work, tdt)
    G.products(m, n, k, N, work)
    full = torch.empty((2, n, m), dtype=torch.float64, device="cuda")
    G.crt_partial(m, n, k, N, tdt, work, 0, N, full)
    Ct = torch.empty((n, m), dtype=tdt, device="cuda")
    G.crt_finish(m, n, k, N, 1.0, 0.0, Ct, m, work, full)
    torch.cuda.synchronize()
    assert _same(Ct.t(), ref)
    parts = [(0, 1), (1, N // 2), (N // 2, N - 1), (N - 1, N)]
    S = torch.zeros((2, n, m), dtype=torch.float64, device="cuda")
    for j0, j1 in parts:
        Sp = torch.empty_like(S)
        G.crt_partial(m, n, k, N, tdt, work, j0, j1, Sp)
        S += Sp
    G.crt_finish(m, n, k, N, 1.0, 0.0, Ct, m, work, S)
    torch.cuda.synchronize()
    numM2 = N >= 8 and dt == "f64"
    if numM2 or N <= 5:  # exact C1 (and numM = 1 with exact sums)
        assert torch.equal(S[0], full[0])
    # one-level moduli at N = 6, 7 sum C = sum NMi r_i beyond 2^53 (rounded in any order: the single call's own
    # error there is of that size); two-level: only the low words' sum is reordered; float: the output rounding
    tol = 2.0 ** (-19 if dt == "f32" else -40 if (numM2 or N <= 5) else -26)
    err = (Ct.t().double() - ref.double()).abs().max().item()
    assert err <= tol * ref.double().abs().max().item(), err
    # alpha / beta through the same epilogue as the single call
    C0 = _rand(m, n, 13, tdt)
    Cab, Cref = C0.t().contiguous().clone(), C0.t().contiguous().clone()
    G.crt_finish(m, n, k, N, 2.5, -0.5, Cab, m, work, full)
    G.recombine(m, n, k, N, 2.5, -0.5, Cref, m, work)
    torch.cuda.synchronize()
    assert _same(Cab, Cref)
    # a column-major sub-matrix view with ldc > m (as gemm() accepts), and the out_dtype check
    ldc = m + 37
    big = torch.full((n + 2, ldc), 7.0, dtype=tdt, device="cuda")
    Cv = big[1:n + 1, :m]
    G.crt_finish(m, n, k, N, 1.0, 0.0, Cv, ldc, work, full, out_dtype=tdt)
    torch.cuda.synchronize()
    assert _same(Cv.t(), ref) and bool((big[0] == 7).all()) and bool((big[n + 1] == 7).all())
    assert bool((big[1:n + 1, m:] == 7).all())
    with pytest.raises(TypeError):
        G.crt_finish(m, n, k, N, 1.0, 0.0, Ct, m, work, full,
                     out_dtype=torch.float32 if tdt == torch.float64 else torch.float64)
    with pytest.raises(ValueError):  # the view's storage ends before the last column
        G.crt_finish(m, n, k, N, 1.0, 0.0, big[3:n + 2, :m], ldc, work, full)


@pytest.mark.parametrize("fast", [True, False])
def test_moduli_ranges_compose_complex_karatsuba(fast):
    """complex at a shape where the size rule runs Karatsuba sub-products (k >= 3072, m >= 1024): split /
    products over moduli ranges + recombine == one call, and the residue planes hold 3 sub-planes"""
    import torch
    import gemmul8 as G
    m, n, k, N = 1024, 300, 3100, 12
    ct = G.COMPLEX_BIG_MATRIX_ENCODE
    L = G.layout(m, n, k, N, ct)
    if L["nsub"] != 3:
        pytest.skip("GEMMUL8_CPLX_PRODUCTS forces the big matrix")
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn((k, m), dtype=torch.complex128, device="cuda", generator=g)  # column-major m x k
    B = torch.randn((n, k), dtype=torch.complex128, device="cuda", generator=g)  # column-major k x n
    ref = torch.empty((n, m), dtype=torch.complex128, device="cuda")
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, ref, m, N, fast, G.alloc_work(m, n, k, N, ct), ct)
    work = G.alloc_work(m, n, k, N, ct)
    if not fast:
        G.split_bound(0, 0, m, n, k, A, m, B, k, N, work, torch.complex128, ct)
    for j0, j1 in ((0, 1), (1, N // 2), (N // 2, N)):
        G.split(0, 0, m, n, k, A, m, B, k, N, fast, work, torch.complex128, j0, j1, ct, bound_ready=not fast)
        G.products(m, n, k, N, work, j0, j1, ct)
    Ct = torch.empty((n, m), dtype=torch.complex128, device="cuda")
    G.recombine(m, n, k, N, 1.0, 0.0, Ct, m, work, ct)
    torch.cuda.synchronize()
    assert _same(Ct, ref)
    assert G.residue_planes(work, m, n, k, N, 0, N, ct).shape == (N, 3 * L["vsA"] * L["vsB"])


def test_accurate_row_blocks_with_combined_bound():
    import torch
    from gemmul8 import dist as GD
    m, n, k, N = 700, 300, 400, 12
    A, B = _rand(m, k, 3, torch.float64), _rand(k, n, 4, torch.float64)
    ref = _single(A, B, N, False, torch.float64)
    blocks = GD.row_partition(m, 3)
    ops = [GD.HipOps() for _ in blocks]  # one per simulated rank (each caches its own workspace)
    states, colmaxes = [], []
    for (r0, r1), o in zip(blocks, ops):
        cm, st = o.row_bound(A[r0:r1].contiguous(), B, N, torch.float64)
        colmaxes.append(cm)
        states.append(st)
    torch.cuda.synchronize()
    comb = torch.stack([c.clone() for c in colmaxes]).amax(0)
    for c in colmaxes:  # what the MAX all-reduce leaves in every rank's workspace
        c.copy_(comb)
    out = torch.cat([o.finish_rows(st) for o, st in zip(ops, states)], 0)
    torch.cuda.synchronize()
    assert _same(out, ref)
    # without the exchange the column shifts differ (the reason the all-reduce exists)
    cm, st = ops[0].row_bound(A[:256].contiguous(), B, N, torch.float64)
    alone = ops[0].finish_rows(st)
    torch.cuda.synchronize()
    assert not _same(alone, ref[:256])


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dist_one_rank_rccl():
    import torch
    import torch.distributed as dist
    import gemmul8 as G
    from gemmul8 import dist as GD
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        m, n, k, N = 520, 300, 260, 14
        A, B = _rand(m, k, 5, torch.float64), _rand(k, n, 6, torch.float64)
        ref = _single(A, B, N, True, torch.float64)
        assert _same(GD.matmul_moduli(A, B, N, True), ref)
        assert _same(GD.matmul_moduli(A, B, N, True, gather=False), ref)
        assert _same(GD.matmul_rows(A, B, N, True, gather=True), ref)
        refa = _single(A, B, N, False, torch.float64)
        assert _same(GD.matmul_rows(A, B, N, False), refa)
        assert _same(GD.matmul_moduli(A, B, N, False), refa)
        # the same shape again with other operands through the cached default workspace: accurate mode
        # depends on the bound area being zeroed by every call
        A2, B2 = _rand(m, k, 15, torch.float64) * 1e3, _rand(k, n, 16, torch.float64)
        assert _same(GD.matmul_moduli(A2, B2, N, False), _single(A2, B2, N, False, torch.float64))
        assert _same(GD.matmul_moduli(A, B, N, False), refa)
        assert _same(GD.matmul_moduli(A, B, N, False, order="columns"), refa)
        # the north star's reduce of partial CRT sums, one rank: the whole moduli range, so the same bits
        Cr = GD.gemm_moduli_reduce(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, True)
        assert _same(Cr.t(), ref)
        Cr = GD.gemm_moduli_reduce(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, False)
        assert _same(Cr.t(), refa)
        os.environ["GEMMUL8_DIST_SIDE_STREAM"] = "0"
        try:
            assert _same(GD.matmul_moduli(A2, B2, N, True), _single(A2, B2, N, True, torch.float64))
        finally:
            del os.environ["GEMMUL8_DIST_SIDE_STREAM"]
        # the default ops keep at most WORKSPACE_CACHE workspaces, and release_workspaces frees them
        for mm in (264, 296, 328):
            GD.matmul_moduli(_rand(mm, k, 7, torch.float64), B, N, True)
        works = [kk for kk in GD._shard_ops().cache.keys() if kk[0] == "work"]
        assert len(works) == GD.WORKSPACE_CACHE and works[-1][1] == 328
        GD.release_workspaces()
        assert GD._shard_ops().cache.keys() == [] and GD._row_ops().cache.keys() == []
    finally:
        dist.destroy_process_group()


def _simulate_moduli_shards(opA, opB, m, n, k, A, lda, B, ldb, N, fast, out_dtype, ct, world, align=256):
    """gemm_moduli's data flow with `world` simulated ranks in one process, each with its own workspace
    (HipShardOps instance): shift blocks assembled, bound maxima MAX-combined, residue column runs copied
    from the producing rank's workspace into the owner's (the P2P transfers), per-rank CRT of its columns."""
    import torch
    from gemmul8 import dist as GD
    plan = GD.ShardPlan(m, n, N, world, align)
    ops = [GD.HipShardOps() for _ in range(world)]
    st = [o.prepare(opA, opB, m, n, k, A, lda, B, ldb, N, fast, out_dtype, ct) for o in ops]
    for r in range(world):
        ops[r].stats(st[r], plan.rows[r], plan.cols[r])
    vecs = [ops[r].shift_vectors(st[r]) for r in range(world)]
    for r in range(world):  # the all-gathers
        (a0, a1), (b0, b1) = plan.rows[r], plan.cols[r]
        for q in range(world):
            if q != r:
                vecs[q][0][a0:a1] = vecs[r][0][a0:a1]
                vecs[q][1][b0:b1] = vecs[r][1][b0:b1]
    if not fast:
        bnd = [ops[r].bound(st[r], plan.cols[r]).clone() for r in range(world)]
        comb = torch.stack(bnd).amax(0)
        for r in range(world):  # the MAX all-reduce
            L = st[r]["L"]
            st[r]["work"][L["offBound"]:L["offBound"] + 4 * comb.numel()].view(torch.int32).copy_(comb)
    for r in range(world):
        j0, j1 = plan.mods[r]
        if j1 > j0 or not fast:  # (accurate: the final shifts even without moduli)
            ops[r].encode(st[r], j0, j1)
    for t in range(plan.stages):
        for r in range(world):
            if t < len(plan.launches[r]):
                ops[r].products(st[r], *plan.launches[r][t])
        for r in range(world):
            for dst, j, a, b in plan.sends(r, t):
                for x, y in zip(ops[r].chunks(st[r], j, a, b), ops[dst].chunks(st[dst], j, a, b)):
                    y.copy_(x)
    out = [ops[r].recombine(st[r], *plan.cols[r]).clone() for r in range(world)]
    torch.cuda.synchronize()
    return torch.cat(out, 0), plan


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("m,n,k,N,fast,dt", [
    (600, 1500, 500, 14, True, "f64"),
    (520, 1300, 333, 9, False, "f64"),
    (300, 1100, 256, 6, True, "f32"),
    (700, 1025, 300, 12, True, "c128"),
    (300, 900, 200, 10, False, "c128"),
])
def test_moduli_column_shards_simulated(world, m, n, k, N, fast, dt):
    """the (modulus, column block) partition of gemm_moduli through the native sharded entry points
    (gemmul8_shard_stats / _shard_bound / _split SHIFTS_READY / _products_cols / _recombine_cols),
    simulated ranks in one process: bit-identical to one gemm call"""
    import torch
    import gemmul8 as G
    tdt = {"f64": torch.float64, "f32": torch.float32, "c128": torch.complex128}[dt]
    ct = G.COMPLEX_BIG_MATRIX_ENCODE if tdt.is_complex else G.REAL_DEFAULT
    A, B = _rand(m, k, 21, tdt), _rand(k, n, 22, tdt)  # row-major = column-major transposes: op T
    ref = torch.empty((n, m), dtype=tdt, device="cuda")
    G.gemm(G.OP_T, G.OP_T, m, n, k, 1.0, A, k, B, n, 0.0, ref, m, N, fast, G.alloc_work(m, n, k, N, ct), ct)
    got, plan = _simulate_moduli_shards(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, fast, tdt, ct, world)
    for j in range(N):  # every modulus' columns covered exactly once
        assert sum(c1 - c0 for us in plan.units for (jj, c0, c1) in us if jj == j) == n
    assert _same(got, ref)


def test_moduli_column_shards_karatsuba_and_op_n():
    """complex at a Karatsuba shape (k >= 3072, m >= 1024: 3 residue sub-planes, one column run per
    sub-plane) and column-major op N operands, fast and accurate"""
    import torch
    import gemmul8 as G
    m, n, k, N = 1024, 800, 3100, 12
    ct = G.COMPLEX_BIG_MATRIX_ENCODE
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn((k, m), dtype=torch.complex128, device="cuda", generator=g)  # column-major m x k
    B = torch.randn((n, k), dtype=torch.complex128, device="cuda", generator=g)  # column-major k x n
    for fast in (True, False):
        ref = torch.empty((n, m), dtype=torch.complex128, device="cuda")
        G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, ref, m, N, fast, G.alloc_work(m, n, k, N, ct), ct)
        got, _ = _simulate_moduli_shards(0, 0, m, n, k, A, m, B, k, N, fast, torch.complex128, ct, 4)
        assert _same(got, ref), fast


def test_products_cols_and_recombine_cols_compose():
    """products over column ranges + CRT over column ranges == one call (one workspace)"""
    import torch
    import gemmul8 as G
    m, n, k, N = 500, 1000, 700, 14
    A, B = _rand(m, k, 31, torch.float64), _rand(k, n, 32, torch.float64)
    ref = _single(A, B, N, True, torch.float64)
    work = G.alloc_work(m, n, k, N)
    G.split(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, True, work, torch.float64)
    for j0, j1, c0, c1 in ((0, 5, 0, 256), (0, 5, 256, 1000), (5, 14, 0, 768), (5, 14, 768, 1000)):
        G.products(m, n, k, N, work, j0, j1, cols=(c0, c1))
    Ct = torch.empty((n, m), dtype=torch.float64, device="cuda")
    for c0, c1 in ((0, 300), (300, 301), (301, 1000)):
        G.recombine(m, n, k, N, 1.0, 0.0, Ct[c0:c1], m, work, cols=(c0, c1))
    torch.cuda.synchronize()
    assert _same(Ct.t(), ref)
    with pytest.raises(G.Gemmul8Error):
        G.products(m, n, k, N, work, 0, 1, cols=(100, 300))  # column ranges start on a tile


@pytest.mark.parametrize("S", [1, 3, 13])
@pytest.mark.parametrize("fast", [True, False])
def test_low_memory_mode_same_bits(S, fast):
    """gemmul8_gemm_lowmem: the moduli in groups of S through S slice planes"""
    import torch
    import gemmul8 as G
    m, n, k, N = 300, 280, 333, 14
    A, B = _rand(m, k, 11, torch.float64), _rand(k, n, 12, torch.float64)
    ref = _single(A, B, N, fast, torch.float64)
    assert G.workSize(m, n, k, N, slice_planes=S) < G.workSize(m, n, k, N)
    work = G.alloc_work(m, n, k, N, slice_planes=S)
    Ct = torch.empty((n, m), dtype=torch.float64, device="cuda")
    G.gemm(G.OP_T, G.OP_T, m, n, k, 1.0, A, k, B, n, 0.0, Ct, m, N, fast, work, slice_planes=S)
    torch.cuda.synchronize()
    assert _same(Ct.t(), ref)


def test_low_memory_mode_complex():
    import torch
    import gemmul8 as G
    m, n, k, N = 200, 150, 170, 12
    A, B = _rand(m, k, 13, torch.complex128), _rand(k, n, 14, torch.complex128)
    Acm, Bcm = A.t().contiguous(), B.t().contiguous()
    out = []
    for S in (None, 5):
        work = G.alloc_work(m, n, k, N, G.COMPLEX_BIG_MATRIX_ENCODE, slice_planes=S)
        Ct = torch.empty((n, m), dtype=torch.complex128, device="cuda")
        G.gemm(0, 0, m, n, k, 1.0, Acm, m, Bcm, k, 0.0, Ct, m, N, True, work, G.COMPLEX_BIG_MATRIX_ENCODE,
               slice_planes=S)
        out.append(Ct)
    torch.cuda.synchronize()
    assert _same(out[0], out[1])


_MULTI_RANK_CHILD = r'''
import os, sys
import torch
import torch.distributed as dist
sys.path[:0] = [sys.argv[1], sys.argv[2]]
from gemmul8 import dist as GD
from test_gpu_phases import _rand, _single, _same
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)  # the ranks share the one GPU; gloo carries the messages
dist.init_process_group("gloo")
try:
    m, n, k, N = 700, 1100, 400, 14
    ok = True
    for dt in (torch.float64, torch.complex128):
        A, B = _rand(m, k, 11, dt), _rand(k, n, 12, dt)
        for fast in (True, False):
            ref = _single(A, B, N, fast, dt)
            C = GD.matmul_moduli(A, B, N, fast)
            if rank == 0:
                ok &= _same(C, ref)
            Cb = GD.matmul_moduli(A, B, N, fast, gather=False)
            c0, c1 = GD.ShardPlan(m, n, N, world).cols[rank]
            ok &= _same(Cb, ref[:, c0:c1])
            r0, r1 = GD.row_partition(m, world)[rank]
            Cr = GD.matmul_rows(A[r0:r1].contiguous(), B, N, fast, gather=True)
            if rank == 0:
                ok &= _same(Cr, ref)
    dist.barrier()
    if rank == 0:
        print("RESULT", "OK" if ok else "MISMATCH")
finally:
    dist.destroy_process_group()
'''


def test_dist_three_ranks_on_one_gpu_gloo():
    """gemmul8.dist with three processes on the one GPU (gloo messages): the (modulus, column block)
    partition with its shift all-gathers, bound all-reduce and staged residue exchange, gathered
    and distributed, and the row partition (accurate mode: the MAX all-reduce of the column bounds),
    real and complex, on the native kernels, bit-identical to the single call"""
    import subprocess
    import sys
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "--no-python", sys.executable, "-c",
           _MULTI_RANK_CHILD, tdir, os.path.join(root, "mixed-gemmul8_amd")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "RESULT OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


_GRID_CHILD = r'''
import os, sys
import torch
import torch.distributed as dist
sys.path[:0] = [sys.argv[1], sys.argv[2]]
from gemmul8 import dist as GD
from gemmul8 import OP_T, REAL_DEFAULT, COMPLEX_BIG_MATRIX_ENCODE
from test_gpu_phases import _rand, _single, _same
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)  # the ranks share the one GPU; gloo carries the messages
dist.init_process_group("gloo")
try:
    m, n, k, N = 900, 1100, 400, 14
    ok = True
    for dt in (torch.float64, torch.complex128):
        ct = COMPLEX_BIG_MATRIX_ENCODE if dt.is_complex else REAL_DEFAULT
        A, B = _rand(m, k, 11, dt), _rand(k, n, 12, dt)
        ref = _single(A, B, N, True, dt)
        # row-major operands: op T on both (A an (m, k) tensor, B an (k, n) one), C (n, m) column-major
        C = GD.gemm_moduli_grid(OP_T, OP_T, m, n, k, A, k, B, n, N, True, dt, ct, row_blocks=2, gather=True)
        if rank == 0:
            ok &= _same(C.t(), ref)
        Cb = GD.gemm_moduli_grid(OP_T, OP_T, m, n, k, A, k, B, n, N, True, dt, ct, row_blocks=2)
        G_ = world // 2
        r0, r1 = GD.blocks(m, 2)[rank // G_]
        c0, c1 = GD.ShardPlan(r1 - r0, n, N, G_).cols[rank % G_]
        ok &= _same(Cb.t(), ref[r0:r1, c0:c1])
    dist.barrier()
    if rank == 0:
        print("RESULT", "OK" if ok else "MISMATCH")
finally:
    dist.destroy_process_group()
'''


def test_dist_grid_four_ranks_on_one_gpu_gloo():
    """gemmul8.dist.gemm_moduli_grid with four processes on the one GPU (gloo): two row blocks of two ranks, each a
    (modulus, column block) partition over its own sub-group, real and complex, gathered and distributed, on the
    native kernels -- bit-identical to the single call"""
    import subprocess
    import sys
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "--no-python", sys.executable, "-c",
           _GRID_CHILD, tdir, os.path.join(root, "mixed-gemmul8_amd")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "RESULT OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def test_cfg3_size_moduli_shards_simulated_8_ranks():
    """BASELINE cfg3 at full size (16384^3, 14 moduli, fast mode, the reference driver's inputs) through the
    8-rank (modulus, column block) data flow, each simulated rank with its own workspace (8 x 11.5 GiB): the
    assembled C is bit-identical to one gemmul8_gemm call"""
    import torch
    import gemmul8 as G
    m = n = k = 16384
    N = 14
    A = G.randmat(m, k, torch.float64, 0.5, 123456)  # column-major m x k, op N (bench.py's cfg3 operands)
    B = G.randmat(k, n, torch.float64, 0.5, 123456)
    ref = torch.empty((n, m), dtype=torch.float64, device="cuda")
    work = G.alloc_work(m, n, k, N)
    G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, ref, m, N, True, work)
    torch.cuda.synchronize()
    del work
    got, plan = _simulate_moduli_shards(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, True, torch.float64, G.REAL_DEFAULT, 8)
    assert [len(x) for x in plan.units] == [7] * 8
    assert torch.equal(got.view(torch.uint8), ref.view(torch.uint8))
    del got
    torch.cuda.empty_cache()


def test_moduli_column_shards_randomized():
    """40 random calls through the simulated (modulus, column block) data flow: random shapes (m, n up to
    1300, k up to 1500), num_moduli 2..20, 2..8 ranks, real f64 / f32 / mixed f64 x f32 / complex, fast and
    accurate, ops N / T (and C for complex) -- each bit-identical to the single call"""
    import torch
    import gemmul8 as G
    rng = np.random.default_rng(int(os.environ.get("GEMMUL8_SHARD_FUZZ_SEED", "2027")))
    tdts = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}
    for case in range(int(os.environ.get("GEMMUL8_SHARD_FUZZ_CASES", "40"))):
        ta = tb = "dszc"[int(rng.integers(4))]
        if ta == "d" and rng.random() < 0.3:
            tb = "s"
        cplx = ta in "zc"
        m, n, k = (int(rng.integers(1, 1300)), int(rng.integers(1, 1300)), int(rng.integers(1, 1500)))
        N = int(rng.integers(2, 21))
        world = int(rng.integers(2, 9))
        fast = bool(rng.integers(2))
        if cplx and not fast and N > 17:
            N = 17
        opA, opB = int(rng.integers(3 if cplx else 2)), int(rng.integers(3 if cplx else 2))
        ct = G.COMPLEX_BIG_MATRIX_ENCODE if cplx else G.REAL_DEFAULT
        out_dtype = tdts["z" if cplx and "z" in (ta, tb) else ("d" if "d" in (ta, tb) else ta)]
        A = (_rand(k, m, 100 + case, tdts[ta]) if opA == 0 else _rand(m, k, 100 + case, tdts[ta]))
        B = (_rand(n, k, 200 + case, tdts[tb]) if opB == 0 else _rand(k, n, 200 + case, tdts[tb]))
        lda, ldb = (m if opA == 0 else k), (k if opB == 0 else n)
        ref = torch.empty((n, m), dtype=out_dtype, device="cuda")
        G.gemm(opA, opB, m, n, k, 1.0, A, lda, B, ldb, 0.0, ref, m, N, fast, G.alloc_work(m, n, k, N, ct), ct)
        got, _ = _simulate_moduli_shards(opA, opB, m, n, k, A, lda, B, ldb, N, fast, out_dtype, ct, world)
        torch.cuda.synchronize()
        assert _same(got, ref), dict(case=case, types=ta + tb, m=m, n=n, k=k, N=N, W=world, fast=fast, op=(opA, opB))


def test_output_blocks_fast_mode_same_bits():
    """fast mode: C blocks of a 2 x 3 rank grid, each from its rows of A and columns of B through plain gemm calls
    on offset operands (bench.py's output-block variant), assemble to the single call's bits"""
    import torch
    import gemmul8 as G
    from gemmul8 import dist as GD
    m, n, k, N = 700, 900, 500, 14
    A = G.randmat(m, k, torch.float64, 0.5, 123456)  # column-major, op N
    B = G.randmat(k, n, torch.float64, 0.5, 654321)
    ref = torch.empty((n, m), dtype=torch.float64, device="cuda")
    G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, ref, m, N, True, G.alloc_work(m, n, k, N))
    out = torch.full_like(ref, float("nan"))
    for a0, a1 in GD.blocks(m, 2):
        for b0, b1 in GD.blocks(n, 3):
            Cb = torch.empty((b1 - b0, a1 - a0), dtype=torch.float64, device="cuda")
            G.gemm(G.OP_N, G.OP_N, a1 - a0, b1 - b0, k, 1.0, A[:, a0:], m, B[b0:], k, 0.0, Cb, a1 - a0, N, True,
                   G.alloc_work(a1 - a0, b1 - b0, k, N))
            out[b0:b1, a0:a1] = Cb
    torch.cuda.synchronize()
    assert _same(out, ref)
