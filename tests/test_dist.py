"""Multi-process tests of gemmul8.dist on the CPU with the gloo backend.

The communication pattern (row blocks gathered on the root; moduli sharded with residue
planes sent to the root) runs for real across 2 and 3 processes; the compute steps are the
CPU oracle (test infrastructure) injected through the ``ops`` hook, so the result must be
bit-identical to one oracle call on the whole problem.  The GPU variant (HipOps over RCCL)
is covered in test_gpu_phases.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class OracleOps:
    """CPU stand-in for gemmul8.dist.HipOps (tests only)."""

    def __init__(self):
        from oracle import oracle as O
        self.O = O

    def full(self, A, B, N, fast, out_dtype):
        npt = torch.empty((), dtype=out_dtype).numpy().dtype
        C = self.O.gemm(A.numpy(), B.numpy(), N, fast, out_dtype=npt)
        return torch.from_numpy(np.ascontiguousarray(C))

    def row_bound(self, A, B, N, out_dtype):
        *_, colmax = self.O.scaling(A.numpy(), B.numpy(), N, False, want_colmax=True)
        colmax = torch.from_numpy(colmax)
        return colmax, {"A": A, "B": B, "N": N, "colmax": colmax, "dtype": out_dtype}

    def finish_rows(self, st):
        A8, B8, sA, sB = self.O.scaling(st["A"].numpy(), st["B"].numpy(), st["N"], False,
                                        colmax_in=st["colmax"].numpy())
        npt = torch.empty((), dtype=st["dtype"]).numpy().dtype
        C = self.O.crt(self.O.residues(A8, B8), sA, sB, npt)
        return torch.from_numpy(np.ascontiguousarray(C))

    def sync(self):
        pass


def _fma1(a, b, c):
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def fma(a, b, c):
    """element-wise correctly rounded a * b + c (the finishing CRT cancels q * M against C1: a separately
    rounded product would lose it)"""
    return np.frompyfunc(_fma1, 3, 1)(*np.broadcast_arrays(np.float64(a), np.float64(b), np.float64(c))).astype(np.float64)


def crt_tables():
    """the CRT constants of mixed-gemmul8_amd/csrc/oz2_tables.inc (hex floats) as numpy arrays"""
    import re
    txt = open(os.path.join(ROOT, "mixed-gemmul8_amd", "csrc", "oz2_tables.inc")).read()

    def arr(name):
        body = re.search(r"\b" + name + r"\[[^=]*=\s*\{(.*?)\};", txt, re.S).group(1)
        return [float.fromhex(x) if "0x" in x else float(x) for x in re.findall(r"-?0x[0-9a-fA-Fp.+-]+|-?\d+\.\d+", body)]
    numM = [int(x) for x in re.search(r"oz2_numM\[19\] = \{(.*?)\}", txt).group(1).split(",")]
    nmi1 = np.zeros((19, 20))
    body1 = re.search(r"oz2_NMi_1\[19\]\[20\] = \{(.*?)\};", txt, re.S).group(1)
    for r, row in enumerate(re.findall(r"\{([^{}]*)\}", body1)):
        vals = [float.fromhex(x) for x in re.findall(r"-?0x[0-9a-fA-Fp.+-]+", row)]
        nmi1[r, :len(vals)] = vals
    nmi2 = np.array(arr("oz2_NMi_2")).reshape(13, 20, 2)
    return {"numM": numM, "NMi_1": nmi1, "NMi_2": nmi2, "invM": np.array(arr("oz2_invM")),
            "M_hi": np.array(arr("oz2_M_hi")), "M_lo": np.array(arr("oz2_M_lo"))}


class OracleShardOps:
    """CPU stand-in for gemmul8.dist.HipShardOps (tests only).  The shifts and residues are computed
    in full by the oracle but published only for this rank's rows / columns / units, so the result
    is right only if gemm_moduli's all-gathers and residue exchange deliver every other part."""

    SENTINEL = -32768

    def __init__(self):
        from oracle import oracle as O
        self.O = O

    def prepare(self, opA, opB, m, n, k, A, lda, B, ldb, N, fast, out_dtype, ct):
        # column-major operands: an (x, ld) row-major tensor holds the column-major ld x x matrix
        Acm = A.numpy().T[:lda]
        Bcm = B.numpy().T[:ldb]
        A8, B8, sA, sB = self.O.scaling(Acm, Bcm, N, fast, opA=opA, opB=opB)
        full = self.O.residues(A8, B8)
        npt = torch.empty((), dtype=out_dtype).numpy().dtype
        # fast mode: the published shifts are what the ranks gather; accurate mode gathers sft0 (stood in for by
        # the same values here) and derives the final shifts in encode (the native finalize), on every rank
        return {"sA": sA, "sB": sB, "full": full, "R": torch.zeros(full.shape, dtype=torch.uint8), "fast": fast, "N": N,
                "pA": torch.full((m,), self.SENTINEL, dtype=torch.int16),
                "pB": torch.full((n,), self.SENTINEL, dtype=torch.int16),
                "gA": torch.full((m,), self.SENTINEL, dtype=torch.int16),
                "gB": torch.full((n,), self.SENTINEL, dtype=torch.int16), "dtype": npt}

    def stats(self, st, rows, cols):
        a, b = (st["pA"], st["pB"]) if st["fast"] else (st["gA"], st["gB"])
        a[rows[0]:rows[1]] = torch.from_numpy(st["sA"][rows[0]:rows[1]])
        b[cols[0]:cols[1]] = torch.from_numpy(st["sB"][cols[0]:cols[1]])

    def shift_vectors(self, st):
        return (st["pA"], st["pB"]) if st["fast"] else (st["gA"], st["gB"])

    def bound(self, st, cols):
        return torch.zeros(8, dtype=torch.int32)  # (the oracle derives accurate shifts itself)

    def encode(self, st, j0, j1):
        if not st["fast"]:  # the final shifts, from the assembled sft0 (complete only after the gathers)
            assert int(st["gA"].min()) != self.SENTINEL or st["gA"].numel() == 0
            st["pA"][:] = torch.from_numpy(st["sA"])
            st["pB"][:] = torch.from_numpy(st["sB"])

    def products(self, st, j0, j1, c0, c1):
        st["R"][j0:j1, c0:c1] = torch.from_numpy(st["full"][j0:j1, c0:c1])

    def chunks(self, st, j, c0, c1):
        return [st["R"][j, c0:c1].view(-1)]

    # the reduce partition (gemm_moduli_reduce): numpy restatement of gemmul8_crt_partial / _finish (mul + add
    # where the library fuses: the C2 sums differ in rounding anyway, the tests compare within ulps)
    def partial(self, st, j0, j1):
        T, N = crt_tables(), st["N"]
        numM1 = T["numM"][N - 2] == 1 or st["dtype"] == np.float32
        n, m = st["full"].shape[1:]
        C1, C2 = np.zeros((n, m)), np.zeros((n, m))
        for j in range(j0, j1):
            r = st["R"][j].numpy().astype(np.float64)
            C1 = (T["NMi_1"][N - 2][j] if numM1 else T["NMi_2"][N - 8][j][0]) * r + C1
            if not numM1:
                C2 = T["NMi_2"][N - 8][j][1] * r + C2
        return torch.from_numpy(np.stack([C1, C2]))

    def finish(self, st, S):
        T, N = crt_tables(), st["N"]
        numM1 = T["numM"][N - 2] == 1 or st["dtype"] == np.float32
        C1, C2 = S[0].numpy(), S[1].numpy()
        invM, M1, M2 = T["invM"][N - 2], T["M_hi"][N - 2], T["M_lo"][N - 2]
        if numM1:
            v = fma(-np.rint(C1 * invM), M1, C1)
        else:
            q = -np.rint(fma(C1, invM, C2 * invM))
            v = fma(q, M2, fma(q, M1, C1) + C2)
        sh = st["pB"].numpy().astype(np.int64)[:, None] + st["pA"].numpy().astype(np.int64)[None, :]
        return torch.from_numpy(np.ldexp(v, sh).astype(st["dtype"]))

    def recombine(self, st, c0, c1):
        C = self.O.crt(np.ascontiguousarray(st["R"][:, c0:c1].numpy()), st["pA"].numpy(),
                       np.ascontiguousarray(st["pB"][c0:c1].numpy()), st["dtype"])
        return torch.from_numpy(np.ascontiguousarray(C.T))

    def sync(self):
        pass


def _worker(rank, world, port, case, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mixed-gemmul8_amd")]
    from gemmul8 import dist as GD
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m, n, k, N, fast, dt = case[:6]
        order = case[6] if len(case) > 6 else "moduli"
        rng = np.random.default_rng(7)
        A = ((rng.random((m, k)) - 0.5) * np.exp(rng.standard_normal((m, k)))).astype(dt)
        B = ((rng.random((k, n)) - 0.5) * np.exp(rng.standard_normal((k, n)))).astype(dt)
        ops = OracleOps()
        # small column blocks (align 16) so that every rank owns units and output columns
        Cm = GD.matmul_moduli(torch.from_numpy(A), torch.from_numpy(B), N, fast, ops=OracleShardOps(), align=16,
                              order=order)
        # the column block of this rank without the gather (C stays distributed)
        Cb = GD.matmul_moduli(torch.from_numpy(A), torch.from_numpy(B), N, fast, gather=False, ops=OracleShardOps(),
                              align=16, order=order)
        np.save(os.path.join(outdir, f"block{rank}.npy"), Cb.contiguous().numpy())
        # the north star's partition: whole moduli per rank, partial CRT sums reduced to the root
        if not np.iscomplexobj(A):  # (real outputs only)
            Cr = GD.gemm_moduli_reduce(1, 1, m, n, k, torch.from_numpy(A), k, torch.from_numpy(B), n, N, fast,
                                       ops=OracleShardOps())
            if rank == 0:
                np.save(os.path.join(outdir, "reduce.npy"), Cr.t().contiguous().numpy())
            else:
                assert Cr is None
        # the 2-D unit grid: two row blocks, each a gemm_moduli over its own sub-group (fast mode, even W)
        if fast and world % 2 == 0:
            Cg = GD.gemm_moduli_grid(1, 1, m, n, k, torch.from_numpy(A), k, torch.from_numpy(B), n, N, fast,
                                     ops=OracleShardOps(), row_blocks=2, gather=True, align=16, order=order)
            if rank == 0:
                np.save(os.path.join(outdir, "grid.npy"), Cg.t().contiguous().numpy())
            else:
                assert Cg is None
        # SURVEY 8(e) variant (i): whole moduli per rank, planes gathered on the root
        Cp = GD.gemm_moduli_planes_to_root(1, 1, m, n, k, torch.from_numpy(A), k, torch.from_numpy(B), n, N, fast,
                                           ops=OracleShardOps())
        if rank == 0:
            np.save(os.path.join(outdir, "planes.npy"), Cp.t().contiguous().numpy())
        else:
            assert Cp is None
        r0, r1 = GD.row_partition(m, world, align=16)[rank]
        Cr = GD.matmul_rows(torch.from_numpy(A[r0:r1].copy()), torch.from_numpy(B), N, fast, gather=True, ops=ops)
        if rank == 0:
            np.save(os.path.join(outdir, "moduli.npy"), Cm.contiguous().numpy())
            np.save(os.path.join(outdir, "rows.npy"), Cr.numpy())
        else:
            assert Cm is None and Cr is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [
    (2, (70, 50, 90, 14, True, np.float64)),
    (2, (64, 33, 120, 5, False, np.float64)),
    (3, (100, 40, 64, 14, True, np.float64)),
    (3, (48, 30, 50, 8, True, np.float32)),
    (3, (90, 30, 70, 9, False, np.float64)),
    (4, (100, 70, 64, 14, True, np.float64)),
    (2, (40, 50, 60, 6, True, np.complex128)),
    (8, (120, 300, 64, 14, True, np.float64)),  # the cfg3 plan: 14 moduli, 8 ranks, 7 units each
    (8, (60, 130, 40, 9, False, np.float64)),
    (7, (90, 45, 50, 3, False, np.float64)),   # accurate: rank 1 multiplies no modulus but owns columns
    (3, (40, 50, 61, 7, False, np.complex128)),
    (8, (120, 300, 64, 14, True, np.float64, "columns")),  # column-block-major units: 7 moduli x 1 block each
    (4, (100, 70, 64, 14, False, np.float64, "columns")),
    (3, (48, 30, 50, 9, True, np.complex128, "columns")),
    (3, (64, 40, 80, 7, True, np.float64)),   # one-level moduli, C1 beyond 2^53: the reduce's looser bound
    (2, (50, 30, 70, 6, False, np.float64)),
])
def test_sharded_equals_single_call(tmp_path, world, case):
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True)
    m, n, k, N, fast, dt = case[:6]
    rng = np.random.default_rng(7)
    A = ((rng.random((m, k)) - 0.5) * np.exp(rng.standard_normal((m, k)))).astype(dt)
    B = ((rng.random((k, n)) - 0.5) * np.exp(rng.standard_normal((k, n)))).astype(dt)
    C = O.gemm(A, B, N, fast)
    names = ("moduli", "rows", "planes") + (("grid",) if fast and world % 2 == 0 else ())
    for name in names:
        got = np.load(tmp_path / f"{name}.npy")
        assert got.shape == C.shape
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(C).view(np.uint8)), name
    # the reduce of partial sums: within a few ulp of the single call (C2's summation order differs)
    if not np.iscomplexobj(A):
        got = np.load(tmp_path / "reduce.npy")
        assert got.shape == C.shape and np.isfinite(got).all()
        # (float output: a C sum a few ulp off can round to the neighbouring float; f64 at N = 6, 7: one-level
        # moduli whose C1 = sum NMi r exceeds 2^53 is rounded in the reduce's order, include/gemmul8_c.h)
        tol = 2.0 ** (-19 if got.dtype == np.float32 else -26 if N in (6, 7) else -40)
        assert np.max(np.abs(got - C)) <= tol * np.max(np.abs(C)), np.max(np.abs(got - C))
    from gemmul8.dist import ShardPlan
    for r, (c0, c1) in enumerate(ShardPlan(m, n, N, world, 16, case[6] if len(case) > 6 else "moduli").cols):
        got = np.load(tmp_path / f"block{r}.npy")
        assert got.shape == (m, c1 - c0)
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(C[:, c0:c1]).view(np.uint8)), r


def _grid_parent_worker(rank, world, port, outdir):
    """gemm_moduli_grid over a parent group of ranks 0-3 of a 6-process world: processes 4 and 5
    never call it, so the row-block sub-groups must be created with local synchronization; op N operands (the
    path bench.py times: A[:, r0:r1] is a strided view of the (k, m) storage with lda = m)"""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mixed-gemmul8_amd")]
    from gemmul8 import dist as GD
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m, n, k, N = 90, 70, 50, 12
        rng = np.random.default_rng(11)
        A = (rng.random((m, k)) - 0.5) * np.exp(rng.standard_normal((m, k)))
        B = (rng.random((k, n)) - 0.5) * np.exp(rng.standard_normal((k, n)))
        parent = dist.new_group([0, 1, 2, 3])  # world-collective: every process enters
        if rank < 4:
            At = torch.from_numpy(np.ascontiguousarray(A.T))  # column-major m x k: the (k, m) tensor
            Bt = torch.from_numpy(np.ascontiguousarray(B.T))
            Cg = GD.gemm_moduli_grid(0, 0, m, n, k, At, m, Bt, k, N, True, ops=OracleShardOps(), group=parent,
                                     row_blocks=2, gather=True, align=16)
            if rank == 0:
                np.save(os.path.join(outdir, "grid_parent.npy"), Cg.t().contiguous().numpy())
            else:
                assert Cg is None
            GD.release_grid_groups()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_grid_over_non_world_parent_group(tmp_path):
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    mp.spawn(_grid_parent_worker, args=(6, _free_port(), str(tmp_path)), nprocs=6, join=True)
    m, n, k, N = 90, 70, 50, 12
    rng = np.random.default_rng(11)
    A = (rng.random((m, k)) - 0.5) * np.exp(rng.standard_normal((m, k)))
    B = (rng.random((k, n)) - 0.5) * np.exp(rng.standard_normal((k, n)))
    C = np.ascontiguousarray(O.gemm(A, B, N, True))
    got = np.load(tmp_path / "grid_parent.npy")
    assert got.shape == C.shape and np.array_equal(got.view(np.uint8), C.view(np.uint8))


def test_partitions():
    sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
    from gemmul8.dist import moduli_partition, row_partition
    assert moduli_partition(14, 8) == [(0, 2), (2, 4), (4, 6), (6, 8), (8, 10), (10, 12), (12, 13), (13, 14)]
    assert moduli_partition(3, 4) == [(0, 1), (1, 2), (2, 3), (3, 3)]
    for N in range(2, 21):
        for w in (1, 2, 3, 8):
            p = moduli_partition(N, w)
            assert p[0][0] == 0 and p[-1][1] == N and all(a[1] == b[0] for a, b in zip(p, p[1:]))
            assert max(b - a for a, b in p) - min(b - a for a, b in p) <= 1
    assert row_partition(16384, 8) == [(2048 * r, 2048 * (r + 1)) for r in range(8)]
    rp = row_partition(1000, 3)
    assert rp == [(0, 512), (512, 768), (768, 1000)]
    assert row_partition(100, 4)[-1] == (100, 100)
