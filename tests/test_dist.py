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
        return {"sA": sA, "sB": sB, "full": full, "R": torch.zeros(full.shape, dtype=torch.uint8), "fast": fast,
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
    for name in ("moduli", "rows", "planes"):
        got = np.load(tmp_path / f"{name}.npy")
        assert got.shape == C.shape
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(C).view(np.uint8)), name
    from gemmul8.dist import ShardPlan
    for r, (c0, c1) in enumerate(ShardPlan(m, n, N, world, 16, case[6] if len(case) > 6 else "moduli").cols):
        got = np.load(tmp_path / f"block{r}.npy")
        assert got.shape == (m, c1 - c0)
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(C[:, c0:c1]).view(np.uint8)), r


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
