"""gemmul8.dist -- one emulated GEMM sharded over the GPUs of a node.

One process per GPU; torch.distributed with the "nccl" backend (RCCL over xGMI on ROCm).
The reference has no multi-GPU path; both partitions here return results bit-identical to
the single-GPU ``gemmul8.gemm`` on the same inputs.

``matmul_rows``    rank r owns a row block of C = A @ B and computes every modulus for it
                   from its own rows of A and the full (replicated) B.  The shift of a row of
                   A depends only on that row and the shifts of B's columns only on B, so the
                   block equals the matching rows of the single-GPU result.  Nothing crosses
                   the fabric on the data path in fast mode; the blocks can optionally be
                   collected on the root (one P2P receive per rank).  Accurate mode derives
                   B's column shifts from the int8 bound product over ALL rows of A, so the
                   ranks combine those column maxima (n int32) with one MAX all-reduce before
                   encoding.  This is the partition bench.py scales.
``matmul_moduli``  rank r owns the moduli [j0, j1): it computes the shifts (cheap, HBM-bound),
                   the slices and the residue planes of its moduli only, sending each plane as
                   soon as its product is launched (the send overlaps the next plane's product),
                   to the root, which receives every rank's planes concurrently (each sender on
                   its own xGMI link) into its workspace and runs the CRT over all N planes.
                   Bytes moved: (N - N_root) * m * n, one byte per residue.  The alternative of
                   reducing partial FP64 CRT sums would move 16 bytes per element per rank and
                   reorder the double-double low-word sum, so it is not used.

The compute steps go through an ``ops`` object (default: ``HipOps``, the native library);
tests substitute a CPU implementation to exercise the communication pattern under gloo.
"""
import torch
import torch.distributed as dist

from . import (OP_T, REAL_DEFAULT, COMPLEX_BIG_MATRIX_ENCODE, alloc_work, gemm, split, split_bound, products,
               recombine, residue_planes)


def moduli_partition(num_moduli, world):
    """Contiguous, balanced moduli ranges [(j0, j1)] per rank (ranks beyond num_moduli get empty ranges)."""
    base, extra = divmod(num_moduli, world)
    out, j = [], 0
    for r in range(world):
        cnt = base + (1 if r < extra else 0)
        out.append((j, j + cnt))
        j += cnt
    return out


def row_partition(m, world, align=256):
    """Row blocks [(r0, r1)] per rank, in multiples of `align` rows (the MFMA tile) except the last."""
    tiles = (m + align - 1) // align
    base, extra = divmod(tiles, world)
    out, t = [], 0
    for r in range(world):
        cnt = base + (1 if r < extra else 0)
        out.append((min(t * align, m), min((t + cnt) * align, m)))
        t += cnt
    return out


class HipOps:
    """Native compute steps on the current CUDA (HIP) device and stream."""

    def full(self, A, B, num_moduli, fastmode, out_dtype):
        m, k = A.shape
        n = B.shape[1]
        Ct = torch.empty((n, m), dtype=out_dtype, device=A.device)
        if A.is_complex():
            work = alloc_work(m, n, k, num_moduli, COMPLEX_BIG_MATRIX_ENCODE, A.device)
            gemm(0, 0, m, n, k, 1.0, A.t().contiguous(), m, B.t().contiguous(), k, 0.0, Ct, m, num_moduli, fastmode,
                 work, COMPLEX_BIG_MATRIX_ENCODE)
        else:
            work = alloc_work(m, n, k, num_moduli, REAL_DEFAULT, A.device)
            gemm(OP_T, OP_T, m, n, k, 1.0, A, k, B, n, 0.0, Ct, m, num_moduli, fastmode, work)
        return Ct.t()

    def row_bound(self, A, B, num_moduli, out_dtype):
        """Accurate mode: bound product of this row block -> (colmax int32 [n] in the workspace, state)."""
        if A.is_complex():
            raise NotImplementedError("accurate mode covers real operands")
        m, k = A.shape
        n = B.shape[1]
        work = alloc_work(m, n, k, num_moduli, REAL_DEFAULT, A.device)
        _, colmax = split_bound(OP_T, OP_T, m, n, k, A, k, B, n, num_moduli, work, out_dtype)
        return colmax, {"A": A, "B": B, "N": num_moduli, "work": work, "dtype": out_dtype}

    def finish_rows(self, st):
        A, B, N, work = st["A"], st["B"], st["N"], st["work"]
        m, k = A.shape
        n = B.shape[1]
        Ct = torch.empty((n, m), dtype=st["dtype"], device=A.device)
        split(OP_T, OP_T, m, n, k, A, k, B, n, N, False, work, st["dtype"], bound_ready=True)
        products(m, n, k, N, work)
        recombine(m, n, k, N, 1.0, 0.0, Ct, m, work)
        return Ct.t()

    def begin(self, A, B, num_moduli, fastmode, out_dtype, j0, j1, need_shifts):
        """Shifts + slices of moduli [j0, j1) (no products yet) -> state for product() / finish()."""
        if A.is_complex():
            raise NotImplementedError("modulus sharding covers real operands")
        m, k = A.shape
        n = B.shape[1]
        work = alloc_work(m, n, k, num_moduli, REAL_DEFAULT, A.device)
        st = {"m": m, "n": n, "k": k, "N": num_moduli, "work": work, "dtype": out_dtype, "device": A.device}
        if j1 > j0:
            split(OP_T, OP_T, m, n, k, A, k, B, n, num_moduli, fastmode, work, out_dtype, j0, j1)
        elif need_shifts:  # a root that owns no modulus still needs the shifts (one unused slice plane)
            split(OP_T, OP_T, m, n, k, A, k, B, n, num_moduli, fastmode, work, out_dtype, 0, 1)
        return st

    def product(self, st, j):
        """Residue plane j (one launch on the current stream) -> its uint8 [plane] view."""
        products(st["m"], st["n"], st["k"], st["N"], st["work"], j, j + 1)
        return residue_planes(st["work"], st["m"], st["n"], st["k"], st["N"], j, j + 1)[0]

    def all_planes(self, st):
        return residue_planes(st["work"], st["m"], st["n"], st["k"], st["N"])

    def sync(self):
        torch.cuda.current_stream().synchronize()

    def finish(self, st):
        m, n = st["m"], st["n"]
        Ct = torch.empty((n, m), dtype=st["dtype"], device=st["device"])
        recombine(m, n, st["k"], st["N"], 1.0, 0.0, Ct, m, st["work"])
        return Ct.t()


def _group_info(group):
    return dist.get_rank(group), dist.get_world_size(group)


def matmul_rows(A_local, B, num_moduli=14, fastmode=True, out_dtype=None, group=None, gather=False, root=0,
                ops=None):
    """C_local = A_local @ B on this rank (A_local: this rank's rows, B replicated).

    With gather=True the root returns the full C (rows concatenated in rank order) and the
    other ranks return None."""
    ops = ops or HipOps()
    out_dtype = out_dtype or torch.promote_types(A_local.dtype, B.dtype)
    rank, world = _group_info(group)
    if fastmode or world == 1:
        C_local = ops.full(A_local, B, num_moduli, fastmode, out_dtype)
    else:
        colmax, st = ops.row_bound(A_local, B, num_moduli, out_dtype)
        ops.sync()
        dist.all_reduce(colmax, op=dist.ReduceOp.MAX, group=group)
        C_local = ops.finish_rows(st)
    if not gather:
        return C_local
    rows = torch.tensor([A_local.shape[0]], dtype=torch.int64, device=A_local.device if A_local.is_cuda else "cpu")
    sizes = [torch.zeros_like(rows) for _ in range(world)]
    dist.all_gather(sizes, rows, group=group)
    sizes = [int(s.item()) for s in sizes]
    ops.sync()
    groot = dist.get_global_rank(group, root) if group is not None else root
    if rank != root:
        dist.send(C_local.contiguous(), dst=groot, group=group)
        return None
    parts = []
    reqs = []
    for r in range(world):
        if r == root:
            parts.append(C_local)
            continue
        buf = torch.empty((sizes[r], C_local.shape[1]), dtype=C_local.dtype, device=C_local.device)
        src = dist.get_global_rank(group, r) if group is not None else r
        reqs.append(dist.irecv(buf, src=src, group=group))
        parts.append(buf)
    for q in reqs:
        q.wait()
    return torch.cat(parts, 0)


def matmul_moduli(A, B, num_moduli=14, fastmode=True, out_dtype=None, group=None, root=0, ops=None):
    """C = A @ B with the moduli sharded over the ranks of `group` (A, B replicated).

    Each rank computes its planes one modulus at a time and sends each as soon as it is launched:
    with RCCL the send of plane j runs on the communication stream behind the products of plane j
    while the products of plane j + 1 run, and the root receives every rank's planes concurrently
    (one xGMI link per sender) while computing its own.  Returns C on the root, None elsewhere."""
    ops = ops or HipOps()
    out_dtype = out_dtype or torch.promote_types(A.dtype, B.dtype)
    rank, world = _group_info(group)
    parts = moduli_partition(num_moduli, world)
    j0, j1 = parts[rank]
    # the gloo backend reads device tensors without waiting on the compute stream
    host_sync = dist.get_backend(group) != "nccl"
    st = ops.begin(A, B, num_moduli, fastmode, out_dtype, j0, j1, rank == root)
    groot = dist.get_global_rank(group, root) if group is not None else root
    if rank != root:
        reqs = []
        for j in range(j0, j1):
            plane = ops.product(st, j)
            if host_sync:
                ops.sync()
            reqs.append(dist.isend(plane, dst=groot, group=group))
        for q in reqs:
            q.wait()
        return None
    allp = ops.all_planes(st)
    reqs = []
    for r in range(world):
        a, b = parts[r]
        if r == root:
            continue
        src = dist.get_global_rank(group, r) if group is not None else r
        for j in range(a, b):  # one receive per plane, in the sender's order
            reqs.append(dist.irecv(allp[j], src=src, group=group))
    for j in range(j0, j1):
        ops.product(st, j)
    for q in reqs:
        q.wait()
    return ops.finish(st)
