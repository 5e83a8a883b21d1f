"""gemmul8.dist -- one emulated GEMM sharded over the GPUs of a node.

One process per GPU; torch.distributed with the "nccl" backend (RCCL over xGMI on ROCm).
The reference has no multi-GPU path; its per-modulus loop (GEMMul8/src/gemmul8.cu:259-275: one
int8 GEMM + one conversion per modulus) is the axis that shards.  Both partitions here return
results bit-identical to the single-GPU ``gemmul8.gemm`` on the same inputs.

``gemm_moduli`` / ``matmul_moduli``   (the cfg3 partition; strong scaling of ONE product)
    The work units are (modulus j, column block of C): N * cb units with cb = W / gcd(N, W)
    column blocks per modulus, N / gcd(N, W) units per rank -- an equal share of the MACs on
    every rank for any N and W (14 moduli over 8 GPUs: 7 quarter-planes each, where whole
    planes would give 2,2,2,2,2,2,1,1).  Per call:
      1. shifts: rank r computes the shifts of its row block of op(A) and its column block of
         op(B) only (1/W of the stats pass) and the ranks all-gather the int16 vectors
         (accurate mode: sft0, then the int8 bound product of its column block and one MAX
         all-reduce of the row / column maxima);
      2. slices of the moduli its units touch (gemmul8_split, SHIFTS_READY / BOUND_READY);
      3. the products of its units (gemmul8_products_cols), cut at the output-column owners'
         boundaries: first the pieces other ranks own, then its own (ShardPlan._schedule);
      4. exchange: rank s owns the CRT of the output column block s, so every unit's residue
         columns go to the owners of those columns.  A column range of a column-major residue
         plane is one contiguous byte run, sent straight from the workspace into the owner's
         workspace at the same offset (no packing).  Stage t's transfers are one grouped P2P
         call posted right after the rank's t-th product launch: RCCL runs them on its own
         stream behind that launch while the next product runs on the compute stream, and the
         last launches (the rank's own columns) send nothing, so the final transfers overlap them;
      5. CRT of its output columns (gemmul8_recombine_cols).
    C stays distributed by column blocks (``gather=True`` collects it on the root).  Bytes per
    rank: N * m * n / W residue bytes received (one byte per residue and modulus of its columns,
    minus what it produced itself) -- at 16384^2, N = 14, W = 8: 0.47 GB per rank, spread over
    the 7 xGMI links, against 16 B per element per rank (4.3 GB) for reducing partial FP64 CRT
    sums (which would also reorder the double-double low-word sum) or 3.2 GB into one root for
    gathering the planes there.

``gemm_moduli_grid``   (the 2-D unit grid: moduli x row blocks x column blocks; fast mode)
    H row blocks of G = W / H ranks, each row block a gemm_moduli over its own sub-group: a rank reads 1/H
    of op(A) instead of all of it and exchanges residues with the G - 1 ranks of its row block only.

``matmul_rows``    rank r owns a row block of C = A @ B and computes every modulus for it
    from its own rows of A and the full (replicated) B.  The shift of a row of A depends only
    on that row and the shifts of B's columns only on B, so the block equals the matching rows
    of the single-GPU result.  Nothing crosses the fabric on the data path in fast mode.
    Accurate mode derives B's column shifts from the int8 bound product over ALL rows of A, so
    the ranks combine those column maxima (n int32) with one MAX all-reduce before encoding.

The compute steps go through an ``ops`` object (default: the native library); tests substitute
a CPU implementation to exercise the communication pattern under gloo.

Workspaces.  The native ops keep the workspaces of the last ``WORKSPACE_CACHE`` shapes (default 2,
least recently used evicted) so that a repeated call allocates only its output; at cfg3 one workspace
is 11.5 GiB.  The default ops objects are per host thread, so two threads never share a workspace;
one ops object serves one call at a time.  ``release_workspaces()`` frees every cached workspace of
the calling thread's default ops (and of any ops objects passed to it).

Fail-fast controls (environment):
    GEMMUL8_DIST_SIDE_STREAM=0   post every transfer stage from the compute stream (default 1: the
                                 receive-only stages from a side stream; ``side_stream_enabled()``)
and ``StageWatchdog``, which ends the process with a message naming the stage and the peers in flight
when a host phase outlives its limit (bench.py arms it around every multi-rank phase).
"""
import collections
import functools
import math
import os
import sys
import threading
import time
import weakref

import torch
import torch.distributed as dist

from . import (OP_N, OP_T, REAL_DEFAULT, COMPLEX_BIG_MATRIX_ENCODE, alloc_work, gemm, layout, split, split_bound,
               products, recombine, shard_stats, shard_bound, crt_partial, crt_finish)

__all__ = ["OP_N", "OP_T", "REAL_DEFAULT", "COMPLEX_BIG_MATRIX_ENCODE", "ShardPlan", "HipShardOps", "HipOps", "blocks",
           "moduli_partition", "row_partition", "gemm_moduli", "gemm_moduli_planes_to_root", "matmul_moduli",
           "matmul_rows", "release_workspaces", "side_stream_enabled", "StageWatchdog", "progress",
           "gemm_moduli_reduce", "gemm_moduli_grid", "grid_groups", "release_grid_groups"]

TILE = 256  # product tile edge: column blocks of the product units start at multiples of it
WORKSPACE_CACHE = 2  # workspaces (shapes) kept per native ops object


def side_stream_enabled():
    """GEMMUL8_DIST_SIDE_STREAM (default 1): receive-only transfer stages posted from a side stream"""
    return os.environ.get("GEMMUL8_DIST_SIDE_STREAM", "1") != "0"


# ------------------------------------------------------------------------------------------------
# progress record + watchdog (fail fast instead of waiting for the communicator's own timeout)
# ------------------------------------------------------------------------------------------------
_PROGRESS = {"call": 0, "stage": "idle", "detail": "", "t": time.monotonic()}
_PROGRESS_LOCK = threading.Lock()


def progress(stage, detail=""):
    """record the host step this rank is at (what the watchdog reports if the rank stalls)"""
    with _PROGRESS_LOCK:
        _PROGRESS.update(stage=stage, detail=detail, t=time.monotonic())


class StageWatchdog:
    """Ends the process (exit status 3) when an armed phase outlives `limit_s` seconds.

    ``arm(phase)`` starts a phase; ``disarm()`` ends it.  The message on stderr names the phase, this rank's
    last recorded step (``progress``: the transfer stage posted last and its peers) and how long ago it was
    recorded.  The process exits with os._exit from the watchdog thread: no exec, nothing restarted.
    ``arm(phase, on_fire)`` makes the phase optional (work after the measurement): when it outlives the limit,
    ``on_fire(message)`` runs on the watchdog thread (bench.py: rank 0 prints its line with what it has
    measured) and the process exits with status 0, so a stuck extra does not void the measurement."""

    def __init__(self, limit_s, rank=0, out=None, exit=True):
        self.limit_s, self.rank, self.out = float(limit_s), rank, out or sys.stderr
        self._phase, self._since, self._on_fire = None, 0.0, None
        self._cv = threading.Condition()
        self._stop = False
        self.fired = None  # the message (tests pass exit=False)
        self.exit_status = None  # the status the process exits (or, with exit=False, would exit) with
        self.exit = exit
        self._thr = threading.Thread(target=self._run, name="gemmul8-watchdog", daemon=True)
        self._thr.start()

    def arm(self, phase, on_fire=None):
        with self._cv:
            self._phase, self._since, self._on_fire = phase, time.monotonic(), on_fire
            self._cv.notify()

    def disarm(self):
        with self._cv:
            self._phase = None
            self._cv.notify()

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thr.join()

    def _run(self):
        with self._cv:
            while not self._stop:
                if self._phase is None:
                    self._cv.wait()
                    continue
                left = self._since + self.limit_s - time.monotonic()
                if left > 0:
                    self._cv.wait(timeout=left)
                    continue
                with _PROGRESS_LOCK:
                    p = dict(_PROGRESS)
                msg = (f"gemmul8 watchdog: rank {self.rank} stuck in phase '{self._phase}' for more than "
                       f"{self.limit_s:.0f} s; last step: call {p['call']} {p['stage']} {p['detail']} "
                       f"({time.monotonic() - p['t']:.1f} s ago)")
                self.fired = msg
                print(msg, file=self.out, flush=True)
                self.exit_status = 3
                if self._on_fire is not None:
                    self.exit_status = 0
                    try:
                        self._on_fire(msg)
                    except Exception as e:  # the exit below must happen whatever the report does
                        print(f"gemmul8 watchdog: report failed: {type(e).__name__}: {e}", file=self.out, flush=True)
                if self.exit:
                    os._exit(self.exit_status)
                self._phase = None


def blocks(n, parts, align=TILE):
    """[(b0, b1)] * parts: equal blocks of ceil(n / align / parts) * align, the last ones shorter or empty."""
    tiles = -(-n // align) if n else 0
    chunk = -(-tiles // parts) * align if tiles else 0
    return [(min(i * chunk, n), min((i + 1) * chunk, n)) for i in range(parts)]


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


class ShardPlan:
    """Who computes what in gemm_moduli (every rank builds the same plan).

    order        how the N * cb units are dealt out in runs of N / g: "moduli" (modulus-major: a rank's units
                 span about N / W moduli and every column block, so its residue columns go to all W - 1 peers,
                 one W-th each) or "columns" (column-block-major: a rank's units are N / g moduli of ONE column
                 block, so it reads and encodes only that block of op(B), but the moduli it encodes for the
                 whole of op(A) grow to N / g, and its remote columns all go to the g - 1 other owners of the
                 block -- one peer at W = 8, N = 14)
    units[r]     rank r's (modulus, c0, c1) product units
    cols[r]      rank r's output columns (its CRT, and the columns of op(B) whose shifts it computes)
    rows[r]      the rows of op(A) whose shifts rank r computes
    launches[r]  rank r's product launches (j0, j1, c0, c1): its units cut at the output-column owners'
                 boundaries; the pieces other ranks own first (consecutive columns of one modulus merged
                 into one launch, each launch's transfers posted right behind it), then the pieces it owns
                 itself (one launch over several moduli where they share the columns), which need no
                 transfer -- so the last transfers run under those products instead of after them
    mods[r]      the moduli range [j0, j1) whose slices rank r encodes
    """

    def __init__(self, m, n, num_moduli, world, align=TILE, order="moduli"):
        if order not in ("moduli", "columns"):
            raise ValueError(f"unit order {order!r}: 'moduli' or 'columns'")
        self.m, self.n, self.N, self.world, self.order = m, n, num_moduli, world, order
        g = math.gcd(num_moduli, world)
        self.col_blocks = world // g  # column blocks per modulus
        pcols = blocks(n, self.col_blocks, align)
        if order == "moduli":
            units = [(j, c0, c1) for j in range(num_moduli) for (c0, c1) in pcols]
        else:  # runs of N / g units never straddle a column block (N / g divides N), so moduli stay contiguous
            units = [(j, c0, c1) for (c0, c1) in pcols for j in range(num_moduli)]
        per = len(units) // world  # = N / g
        self.units = [[u for u in units[r * per:(r + 1) * per] if u[2] > u[1]] for r in range(world)]
        self.cols = blocks(n, world, align)
        self.rows = blocks(m, world, align)
        self.launches = [self._schedule(r) for r in range(world)]
        self.mods = [((us[0][0], us[-1][0] + 1) if us else (0, 0)) for us in self.units]
        self.stages = max((len(x) for x in self.launches), default=0)

    def owners(self, c0, c1):
        """[(owner, lo, hi)]: the output-column owners of the columns [c0, c1)"""
        return [(s, max(c0, s0), min(c1, s1)) for s, (s0, s1) in enumerate(self.cols) if max(c0, s0) < min(c1, s1)]

    def _schedule(self, r):
        pieces = [(j, lo, hi, s) for j, c0, c1 in self.units[r] for s, lo, hi in self.owners(c0, c1)]
        remote, local = [], []
        for j, lo, hi, s in pieces:
            if s != r:  # one modulus per launch, consecutive columns merged
                if remote and remote[-1][0] == j and remote[-1][3] == lo:
                    remote[-1] = (j, j + 1, remote[-1][2], hi)
                else:
                    remote.append((j, j + 1, lo, hi))
            else:  # the same columns over consecutive moduli merged
                if local and local[-1][1] == j and local[-1][2:] == (lo, hi):
                    local[-1] = (local[-1][0], j + 1, lo, hi)
                else:
                    local.append((j, j + 1, lo, hi))
        return remote + local

    def sends(self, r, t):
        """[(dst, j, c0, c1)]: residue column runs rank r sends after its launch t"""
        if t >= len(self.launches[r]):
            return []
        j0, j1, a, b = self.launches[r][t]
        return [(s, j, lo, hi) for j in range(j0, j1) for s, lo, hi in self.owners(a, b) if s != r]

    def recvs(self, r, t):
        """[(src, j, c0, c1)]: residue column runs rank r receives in stage t"""
        out = []
        for q in range(self.world):
            if q != r:
                out += [(q, j, a, b) for (s, j, a, b) in self.sends(q, t) if s == r]
        return out


@functools.lru_cache(maxsize=64)
def _plan(m, n, num_moduli, world, align, order="moduli"):
    return ShardPlan(m, n, num_moduli, world, align, order)


# ------------------------------------------------------------------------------------------------
# native compute steps
# ------------------------------------------------------------------------------------------------
class _WorkCache:
    """workspaces per key, reused across calls (no workspace allocation in a timed loop); at most `cap`
    workspace entries are kept, the least recently used one is dropped first (other entries: unbounded)"""

    def __init__(self, cap=None):
        self._d = collections.OrderedDict()
        self.cap = cap

    def get(self, key, make):
        t = self._d.get(key)
        if t is None:
            if key[0] == "work":
                cap = WORKSPACE_CACHE if self.cap is None else self.cap
                works = [kk for kk in self._d if kk[0] == "work"]
                for kk in works[:max(0, len(works) - cap + 1)]:
                    del self._d[kk]  # (released before the new one is allocated)
            t = self._d[key] = make()
        else:
            self._d.move_to_end(key)
        return t

    def keys(self):
        return list(self._d)

    def clear(self):
        self._d.clear()


class HipShardOps:
    """Native steps of gemm_moduli on the current CUDA (HIP) device and stream."""

    def __init__(self):
        self.cache = _WorkCache()

    def prepare(self, opA, opB, m, n, k, A, lda, B, ldb, N, fast, out_dtype, ctype):
        dev = A.device
        work = self.cache.get(("work", m, n, k, N, ctype, dev), lambda: alloc_work(m, n, k, N, ctype, dev))
        L = layout(m, n, k, N, ctype)
        return {"args": (opA, opB, m, n, k, A, lda, B, ldb, N), "fast": fast, "dtype": out_dtype, "ct": ctype,
                "work": work, "L": L, "m": m, "n": n, "k": k, "N": N, "dev": dev}

    def stats(self, st, rows, cols):
        opA, opB, m, n, k, A, lda, B, ldb, N = st["args"]
        shard_stats(opA, opB, m, n, k, A, lda, B, ldb, N, st["fast"], st["work"], st["dtype"], rows, cols, st["ct"])

    def shift_vectors(self, st):
        """the int16 vectors the ranks assemble: fast sftA [m], sftB [n]; accurate sft0 of A's rows / B's columns"""
        L, w, m, n = st["L"], st["work"], st["m"], st["n"]
        if st["fast"]:
            a, b = L["offSftA"], L["offSftB"]
        else:
            a, b = L["offSft0"], L["offSft0"] + 2 * L["bm_pad"]
        return w[a:a + 2 * m].view(torch.int16), w[b:b + 2 * n].view(torch.int16)

    def bound(self, st, cols):
        """accurate mode: bound product of the column block -> the int32 maxima area to MAX-combine"""
        opA, opB, m, n, k, A, lda, B, ldb, N = st["args"]
        shard_bound(opA, opB, m, n, k, A, lda, B, ldb, N, st["work"], st["dtype"], cols, st["ct"])
        L = st["L"]
        o = L["offBound"]
        return st["work"][o:o + 4 * (L["bm_pad"] + -(-n // TILE) * TILE)].view(torch.int32)

    def encode(self, st, j0, j1):
        """slices of moduli [j0, j1); accurate mode also derives the final shifts (j0 == j1: only those)"""
        opA, opB, m, n, k, A, lda, B, ldb, N = st["args"]
        fast = st["fast"]
        split(opA, opB, m, n, k, A, lda, B, ldb, N, fast, st["work"], st["dtype"], j0, j1, st["ct"],
              bound_ready=not fast, shifts_ready=fast)

    def products(self, st, j0, j1, c0, c1):
        products(st["m"], st["n"], st["k"], st["N"], st["work"], j0, j1, st["ct"], cols=(c0, c1))

    def chunks(self, st, j, c0, c1):
        """uint8 views of the residue columns [c0, c1) of plane j (Karatsuba: one per sub-plane)"""
        L, w = st["L"], st["work"]
        base = L["offR"] + j * L["planeR"]
        subs = [s * L["subR"] for s in range(L["nsub"])]
        return [w[base + s + c0 * L["ldr"]:base + s + c1 * L["ldr"]] for s in subs]

    def recombine(self, st, c0, c1):
        m = st["m"]
        Cb = torch.empty((c1 - c0, m), dtype=st["dtype"], device=st["dev"])
        if c1 > c0:
            recombine(m, st["n"], st["k"], st["N"], 1.0, 0.0, Cb, m, st["work"], st["ct"], cols=(c0, c1))
        return Cb

    def partial(self, st, j0, j1):
        """partial CRT sums (C1, C2) of moduli [j0, j1) as a float64 (2, n, m) tensor (zeros for an empty range)"""
        m, n = st["m"], st["n"]
        S = torch.zeros((2, n, m), dtype=torch.float64, device=st["dev"]) if j1 <= j0 else \
            torch.empty((2, n, m), dtype=torch.float64, device=st["dev"])
        if j1 > j0:
            crt_partial(m, n, st["k"], st["N"], st["dtype"], st["work"], j0, j1, S)
        return S

    def finish(self, st, S):
        """C (an (n, m) tensor) from the summed partial CRT sums and the workspace's shifts"""
        m, n = st["m"], st["n"]
        C = torch.empty((n, m), dtype=st["dtype"], device=st["dev"])
        crt_finish(m, n, st["k"], st["N"], 1.0, 0.0, C, m, st["work"], S, out_dtype=st["dtype"])
        return C

    def side_stream(self):
        """a stream with no work of this call on it (receive-only transfer stages are posted from it)"""
        dev = torch.cuda.current_device()
        return self.cache.get(("side", dev), lambda: torch.cuda.Stream(device=dev))

    def sync(self):
        torch.cuda.current_stream().synchronize()


_DEFAULT = threading.local()  # the default ops objects, one set per host thread


def _shard_ops():
    ops = getattr(_DEFAULT, "shard", None)
    if ops is None:
        ops = _DEFAULT.shard = HipShardOps()
    return ops


def _row_ops():
    ops = getattr(_DEFAULT, "rows", None)
    if ops is None:
        ops = _DEFAULT.rows = HipOps()
    return ops


def release_workspaces(*ops_objects):
    """Free the cached workspaces (and side streams) of the calling thread's default ops and of `ops_objects`;
    the next call allocates afresh.  The memory returns to torch's caching allocator
    (torch.cuda.empty_cache() hands it back to the device)."""
    for o in (getattr(_DEFAULT, "shard", None), getattr(_DEFAULT, "rows", None)) + ops_objects:
        if o is not None:
            o.cache.clear()


def _group_info(group):
    return dist.get_rank(group), dist.get_world_size(group)


def _global(group, r):
    return dist.get_global_rank(group, r) if group is not None else r


def _send(t, dst, group):
    """one send posted as a batched P2P op: RCCL matches it against the receiver's batched irecv on the
    group's own communicator whether or not the group was initialised eagerly (a plain dist.send on a lazily
    initialised NCCL group goes over a separate two-rank communicator and never meets a batched receive)"""
    for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, dst, group)]):
        q.wait()


def _allgather_blocks(vecs, blks, rank, group):
    """vec[b0:b1] of every rank's block (blocks(len, W) layout) assembled into every rank's vec, for each
    (vec, blks) pair of the lists -- one all-gather for all of them"""
    chunks = [b[0][1] - b[0][0] for b in blks]
    total = sum(chunks)
    if total == 0:
        return
    mine = vecs[0].new_zeros(total)
    o = 0
    for vec, b, ch in zip(vecs, blks, chunks):
        b0, b1 = b[rank]
        mine[o:o + b1 - b0] = vec[b0:b1]
        o += ch
    parts = [mine.new_empty(total) for _ in blks[0]]
    # moved as bytes: RCCL has no 16-bit integer type
    dist.all_gather([p.view(torch.uint8) for p in parts], mine.view(torch.uint8), group=group)
    allp = torch.stack(parts)  # [rank][total]
    o = 0
    for vec, ch in zip(vecs, chunks):
        if ch:
            vec.copy_(allp[:, o:o + ch].reshape(-1)[:vec.numel()])
        o += ch


def gemm_moduli(opA, opB, m, n, k, A, lda, B, ldb, num_moduli=14, fastmode=True, out_dtype=None,
                computeType=REAL_DEFAULT, group=None, gather=False, root=0, ops=None, align=TILE, trace=None,
                order="moduli"):
    """C = op(A) op(B) (column-major operands, alpha = 1, beta = 0) with the work split over the ranks of
    `group` by (modulus, column block) units; A and B replicated on every rank.

    Returns this rank's output columns [c0, c1) = ShardPlan.cols[rank] as an (c1 - c0, m) tensor (the
    column-major m x (c1 - c0) block), or with gather=True the whole (n, m) C on the root and None elsewhere.
    trace: a list that receives (phase, torch.cuda.Event) pairs recorded on the current stream at the phase
    boundaries (start, shifts, encode, products, exchange, crt).  order: ShardPlan's unit order."""
    ops = ops or _shard_ops()
    out_dtype = out_dtype or torch.promote_types(A.dtype, B.dtype)
    rank, world = _group_info(group)
    plan = _plan(m, n, num_moduli, world, align, order)  # (align: the native products need TILE)
    # the gloo backend reads device tensors without waiting on the compute stream
    host_sync = dist.get_backend(group) != "nccl"
    with _PROGRESS_LOCK:
        _PROGRESS["call"] += 1
    progress("shifts", f"all-gather of {m} + {n} int16 over {world} ranks")
    st = ops.prepare(opA, opB, m, n, k, A, lda, B, ldb, num_moduli, fastmode, out_dtype, computeType)
    c0, c1 = plan.cols[rank]

    def mark(name):
        if trace is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            trace.append((name, ev))

    mark("start")

    # 1. shifts of this rank's rows / columns, assembled on every rank
    ops.stats(st, plan.rows[rank], plan.cols[rank])
    if host_sync:
        ops.sync()
    va, vb = ops.shift_vectors(st)
    _allgather_blocks([va, vb], [plan.rows, plan.cols], rank, group)
    if not fastmode:
        bnd = ops.bound(st, plan.cols[rank])
        if host_sync:
            ops.sync()
        dist.all_reduce(bnd, op=dist.ReduceOp.MAX, group=group)
    mark("shifts")

    # 2. slices of this rank's moduli (accurate mode derives the final shifts here too, from sft0 and the bound
    # maxima: a rank without moduli still needs them for the CRT of its columns)
    j0, j1 = plan.mods[rank]
    progress("encode", f"moduli [{j0}, {j1})")
    if j1 > j0 or not fastmode:
        ops.encode(st, j0, j1)
    mark("encode")

    # 3 + 4. products, each launch followed by the grouped transfers of its residue columns.  RCCL orders
    # a call's transfers behind the work enqueued on the current stream so far: a stage that only
    # receives (its buffers are columns no launch of this rank writes) is posted from a side stream so
    # that it does not wait for this rank's remaining products
    reqs = []
    mine = plan.launches[rank]
    side = None if (host_sync or not side_stream_enabled()) else ops.side_stream()
    if side is not None:
        # ... but after everything enqueued before this call (the previous call's CRT reads these columns)
        side.wait_stream(torch.cuda.current_stream())
    for t in range(plan.stages):
        if t < len(mine):
            progress(f"products stage {t}", "launch (j0, j1, c0, c1) = %s" % (mine[t],))
            ops.products(st, *mine[t])
        sends, recvs = plan.sends(rank, t), plan.recvs(rank, t)
        snd = [dist.P2POp(dist.isend, x, _global(group, dst), group)
               for dst, j, a, b in sends for x in ops.chunks(st, j, a, b)]
        rcv = [dist.P2POp(dist.irecv, x, _global(group, src), group)
               for src, j, a, b in recvs for x in ops.chunks(st, j, a, b)]
        if not snd and not rcv:
            continue
        progress(f"exchange stage {t}", "sends to %s, receives from %s (%s stream)" % (
            sorted({x[0] for x in sends}), sorted({x[0] for x in recvs}),
            "side" if (side is not None and not snd) else "compute"))
        if host_sync:
            ops.sync()
        if snd or side is None:
            reqs += dist.batch_isend_irecv(snd + rcv)
        else:
            with torch.cuda.stream(side):
                reqs += dist.batch_isend_irecv(rcv)
    mark("products")
    progress("exchange wait", f"{len(reqs)} grouped transfer calls")
    for q in reqs:
        q.wait()
    mark("exchange")

    # 5. CRT of this rank's output columns
    progress("crt", f"columns [{c0}, {c1})")
    Cb = ops.recombine(st, c0, c1)
    mark("crt")
    progress("done")
    if not gather:
        return Cb
    if host_sync:
        ops.sync()
    if rank != root:
        if c1 > c0:
            _send(Cb.contiguous(), _global(group, root), group)
        return None
    C = torch.empty((n, m), dtype=out_dtype, device=Cb.device)
    C[c0:c1] = Cb
    # one group: the blocks arrive concurrently, each over its sender's own link
    rq = [dist.P2POp(dist.irecv, C[s0:s1], _global(group, s), group)
          for s, (s0, s1) in enumerate(plan.cols) if s != root and s1 > s0]
    for q in (dist.batch_isend_irecv(rq) if rq else []):
        q.wait()
    return C


def gemm_moduli_planes_to_root(opA, opB, m, n, k, A, lda, B, ldb, num_moduli=14, fastmode=True, out_dtype=None,
                               computeType=REAL_DEFAULT, group=None, root=0, ops=None):
    """SURVEY 8(e) variant (i), kept for comparison with gemm_moduli (bench.py times both): rank r multiplies
    whole moduli [j0, j1) of moduli_partition (14 over 8 ranks: 2,2,2,2,2,2,1,1) with full shifts of its own,
    sends each residue plane to the root as soon as it is produced, and the root runs the CRT of all of C.
    (N - N_root) m n bytes converge on the root; returns C on the root, None elsewhere."""
    ops = ops or _shard_ops()
    out_dtype = out_dtype or torch.promote_types(A.dtype, B.dtype)
    rank, world = _group_info(group)
    host_sync = dist.get_backend(group) != "nccl"
    parts = moduli_partition(num_moduli, world)
    j0, j1 = parts[rank]
    st = ops.prepare(opA, opB, m, n, k, A, lda, B, ldb, num_moduli, fastmode, out_dtype, computeType)
    with _PROGRESS_LOCK:
        _PROGRESS["call"] += 1
    progress("planes to root: shifts / encode", f"moduli [{j0}, {j1})")
    if j1 > j0 or rank == root:  # every shift on every such rank (a root without moduli needs them for the CRT)
        ops.stats(st, (0, m), (0, n))
        if not fastmode:
            ops.bound(st, (0, n))
        if j1 > j0 or not fastmode:  # (accurate: the final shifts even without moduli)
            ops.encode(st, j0, j1)
    groot = _global(group, root)
    if rank != root:
        reqs = []
        for j in range(j0, j1):
            ops.products(st, j, j + 1, 0, n)
            if host_sync:
                ops.sync()
            progress("planes to root: send", f"plane {j} to rank {root}")
            reqs += dist.batch_isend_irecv([dist.P2POp(dist.isend, x, groot, group) for x in ops.chunks(st, j, 0, n)])
        for q in reqs:
            q.wait()
        progress("done")
        return None
    rcv = [dist.P2POp(dist.irecv, x, _global(group, r), group)
           for r, (a, b) in enumerate(parts) if r != root for j in range(a, b) for x in ops.chunks(st, j, 0, n)]
    side = None if host_sync else ops.side_stream()
    reqs = []
    if rcv:
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                reqs = dist.batch_isend_irecv(rcv)
        else:
            reqs = dist.batch_isend_irecv(rcv)
    for j in range(j0, j1):
        ops.products(st, j, j + 1, 0, n)
    progress("planes to root: receive", f"{num_moduli - (j1 - j0)} planes from {world - 1} ranks")
    for q in reqs:
        q.wait()
    C = ops.recombine(st, 0, n)
    progress("done")
    return C


def gemm_moduli_reduce(opA, opB, m, n, k, A, lda, B, ldb, num_moduli=14, fastmode=True, out_dtype=None, group=None,
                       root=0, ops=None):
    """The north star's partition (BASELINE.json): whole moduli per rank (moduli_partition: 14 over 8 ranks
    2,2,2,2,2,2,1,1), every rank its own shifts, residue planes and partial CRT sums (C1, C2) of its moduli, ONE
    RCCL sum-reduce of the two FP64 m x n planes to the root, and the root's finishing CRT (include/gemmul8_c.h
    gemmul8_crt_partial / gemmul8_crt_finish).  Real outputs, alpha = 1, beta = 0.  Not bit-identical to the
    single call; the bound depends on the moduli level (include/gemmul8_c.h): two-level moduli (f64 output,
    N >= 8) and f64 N <= 5 sum C1 exactly in any order, only C2's rounded sum is reordered (C within 2^-40 of
    max |C|); f64 N = 6, 7 round C1 = sum NMi_i r_i beyond 2^53 in the reduce's order (within 2^-26 of max |C|);
    float output is one-level at every N (within 2^-19 of max |C|).  The reduce moves 16 B per element per rank
    (4.3 GB at cfg3) against gemm_moduli's residue exchange (N m n / W bytes received per rank, 0.47 GB).  Kept
    for comparison (bench.py times it).  Returns C (n, m) on the root, None elsewhere."""
    # argument errors before any collective is posted (a failure inside the native calls could leave the
    # other ranks waiting in the reduce)
    if A.is_complex() or B.is_complex():
        raise ValueError("gemm_moduli_reduce: real operands only (the partial CRT sums have no complex form)")
    if out_dtype is not None and out_dtype not in (torch.float32, torch.float64):
        raise ValueError(f"gemm_moduli_reduce: out_dtype must be float32 or float64, not {out_dtype}")
    ops = ops or _shard_ops()
    out_dtype = out_dtype or torch.promote_types(A.dtype, B.dtype)
    rank, world = _group_info(group)
    host_sync = dist.get_backend(group) != "nccl"
    j0, j1 = moduli_partition(num_moduli, world)[rank]
    st = ops.prepare(opA, opB, m, n, k, A, lda, B, ldb, num_moduli, fastmode, out_dtype, REAL_DEFAULT)
    with _PROGRESS_LOCK:
        _PROGRESS["call"] += 1
    progress("reduce: shifts / encode", f"moduli [{j0}, {j1})")
    ops.stats(st, (0, m), (0, n))
    if not fastmode:
        ops.bound(st, (0, n))
    if j1 > j0 or not fastmode:
        ops.encode(st, j0, j1)
    if j1 > j0:
        ops.products(st, j0, j1, 0, n)
    S = ops.partial(st, j0, j1)
    if host_sync:
        ops.sync()
    progress("reduce: sum of partial CRT sums", f"2 x {m} x {n} f64 to rank {root}")
    dist.reduce(S, dst=_global(group, root), op=dist.ReduceOp.SUM, group=group)
    if rank != root:
        progress("done")
        return None
    C = ops.finish(st, S)
    progress("done")
    return C


_GRID_GROUPS = {}


def grid_groups(world, row_blocks, group=None):
    """The sub-groups of gemm_moduli_grid: row block h owns the ranks [h G, (h + 1) G) of `group`, G = W / H.
    Created once per (group, W, H), by every rank of `group`, all of them in the same order.

    dist.new_group is collective over the default (WORLD) group unless use_local_synchronization=True: with
    `group` the WORLD group (or None) every process enters it, as required; with a smaller parent group the
    processes outside it never call here, so the sub-groups are created with local synchronization (only the
    members of each sub-group synchronise; a rank of `group` outside a sub-group gets the non-member handle)."""
    # checked against the parent group object itself (the default group: the current WORLD, so a re-initialised
    # process group gets new sub-groups), held by a weak reference: a process group kept alive past
    # destroy_process_group is torn down at interpreter exit, where gloo's threads abort the process
    wgroup = getattr(getattr(dist, "group", None), "WORLD", None)
    base = group if group is not None else wgroup
    # (the global rank is part of the key only for ranks simulated as threads of one process, tests/fake_nccl.py:
    # every rank must enter the creation itself)
    key = (id(base), world, row_blocks, dist.get_rank())
    hit = _GRID_GROUPS.get(key)
    if hit is None or hit[0]() is not base:
        G = world // row_blocks
        ranks = [_global(group, r) for r in range(world)]
        ref = weakref.ref(base) if base is not None else (lambda: None)
        kw = {} if base is wgroup else {"use_local_synchronization": True}
        hit = _GRID_GROUPS[key] = (ref, [dist.new_group(ranks[h * G:(h + 1) * G], **kw) for h in range(row_blocks)])
    return hit[1]


def release_grid_groups():
    """Drop the cached sub-groups of gemm_moduli_grid (call before destroy_process_group: the handles are useless
    afterwards and need not outlive it)."""
    _GRID_GROUPS.clear()


def gemm_moduli_grid(opA, opB, m, n, k, A, lda, B, ldb, num_moduli=14, fastmode=True, out_dtype=None,
                     computeType=REAL_DEFAULT, group=None, row_blocks=2, gather=False, root=0, ops=None,
                     align=TILE, order="moduli", trace=None):
    """The 2-D unit grid (moduli x row blocks x column blocks): the W ranks form H row blocks of G = W / H ranks;
    the ranks of row block h run gemm_moduli on its rows of op(A) (rows blocks(m, H)[h], B replicated) over their
    own sub-group, i.e. (modulus, column block) units of that row block and the residue exchange among those G
    ranks only.  A rank's encode reads 1/H of op(A) instead of all of it (gemm_moduli: every rank reads all rows
    of op(A), 2.15 GB of its 4.3 GB at cfg3, W = 8), its exchange stays inside its row block (G - 1 peers), and
    each rank still multiplies 1/W of the MACs.  Fast-mode shifts depend on one row or column each, so every
    block is bit-identical to the single call's.  Fast mode only: the accurate-mode column shifts of op(B) come
    from the bound product over ALL rows of op(A), a reduction across row blocks gemm_moduli does not make.

    Returns this rank's block -- rows blocks(m, H)[h], columns ShardPlan(m_h, n, N, G).cols[rank % G] -- as a
    (c1 - c0, m_h) tensor (column-major), or with gather=True the whole (n, m) C on the root and None
    elsewhere.  A, B: column-major storage as in gemm_moduli (op N: an (k, m) tensor; op T: an (m, k) one).
    trace: as gemm_moduli's, for this rank's row-block call."""
    if not fastmode:
        raise ValueError("gemm_moduli_grid: fast mode only (accurate-mode column shifts span every row block)")
    rank, world = _group_info(group)
    if row_blocks < 1 or world % row_blocks:
        raise ValueError(f"gemm_moduli_grid: {row_blocks} row blocks do not divide {world} ranks")
    if gather and root != 0:
        raise ValueError("gemm_moduli_grid: gather=True collects C on rank 0 of the group")
    out_dtype = out_dtype or torch.promote_types(A.dtype, B.dtype)
    G = world // row_blocks
    h, sub = divmod(rank, G)
    rblocks = blocks(m, row_blocks, align)
    r0, r1 = rblocks[h]
    subgroups = grid_groups(world, row_blocks, group)
    # rows [r0, r1) of op(A): a column range of op(A)'s storage for op N (column-major m x k: the (k, m) tensor's
    # second index), a row range of the (m, k) tensor for op T / C
    Ah = A[:, r0:r1] if opA == OP_N else A[r0:r1]
    mh = r1 - r0
    if mh > 0:
        Cb = gemm_moduli(opA, opB, mh, n, k, Ah, lda, B, ldb, num_moduli, fastmode, out_dtype, computeType,
                         group=subgroups[h], gather=gather, root=0, ops=ops, align=align, trace=trace, order=order)
    elif gather:  # (every rank of an empty row block skips, so its sub-group stays consistent)
        Cb = torch.empty((n, 0), dtype=out_dtype, device=A.device) if sub == 0 else None
    else:
        Cb = torch.empty((0, 0), dtype=out_dtype, device=A.device)
    if not gather:
        return Cb
    # the row blocks' roots (sub-group rank 0) hold their (n, m_h) blocks: to the global root
    host_sync = dist.get_backend(group) != "nccl"
    if host_sync and A.is_cuda:
        torch.cuda.current_stream().synchronize()
    groot = _global(group, root)
    if sub != 0:
        return None
    if rank != root:
        if mh > 0:
            _send(Cb.contiguous(), groot, group)
        return None
    C = torch.empty((n, m), dtype=out_dtype, device=Cb.device)
    bufs, rq = {}, []
    for hh, (a, b) in enumerate(rblocks):
        src = hh * G
        if b <= a:
            continue
        if src == rank:
            C[:, a:b] = Cb
            continue
        bufs[hh] = torch.empty((n, b - a), dtype=out_dtype, device=Cb.device)
        rq.append(dist.P2POp(dist.irecv, bufs[hh], _global(group, src), group))
    for q in (dist.batch_isend_irecv(rq) if rq else []):
        q.wait()
    for hh, buf in bufs.items():
        a, b = rblocks[hh]
        C[:, a:b] = buf
    return C


def matmul_moduli(A, B, num_moduli=14, fastmode=True, out_dtype=None, group=None, gather=True, root=0, ops=None,
                  align=TILE, order="moduli"):
    """C = A @ B (row-major torch tensors, A, B replicated) sharded over the ranks of `group` (gemm_moduli).

    gather=True: the whole C (m x n) on the root, None elsewhere; gather=False: this rank's column block
    C[:, c0:c1] (c0, c1 = ShardPlan.cols[rank]) as an m x (c1 - c0) tensor, a transposed view of the
    column-major buffer.  The default ops cache this shape's workspace (see the module docstring;
    release_workspaces() frees it)."""
    m, k = A.shape
    n = B.shape[1]
    ct = COMPLEX_BIG_MATRIX_ENCODE if A.is_complex() else REAL_DEFAULT
    # a row-major (m x k) tensor is the column-major k x m matrix: op T on both operands, no copies
    out = gemm_moduli(OP_T, OP_T, m, n, k, A.contiguous(), k, B.contiguous(), n, num_moduli, fastmode, out_dtype, ct,
                      group, gather, root, ops, align, order=order)
    return None if out is None else out.t()


# ------------------------------------------------------------------------------------------------
# row partition
# ------------------------------------------------------------------------------------------------
class HipOps:
    """Native compute steps of matmul_rows on the current CUDA (HIP) device and stream."""

    def __init__(self):
        self.cache = _WorkCache()

    def _work(self, m, n, k, N, ct, dev):
        return self.cache.get(("work", m, n, k, N, ct, dev), lambda: alloc_work(m, n, k, N, ct, dev))

    def full(self, A, B, num_moduli, fastmode, out_dtype):
        m, k = A.shape
        n = B.shape[1]
        Ct = torch.empty((n, m), dtype=out_dtype, device=A.device)
        if A.is_complex():
            ct = COMPLEX_BIG_MATRIX_ENCODE
            gemm(OP_T, OP_T, m, n, k, 1.0, A, k, B, n, 0.0, Ct, m, num_moduli, fastmode,
                 self._work(m, n, k, num_moduli, ct, A.device), ct)
        else:
            gemm(OP_T, OP_T, m, n, k, 1.0, A, k, B, n, 0.0, Ct, m, num_moduli, fastmode,
                 self._work(m, n, k, num_moduli, REAL_DEFAULT, A.device))
        return Ct.t()

    def row_bound(self, A, B, num_moduli, out_dtype):
        """Accurate mode: bound product of this row block -> (colmax int32 [n] in the workspace, state)."""
        m, k = A.shape
        n = B.shape[1]
        ct = COMPLEX_BIG_MATRIX_ENCODE if A.is_complex() else REAL_DEFAULT
        work = self._work(m, n, k, num_moduli, ct, A.device)
        _, colmax = split_bound(OP_T, OP_T, m, n, k, A, k, B, n, num_moduli, work, out_dtype, ct)
        return colmax, {"A": A, "B": B, "N": num_moduli, "work": work, "dtype": out_dtype, "ct": ct}

    def finish_rows(self, st):
        A, B, N, work, ct = st["A"], st["B"], st["N"], st["work"], st["ct"]
        m, k = A.shape
        n = B.shape[1]
        Ct = torch.empty((n, m), dtype=st["dtype"], device=A.device)
        split(OP_T, OP_T, m, n, k, A, k, B, n, N, False, work, st["dtype"], computeType=ct, bound_ready=True)
        products(m, n, k, N, work, computeType=ct)
        recombine(m, n, k, N, 1.0, 0.0, Ct, m, work, ct)
        return Ct.t()

    def sync(self):
        torch.cuda.current_stream().synchronize()


def matmul_rows(A_local, B, num_moduli=14, fastmode=True, out_dtype=None, group=None, gather=False, root=0,
                ops=None):
    """C_local = A_local @ B on this rank (A_local: this rank's rows, B replicated).

    With gather=True the root returns the full C (rows concatenated in rank order) and the
    other ranks return None.  The default ops cache this shape's workspace (see the module docstring;
    release_workspaces() frees it)."""
    ops = ops or _row_ops()
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
    groot = _global(group, root)
    if rank != root:
        if C_local.shape[0]:
            _send(C_local.contiguous(), groot, group)
        return None
    parts = []
    ops_ = []
    for r in range(world):
        if r == root:
            parts.append(C_local)
            continue
        buf = torch.empty((sizes[r], C_local.shape[1]), dtype=C_local.dtype, device=C_local.device)
        if sizes[r]:
            ops_.append(dist.P2POp(dist.irecv, buf, _global(group, r), group))
        parts.append(buf)
    for q in (dist.batch_isend_irecv(ops_) if ops_ else []):  # concurrent, one link per sender
        q.wait()
    return torch.cat(parts, 0)
