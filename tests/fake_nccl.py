"""fake_nccl.py -- test infrastructure: a stream-ordered stand-in for torch.distributed's NCCL backend, with the
ranks as threads of one process on one GPU.

Why: gemmul8/dist.py takes a different branch under NCCL than under gloo.  With gloo it synchronises the host
before every transfer (gloo reads device tensors without waiting on the compute stream); with NCCL it posts the
transfers in stream order, receive-only stages from a side stream, and relies on the communication stream's
ordering for buffer reuse across calls.  A one-GPU box cannot run RCCL with more than one rank (RCCL refuses two
ranks on one device), so this module models the part of ProcessGroupNCCL that branch depends on, on real HIP
streams, and the GPU tests run the real native steps through it (tests/test_gpu_dist_streams.py):

- each rank has ONE internal communication stream; every call first makes it wait for the caller's current
  stream (the data dependency ProcessGroupNCCL records at the call), and all of a rank's calls run on it in
  posting order;
- batch_isend_irecv: a receive copies the matching send's tensor (matched per (src, dst) channel in posting
  order, sizes checked) on the receiver's communication stream after the sender's stream reached the call;
  a send completes when its receiver's copy has, so the sender's communication stream waits for that copy;
- all_gather / all_reduce (SUM, MAX) / reduce: every rank's inputs are read after all ranks reached the call,
  outputs are written after all ranks have read;
- synchronous collectives make the caller's current stream wait for their end; a Work's wait() does the same
  for its batch (Work.wait() under ProcessGroupNCCL);
- delay_cycles > 0 puts a bounded GPU spin (torch.cuda._sleep) in front of every received copy, so transfers
  land late.  A consumer that does not wait for them then reads stale columns whenever its stream runs on a
  hardware queue of its own; HIP maps a process's streams onto GPU_MAX_HW_QUEUES (4 here) queues, and two streams
  on one queue run in order, so a missing dependency is caught with high probability, not with certainty;
- drop_receives=True completes receives without copying (the negative control: results must then differ);
- new_group(ranks): sub-groups as ProcessGroupNCCL has them: their own communicator (P2P channels and collective
  sequence per group), peers and roots named by global rank, get_rank / get_world_size / get_global_rank per group.
The host side blocks only to match peers (a send's receiver must have posted before the sender's batch returns,
a receive's sender before the copy is enqueued), which can only deadlock where the stream-ordered NCCL schedule
would.  Every tensor a communication stream touches is recorded on it for the caching allocator.
"""
import collections
import threading
import types

import torch


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self):
        return self.ev.query()


class _Group:
    def __init__(self, gid, ranks):
        self.gid, self.ranks = gid, ranks


class FakeNcclWorld:
    def __init__(self, world, timeout_s=120.0, delay_cycles=0, drop_receives=False):
        self.world = world
        self.timeout_s = timeout_s
        self.delay_cycles = int(delay_cycles)
        self.drop_receives = drop_receives
        self._cv = threading.Condition()
        self._chan = collections.defaultdict(list)       # (src, dst) -> posted sends, in order
        self._recv_next = collections.defaultdict(int)   # (src, dst) -> index of the next receive
        self._coll = collections.defaultdict(dict)       # (group id, sequence number) -> {group rank: payload}
        self._coll_seq = collections.defaultdict(int)    # (group id, rank) -> next sequence number
        self._groups = {}                                # ranks tuple -> _Group (shared by the rank threads)
        self._tls = threading.local()
        self.calls = collections.Counter()               # what the ranks called (tests assert on it)
        self.module = self._make_module()

    # ---- per-thread rank ----
    def enter(self, rank):
        """called first in each rank's thread"""
        torch.cuda.set_device(0)
        self._tls.rank = rank
        self._tls.comm = torch.cuda.Stream()

    @property
    def rank(self):
        return self._tls.rank

    def _wait(self, pred):
        if not self._cv.wait_for(pred, timeout=self.timeout_s):
            raise TimeoutError(f"fake NCCL: rank {self.rank} waited {self.timeout_s} s for a peer")

    def _start(self):
        """the communication stream of this rank, after the caller's current stream"""
        comm = self._tls.comm
        comm.wait_stream(torch.cuda.current_stream())
        return comm

    @staticmethod
    def _event(stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    # ---- groups ----
    def new_group(self, ranks=None, use_local_synchronization=False, **kw):
        """torch.distributed's rule: new_group is collective over the WHOLE world (every process enters it, in
        the same order) unless use_local_synchronization=True, when only the members synchronise and a
        non-member returns at once.  A rank that skips a world-collective creation leaves the others waiting
        (TimeoutError here, a hang under NCCL)."""
        key = tuple(range(self.world)) if ranks is None else tuple(int(r) for r in ranks)
        with self._cv:
            if key not in self._groups:
                self._groups[key] = _Group(len(self._groups) + 1, key)
            g = self._groups[key]
        self.calls["new_group"] += 1
        if not use_local_synchronization:
            self._rendezvous(("new_group", key))  # the world group's sequence: every rank, same order
        elif self.rank in key:
            self._rendezvous(("new_group_local", key), g)
        return g

    def _members(self, group):
        return tuple(range(self.world)) if group is None else group.ranks

    def _grank(self, group):
        m = self._members(group)
        return m.index(self.rank) if self.rank in m else -1

    def _rendezvous(self, payload, group=None):
        """every member's payload of this collective, by group rank (the members call the group's collectives in
        the same order)"""
        gid, size, r = (0 if group is None else group.gid), len(self._members(group)), self._grank(group)
        if r < 0:
            raise RuntimeError(f"fake NCCL: rank {self.rank} is not a member of group {self._members(group)}")
        with self._cv:
            seq = self._coll_seq[(gid, r)]
            self._coll_seq[(gid, r)] += 1
            d = self._coll[(gid, seq)]
            d[r] = payload
            self._cv.notify_all()
            self._wait(lambda: len(d) == size)
            return dict(d)

    def _finish(self, comm, sync=True):
        end = self._event(comm)
        if sync:
            torch.cuda.current_stream().wait_event(end)
        return end

    # ---- point to point ----
    def batch_isend_irecv(self, ops):
        r = self.rank
        self.calls["batch_isend_irecv"] += 1
        comm = self._start()
        ready = self._event(comm)
        mine = []
        with self._cv:
            for op in ops:
                if op.op is self.module.isend:
                    op.tensor.record_stream(comm)
                    e = {"t": op.tensor, "ready": ready, "done": None}
                    self._chan[(0 if op.group is None else op.group.gid, r, op.peer)].append(e)
                    mine.append(e)
            self._cv.notify_all()
        for op in ops:
            if op.op is not self.module.irecv:
                continue
            key = (0 if op.group is None else op.group.gid, op.peer, r)
            with self._cv:
                idx = self._recv_next[key]
                self._recv_next[key] += 1
                self._wait(lambda: len(self._chan[key]) > idx)
                e = self._chan[key][idx]
            src, dst = e["t"], op.tensor
            if src.numel() * src.element_size() != dst.numel() * dst.element_size() or src.dtype != dst.dtype:
                raise RuntimeError(f"fake NCCL: rank {r} receives {tuple(dst.shape)} {dst.dtype} from rank "
                                   f"{op.peer}, which sent {tuple(src.shape)} {src.dtype}")
            dst.record_stream(comm)
            comm.wait_event(e["ready"])
            with torch.cuda.stream(comm):
                if self.delay_cycles:
                    torch.cuda._sleep(self.delay_cycles)
                if not self.drop_receives:
                    dst.copy_(src)
            done = self._event(comm)
            with self._cv:
                e["done"] = done
                self._cv.notify_all()
        for e in mine:
            with self._cv:
                self._wait(lambda: e["done"] is not None)
            comm.wait_event(e["done"])
        return [_Work(self._finish(comm, sync=False))]

    # ---- collectives ----
    def all_gather(self, outs, inp, group=None, async_op=False):
        self.calls["all_gather"] += 1
        comm = self._start()
        inp.record_stream(comm)
        d = self._rendezvous((inp, self._event(comm)), group)
        with torch.cuda.stream(comm):
            for q in range(len(d)):
                comm.wait_event(d[q][1])
                outs[q].record_stream(comm)
                outs[q].copy_(d[q][0])
        done = self._rendezvous(self._event(comm), group)
        for q in range(len(done)):
            comm.wait_event(done[q])
        self._finish(comm)

    def _combine(self, t, op, root=None, group=None):
        comm = self._start()
        t.record_stream(comm)
        d = self._rendezvous((t, self._event(comm)), group)
        acc = None
        if root is None or self.rank == root:  # (root: a global rank, as torch.distributed names it)
            with torch.cuda.stream(comm):
                for q in range(len(d)):
                    comm.wait_event(d[q][1])
                    x = d[q][0]
                    if acc is None:
                        acc = x.clone()
                    elif op == "max":
                        torch.maximum(acc, x, out=acc)
                    else:
                        acc.add_(x)
        done = self._rendezvous(self._event(comm), group)  # every member has read every input
        for q in range(len(done)):
            comm.wait_event(done[q])
        if acc is not None:
            with torch.cuda.stream(comm):
                t.copy_(acc)
            acc.record_stream(comm)
        self._finish(comm)

    def all_reduce(self, t, op=None, group=None, async_op=False):
        self.calls["all_reduce"] += 1
        self._combine(t, op or "sum", group=group)

    def reduce(self, t, dst, op=None, group=None, async_op=False):
        self.calls["reduce"] += 1
        self._combine(t, op or "sum", root=dst, group=group)

    def barrier(self, group=None):
        self.calls["barrier"] += 1
        comm = self._start()
        self._rendezvous(None, group)
        self._finish(comm)

    def _make_module(self):
        world = self

        class P2POp:
            def __init__(self, op, tensor, peer, group=None):
                self.op, self.tensor, self.peer, self.group = op, tensor, peer, group

        def isend(*a, **k):
            raise NotImplementedError("fake NCCL: use batch_isend_irecv")

        def irecv(*a, **k):
            raise NotImplementedError("fake NCCL: use batch_isend_irecv")

        return types.SimpleNamespace(
            get_rank=lambda group=None: world._grank(group),
            get_world_size=lambda group=None: len(world._members(group)),
            get_backend=lambda group=None: "nccl",
            get_global_rank=lambda group, r: world._members(group)[r],
            new_group=world.new_group,
            P2POp=P2POp, isend=isend, irecv=irecv,
            ReduceOp=types.SimpleNamespace(SUM="sum", MAX="max"),
            batch_isend_irecv=world.batch_isend_irecv,
            all_gather=world.all_gather, all_reduce=world.all_reduce, reduce=world.reduce,
            barrier=world.barrier)


def run_ranks(world, fn, timeout_s=300.0):
    """fn(rank) in one thread per rank (each entered into `world` first); returns the results in rank order and
    re-raises the first rank's exception"""
    out, err = [None] * world.world, [None] * world.world

    def main(r):
        try:
            world.enter(r)
            out[r] = fn(r)
            torch.cuda.synchronize()
        except BaseException as e:  # noqa: B036 -- reported to the caller below
            err[r] = e
            with world._cv:
                world._cv.notify_all()

    ths = [threading.Thread(target=main, args=(r,), daemon=True) for r in range(world.world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout_s)
    if any(t.is_alive() for t in ths):
        raise TimeoutError("fake NCCL ranks did not finish")
    for e in err:
        if e is not None:
            raise e
    return out
