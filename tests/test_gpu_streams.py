"""Stream semantics of the drop-in call (SURVEY.md 8(b) "Threading and streams"): the reference
runs every kernel on the null stream with hipDeviceSynchronize around each phase
(gemmul8.cu:251-289) and keeps its launch configuration in globals (common.hpp:11-20), so it can
neither be captured into a graph nor called from two threads at once.  This build runs every
kernel on the caller's stream with no device-wide synchronisation and per-call state only; these
tests hold it to that:
  * a call captured into a HIP graph and replayed gives the same bits as a direct call
    (nothing in the call path allocates, synchronises or reads back);
  * two host threads calling on two streams at once, each with its own workspace, give the same
    bits as the calls one after the other."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Lazy:  # the library is imported on first use (CPU collection does not load it)
    def __getattr__(self, name):
        import gemmul8
        return getattr(gemmul8, name)


G = _Lazy()


def _same(a, b):
    return a.shape == b.shape and torch.equal(a.contiguous().view(torch.uint8), b.contiguous().view(torch.uint8))


def _inputs(m, n, k, seed, dtype=torch.float64):
    A = G.randmat(m, k, dtype, 0.5, seed)
    B = G.randmat(k, n, dtype, 0.5, seed + 1)
    return A, B


@pytest.mark.parametrize("dtype,ctype,fast,S,big", [
    (torch.float64, 0, True, None, False),
    (torch.float64, 0, False, None, False),
    (torch.float32, 0, False, None, False),
    (torch.complex128, 1, False, None, False),   # COMPLEX_BIG_MATRIX_ENCODE, accurate (bound of 2m rows)
    (torch.complex128, 3, True, None, False),    # COMPLEX_KARATSUBA_MULT
    (torch.float64, 0, False, 4, False),         # low-memory mode: moduli in groups of 4
    # (m + n) k >= 2^25: accurate mode runs operand B's split on the second stream (fork / join in the
    # graph); fast mode with one element type runs the pair split kernels on the call's stream
    (torch.float64, 0, True, None, True),
    (torch.float64, 0, False, None, True),
    (torch.float64, 0, False, 4, True),
])
def test_graph_capture_replay_same_bits(dtype, ctype, fast, S, big):
    m, n, k, N = (2048, 2040, 8192, 14) if big else (300, 260, 513, 14 if ctype == 0 else 7)
    A, B = _inputs(m, n, k, 11, dtype)
    W = G.alloc_work(m, n, k, N, ctype, slice_planes=S)

    def direct(A, B, W):
        C = torch.zeros((n, m), dtype=dtype, device="cuda")
        G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, W, ctype, slice_planes=S)
        torch.cuda.synchronize()
        return C

    C_ref = direct(A, B, W)
    C = torch.zeros_like(C_ref)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, W, ctype, stream=s, slice_planes=S)
    torch.cuda.synchronize()
    C.zero_()
    W.zero_()  # the replay must rebuild everything it reads from the workspace
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert _same(C, C_ref)

    # replay picks up new operand values written into the captured buffers (accurate mode: the
    # bound maxima of the previous replay must not survive)
    A2, B2 = _inputs(m, n, k, 99, dtype)
    A.copy_(A2)
    B.copy_(B2)
    g.replay()
    torch.cuda.synchronize()
    assert _same(C, direct(A2, B2, G.alloc_work(m, n, k, N, ctype, slice_planes=S)))


def test_two_threads_two_streams_same_bits():
    shapes = [(520, 384, 700, 14, True, torch.float64), (256, 640, 1100, 9, False, torch.float32),
              (2048, 2048, 8192, 12, False, torch.float64), (1800, 2300, 8000, 14, True, torch.float64)]
    jobs = []
    for i, (m, n, k, N, fast, dt) in enumerate(shapes):
        A, B = _inputs(m, n, k, 100 + i, dt)
        jobs.append(dict(m=m, n=n, k=k, N=N, fast=fast, A=A, B=B, W=G.alloc_work(m, n, k, N),
                         C=torch.zeros((n, m), dtype=dt, device="cuda"), ref=None))
    for j in jobs:  # one after the other on the default stream
        C = torch.zeros_like(j["C"])
        G.gemm(G.OP_N, G.OP_N, j["m"], j["n"], j["k"], 1.0, j["A"], j["m"], j["B"], j["k"], 0.0, C, j["m"], j["N"],
               j["fast"], j["W"])
        j["ref"] = C
    torch.cuda.synchronize()

    errors = []
    barrier = threading.Barrier(len(jobs))

    def worker(j):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                barrier.wait()
                for _ in range(5):
                    G.gemm(G.OP_N, G.OP_N, j["m"], j["n"], j["k"], 1.0, j["A"], j["m"], j["B"], j["k"], 0.0, j["C"],
                           j["m"], j["N"], j["fast"], j["W"], stream=s)
                s.synchronize()
        except Exception as e:  # surfaced below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(j,)) for j in jobs]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    for j in jobs:
        assert _same(j["C"], j["ref"])
    assert np.isfinite(jobs[0]["C"].cpu().numpy()).all()


def test_eager_call_during_foreign_capture_gets_no_captured_lane():
    """Operand B's split runs on a pooled second stream (a "lane") for big non-pair forms.  A call
    captured into a graph must not take a lane: forked into the capture, the lane stays part of it
    until the capture ends, and an eager call that picked it from the pool meanwhile would record
    its B split into the foreign graph instead of running it.  Deterministic form: an eager call on
    another stream while the capture is still open (relaxed capture mode)."""
    m, n, k, N = 2048, 2040, 8192, 14  # (m + n) k >= 2^25, accurate mode: the two-stream split
    A, B = _inputs(m, n, k, 21)
    A2, B2 = _inputs(m, n, k, 23)
    W, W2 = G.alloc_work(m, n, k, N), G.alloc_work(m, n, k, N)
    C_ref2 = torch.zeros((n, m), dtype=torch.float64, device="cuda")
    G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A2, m, B2, k, 0.0, C_ref2, m, N, False, W2)  # leaves a lane in the pool
    C_ref = torch.zeros_like(C_ref2)
    G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C_ref, m, N, False, W)
    torch.cuda.synchronize()
    C = torch.zeros_like(C_ref)
    C2 = torch.zeros_like(C_ref2)
    s, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, False, W, stream=s)
            # still capturing on s: an eager call on s2 takes a lane from the pool
            G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A2, m, B2, k, 0.0, C2, m, N, False, W2, stream=s2)
    torch.cuda.synchronize()
    assert _same(C2, C_ref2)  # the eager call ran in full (its B split was not recorded into g)
    W.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert _same(C, C_ref)
