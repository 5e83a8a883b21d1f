"""Phase timers of the drop-in call.  The reference's gemm() returns the four phase times in ns
(gemmul8.hpp:29-47), measured with hipDeviceSynchronize around every phase (gemmul8.cu:10-18,
251-289).  Here they come from HIP events attached to the phase kernels' own dispatches
(oz2_split.hpp launch(), no marker packets): split = first split launch to the product kernel's
start, products = the product launch(es), CRT = product end to CRT end; the conversion phase is
fused into the products and reads 0.  These tests hold the timers to that in every call form."""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


class _Lazy:  # the library is imported on first use (CPU collection does not load it)
    def __getattr__(self, name):
        import gemmul8
        return getattr(gemmul8, name)


G = _Lazy()


def _call(m, n, k, N, dtype=torch.float64, ctype=0, fast=True, S=None, stream=None, phase_times=False, seed=5):
    A = G.randmat(m, k, dtype, 0.5, seed)
    B = G.randmat(k, n, dtype, 0.5, seed + 1)
    C = torch.zeros((n, m), dtype=dtype, device="cuda")
    W = G.alloc_work(m, n, k, N, ctype, slice_planes=S)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t = G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, W, ctype, stream=stream,
               phase_times=phase_times, slice_planes=S)
    torch.cuda.synchronize()
    return t, (time.perf_counter() - t0) * 1e9, C


@pytest.mark.parametrize("m,n,k,N,dtype,ctype,fast,S", [
    (2048, 2048, 2048, 14, torch.float64, 0, True, None),    # pair split kernels, persistent products
    (2048, 2040, 8192, 12, torch.float64, 0, False, None),   # accurate mode, B's split on the second stream
    (1500, 1300, 3000, 14, torch.float64, 0, True, 4),       # low-memory: encodes + products in groups
    (1024, 1024, 4096, 12, torch.complex128, 3, True, None),  # Karatsuba complex
    (700, 500, 900, 9, torch.float32, 0, True, None),
])
def test_phase_times_cover_the_call(m, n, k, N, dtype, ctype, fast, S):
    t, wall, _ = _call(m, n, k, N, dtype, ctype, fast, S, phase_times=True)
    assert len(t) == 4 and t[2] == 0.0
    assert t[0] > 0 and t[1] > 0 and t[3] > 0, t
    # the events bracket stream work inside the host's window around the synchronous call
    assert sum(t) <= wall, (t, wall)
    assert sum(t) >= 0.2 * wall, (t, wall)


def test_timing_accumulates_per_call_and_resets():
    m = n = k = 2048
    A = G.randmat(m, k, torch.float64, 0.5, 1)
    B = G.randmat(k, n, torch.float64, 0.5, 2)
    C = torch.zeros((n, m), dtype=torch.float64, device="cuda")
    W = G.alloc_work(m, n, k, 14)
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)
    G.timing_enable(True)
    G.timing_read()
    for _ in range(3):
        G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)
    G.timing_enable(False)
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)  # not recorded
    ph, calls = G.timing_read()
    assert calls == 3
    assert ph[0] > 0 and ph[1] > 0 and ph[2] == 0 and ph[3] > 0
    # one product launch per call: 3 x (2 m n k N) int8 ops cannot take less than at 5 POPS
    assert ph[1] * 1e-3 >= 3 * 2.0 * m * n * k * 14 / 5.1e15
    ph2, calls2 = G.timing_read()
    assert calls2 == 0 and ph2 == [0.0, 0.0, 0.0, 0.0]


def test_products_entry_point_times_the_products_only():
    m, n, k, N = 1024, 768, 2048, 10
    A = torch.randn((k, m), dtype=torch.float64, device="cuda")  # row-major m x k = column-major k x m
    B = torch.randn((n, k), dtype=torch.float64, device="cuda")
    W = G.alloc_work(m, n, k, N)
    G.split(G.OP_T, G.OP_T, m, n, k, A, k, B, n, N, True, W, torch.float64)
    G.timing_enable(True)
    G.timing_read()
    G.products(m, n, k, N, W, 0, 5)
    G.products(m, n, k, N, W, 5, N)
    G.timing_enable(False)
    ph, calls = G.timing_read()
    assert calls == 2
    assert ph[0] == 0.0 and ph[2] == 0.0 and ph[3] == 0.0 and ph[1] > 0


def test_timed_call_leaves_nothing_armed():
    """After a timed call on one stream, an untimed call on another stream and a timed call captured
    into a graph (no events recorded there: phase times read 0) give the bits of a plain call."""
    m, n, k, N = 600, 520, 700, 14
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    _, _, C_ref = _call(m, n, k, N)
    t, _, C1 = _call(m, n, k, N, stream=s1, phase_times=True)
    assert t[1] > 0
    _, _, C2 = _call(m, n, k, N, stream=s2)
    assert torch.equal(C1, C_ref) and torch.equal(C2, C_ref)
    A = G.randmat(m, k, torch.float64, 0.5, 5)
    B = G.randmat(k, n, torch.float64, 0.5, 6)
    C = torch.zeros((n, m), dtype=torch.float64, device="cuda")
    W = G.alloc_work(m, n, k, N)
    s2.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s2):
        with torch.cuda.graph(g, stream=s2):
            tc = G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, W, stream=s2, phase_times=True)
    assert tc == [0.0, 0.0, 0.0, 0.0]
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(C, C_ref)
