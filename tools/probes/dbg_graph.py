"""Debug probe: the graph-capture test flow (tests/test_gpu_streams.py) with per-step checks
against the CPU oracle."""
import sys
import numpy as np
import torch
sys.path.insert(0, "mixed-gemmul8_amd"); sys.path.insert(0, ".")
import gemmul8 as G
from oracle import oracle as O

m, n, k, N = 300, 260, 513, 14


def inputs(seed):
    return G.randmat(m, k, torch.float64, 0.5, seed), G.randmat(k, n, torch.float64, 0.5, seed + 1)


def oracle(A, B, fast):
    An = A.cpu().numpy().T.copy(order="F"); Bn = B.cpu().numpy().T.copy(order="F")
    return np.asfortranarray(O.gemm(An, Bn, N, fast))


def same(x, y):
    return np.asfortranarray(x.cpu().numpy().T).tobytes() == y.tobytes()


for fast in (True, False):
    A, B = inputs(11)
    W = G.alloc_work(m, n, k, N)
    C_ref = torch.zeros((n, m), dtype=torch.float64, device="cuda")
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C_ref, m, N, fast, W)
    torch.cuda.synchronize()
    print(fast, "direct vs oracle", same(C_ref, oracle(A, B, fast)))
    C = torch.zeros_like(C_ref)
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, W, stream=s)
    torch.cuda.synchronize()
    C.zero_(); W.zero_()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(fast, "replay vs direct", bool(torch.equal(C, C_ref)))
    A2, B2 = inputs(99)
    A.copy_(A2); B.copy_(B2)
    g.replay()
    torch.cuda.synchronize()
    Co = oracle(A2, B2, fast)
    print(fast, "replay(new data) vs oracle", same(C, Co))
    C2 = torch.zeros_like(C_ref)
    G.gemm(0, 0, m, n, k, 1.0, A2, m, B2, k, 0.0, C2, m, N, fast, G.alloc_work(m, n, k, N))
    torch.cuda.synchronize()
    print(fast, "direct(new data) vs oracle", same(C2, Co))
    d = (C - C2).abs()
    print(fast, "diff count", int((d > 0).sum()), "max", float(d.max()))
    if int((d > 0).sum()):
        idx = torch.nonzero(d > 0)[:5]
        print(idx.tolist())
