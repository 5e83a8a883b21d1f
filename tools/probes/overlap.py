"""Does an encode overlap with a running product launch?  cfg2 shapes, phases through the C ABI.
seq: split(0..14) products(0..14) recombine
two: split(0..7) -> [products(0..7) on s2 || split(7..14) on s1] -> products(7..14) -> recombine"""
import os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mixed-gemmul8_amd"))
import gemmul8 as G

m = n = k = 8192
N = 14
A = G.randmat(m, k)
B = G.randmat(k, n)
C = torch.empty((n, m), dtype=torch.float64, device="cuda")
work = G.alloc_work(m, n, k, N)
s1 = torch.cuda.current_stream()
s2 = torch.cuda.Stream()
dt = torch.float64


def seq():
    G.split(0, 0, m, n, k, A, m, B, k, N, True, work, dt, 0, 7)
    G.split(0, 0, m, n, k, A, m, B, k, N, True, work, dt, 7, 14)
    G.products(m, n, k, N, work, 0, 14)
    G.recombine(m, n, k, N, 1.0, 0.0, C, m, work)


def two():
    G.split(0, 0, m, n, k, A, m, B, k, N, True, work, dt, 0, 7)
    e = torch.cuda.Event()
    e.record(s1)
    s2.wait_event(e)
    G.products(m, n, k, N, work, 0, 7, stream=s2)
    G.split(0, 0, m, n, k, A, m, B, k, N, True, work, dt, 7, 14)
    G.products(m, n, k, N, work, 7, 14)
    e2 = torch.cuda.Event()
    e2.record(s2)
    s1.wait_event(e2)
    G.recombine(m, n, k, N, 1.0, 0.0, C, m, work)


def timeit(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


seq()
torch.cuda.synchronize()
ref = C.clone()
two()
torch.cuda.synchronize()
assert torch.equal(ref, C)
for _ in range(2):
    print("seq %.3f ms   two %.3f ms" % (timeit(seq), timeit(two)), flush=True)
