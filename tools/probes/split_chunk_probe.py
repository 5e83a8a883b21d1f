"""Split phase at 8192^3 (N = 14, fast, f64 op N x op N): one split over the whole operands against the same
bytes split in vector chunks (rows [r0, r1) of op(A) with columns [r0, r1) of op(B) per call), so that each
chunk's encode re-reads operand data its shift pass has just left in the 256 MB Infinity Cache.  Every timed run
starts after a 1 GiB write (the cache holds none of the operands).  Interleaved rounds, medians.
python split_chunk_probe.py [rounds] [chunks...]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
import torch
import gemmul8 as G

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
chunks = [int(x) for x in sys.argv[2:]] or [2048, 1024, 512]
M = K = 8192
N = 14
A = G.randmat(M, K, torch.float64, 0.5, 123456)   # (k, m) storage: column-major m x k, lda = m
B = G.randmat(K, M, torch.float64, 0.5, 654321)   # (n, k) storage: column-major k x n, ldb = k
flush = torch.empty(1 << 27, dtype=torch.float64, device="cuda")
works = {M: G.alloc_work(M, M, K, N)}
for c in chunks:
    works[c] = G.alloc_work(c, c, K, N)


def full():
    G.split(G.OP_N, G.OP_N, M, M, K, A, M, B, K, N, True, works[M], torch.float64)


def chunked(c):
    def f():
        for r0 in range(0, M, c):
            G.split(G.OP_N, G.OP_N, c, c, K, A[:, r0:], M, B[r0:], K, N, True, works[c], torch.float64)
    return f


variants = [("full", full)] + [(f"chunk{c}", chunked(c)) for c in chunks]
for _, f in variants:
    f()
torch.cuda.synchronize()
times = {name: [] for name, _ in variants}
for r in range(rounds):
    for name, f in variants:
        flush.fill_(float(r))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1))
    print("round", r, {k: round(v[-1], 4) for k, v in times.items()}, flush=True)
alg = 2 * M * K * 8 + 2 * M * K * N  # operands read once + slices written
for name, t in times.items():
    med = statistics.median(t)
    print(f"{name:10s} median {med:.4f} ms  min {min(t):.4f}  {alg / med / 1e6:.0f} GB/s algorithmic", flush=True)
