"""GPU: the hipBLAS/rocBLAS GEMM interposer (mixed-gemmul8_amd/csrc/hijack.cpp) under an unmodified
PyTorch.  A child process loads libgemmul8_hijack.so into the global symbol scope before torch
(the in-process equivalent of LD_PRELOAD), then calls torch.matmul: float64 / complex128
products at or above the intercept thresholds must be the emulator's result bit for bit, smaller
ones must reach the vendor routine.  Under CUDA-graph capture every call is emulated in a workspace
of the capture's own (never the stream's eager buffer): a later, larger eager call on the same
stream must not pull it from under the graph, and two graphs captured on one stream must replay
concurrently on two streams without sharing it.  A HIP error left pending by the application before
an interposed DGEMM with beta != 0 must not make the call look failed (which used to forward it to
the vendor routine after the emulator had written C, applying beta twice).  Two threads on one stream
with growing sizes must get the emulator's bits (a growing call frees the stream's eager buffer)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIJACK = os.path.join(ROOT, "mixed-gemmul8_amd", "gemmul8", "libgemmul8_hijack.so")

CHILD = r'''
import ctypes, json, os, sys
hj = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)
hj.gemmul8_hijack_last_workspace.restype = ctypes.c_void_p
import torch
sys.path.insert(0, sys.argv[2])
import gemmul8 as G
out = {}
g = torch.Generator(device="cuda").manual_seed(5)
for name, dt, (m, k, n) in (("d", torch.float64, (512, 448, 384)), ("z", torch.complex128, (300, 260, 280))):
    A = torch.randn(m, k, dtype=dt, device="cuda", generator=g)
    B = torch.randn(k, n, dtype=dt, device="cuda", generator=g)
    C = torch.matmul(A, B)                       # torch -> hipblas{D,Z}gemm -> interposer
    # torch multiplies column-major: C^T = B^T A^T, so the emulated "A" operand is B^T
    E = G.matmul(B.t().contiguous(), A.t().contiguous(), 14).t()
    exact = (A.cpu().to(torch.complex128) @ B.cpu().to(torch.complex128))
    out[name] = {"bits": bool(torch.equal(C, E)),
                 "relerr": float(((C.cpu().to(torch.complex128) - exact).abs() / exact.abs()).max())}
Ab = torch.randn(3, 300, 260, dtype=torch.float64, device="cuda", generator=g)
Bb = torch.randn(3, 260, 280, dtype=torch.float64, device="cuda", generator=g)
Cb = torch.bmm(Ab, Bb)                           # -> hipblasDgemmStridedBatched -> interposer
Eb = torch.stack([G.matmul(Bb[i].t().contiguous(), Ab[i].t().contiguous(), 14).t() for i in range(3)])
out["bmm_bits"] = bool(torch.equal(Cb, Eb))
# under CUDA-graph capture every call is emulated, in a workspace of the capture's own
A = torch.randn(512, 448, dtype=torch.float64, device="cuda", generator=g)
B = torch.randn(448, 384, dtype=torch.float64, device="cuda", generator=g)
E = G.matmul(B.t().contiguous(), A.t().contiguous(), 14).t()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    torch.matmul(A, B)                           # warms the workspace of stream s
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr, stream=s):
    Cg = torch.matmul(A, B)
gr.replay()
torch.cuda.synchronize()
out["graph_bits"] = bool(torch.equal(Cg, E))
A2 = torch.randn(520, 450, dtype=torch.float64, device="cuda", generator=g)
B2 = torch.randn(450, 390, dtype=torch.float64, device="cuda", generator=g)
s2 = torch.cuda.Stream()
s2.wait_stream(torch.cuda.current_stream())
gr2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr2, stream=s2):
    C2 = torch.matmul(A2, B2)                    # no eager workspace on s2: the capture gets its own
gr2.replay()
torch.cuda.synchronize()
ex2 = A2.cpu() @ B2.cpu()
out["graph_cold_relerr"] = float(((C2.cpu() - ex2).abs() / ex2.abs()).max())
out["graph_cold_bits"] = bool(torch.equal(C2, G.matmul(B2.t().contiguous(), A2.t().contiguous(), 14).t()))

def mats(m, k, n):
    return (torch.randn(m, k, dtype=torch.float64, device="cuda", generator=g),
            torch.randn(k, n, dtype=torch.float64, device="cuda", generator=g))

def emu(A, B):
    return G.matmul(B.t().contiguous(), A.t().contiguous(), 14).t()

# capture, then grow the stream's eager workspace with a larger call, then replay on new values
s3 = torch.cuda.Stream()
s3.wait_stream(torch.cuda.current_stream())
A3, B3 = mats(512, 448, 384)
with torch.cuda.stream(s3):
    torch.matmul(A3, B3)
torch.cuda.synchronize()
eager_ws = hj.gemmul8_hijack_last_workspace()
gr3 = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr3, stream=s3):
    C3 = torch.matmul(A3, B3)
cap_ws = hj.gemmul8_hijack_last_workspace()
out["capture_own_ws"] = bool(cap_ws != eager_ws)
if out["capture_own_ws"]:                        # otherwise the replay below would read freed memory
    Ab, Bb = mats(1536, 1280, 1024)
    with torch.cuda.stream(s3):
        torch.matmul(Ab, Bb)                     # grows (frees and reallocates) s3's eager buffer
    torch.cuda.synchronize()
    A3n, B3n = mats(512, 448, 384)
    A3.copy_(A3n)
    B3.copy_(B3n)
    torch.cuda.synchronize()
    gr3.replay()
    torch.cuda.synchronize()
    out["graph_after_grow_bits"] = bool(torch.equal(C3, emu(A3n, B3n)))

# two graphs captured on one stream, replayed concurrently on two streams
s4 = torch.cuda.Stream()
s4.wait_stream(torch.cuda.current_stream())
Ax, Bx = mats(1024, 1024, 1024)
Ay, By = mats(1024, 1024, 1024)
gx, gy = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
with torch.cuda.graph(gx, stream=s4):
    Cx = torch.matmul(Ax, Bx)
with torch.cuda.graph(gy, stream=s4):
    Cy = torch.matmul(Ay, By)
torch.cuda.synchronize()
s5, s6 = torch.cuda.Stream(), torch.cuda.Stream()
ok = True
Ex, Ey = emu(Ax, Bx), emu(Ay, By)
for _ in range(4):
    Cx.zero_()
    Cy.zero_()
    torch.cuda.synchronize()
    with torch.cuda.stream(s5):
        gx.replay()
    with torch.cuda.stream(s6):
        gy.replay()
    torch.cuda.synchronize()
    ok = ok and bool(torch.equal(Cx, Ex)) and bool(torch.equal(Cy, Ey))
out["concurrent_replays_bits"] = ok

# two threads on the one default stream, sizes growing: each growth frees the stream's eager buffer,
# which must not happen between the other thread's workspace lookup and its enqueue
import threading
res_t = []
def worker(seed):
    gg = torch.Generator(device="cuda").manual_seed(seed)
    ok = True
    for m in (256, 384, 640, 896, 1152, 1408, 1664):
        A = torch.randn(m, m - 64, dtype=torch.float64, device="cuda", generator=gg)
        B = torch.randn(m - 64, m + 32, dtype=torch.float64, device="cuda", generator=gg)
        C = torch.matmul(A, B)
        ok = ok and bool(torch.equal(C, emu(A, B)))
    res_t.append(ok)
ths = [threading.Thread(target=worker, args=(100 + i,)) for i in range(2)]
for t in ths:
    t.start()
for t in ths:
    t.join()
out["threads_same_stream_bits"] = len(res_t) == 2 and all(res_t)

# a HIP error left pending by the application, then an interposed DGEMM with beta = 0.5
hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_LAZY)
A5, B5 = mats(512, 448, 384)
C0 = torch.randn(512, 384, dtype=torch.float64, device="cuda", generator=g)
Cexp = C0.clone()
W5 = G.alloc_work(384, 512, 448, 14)
# the call the interposer receives: column-major C^T = 1 * B^T A^T + 0.5 * C^T
G.gemm(G.OP_N, G.OP_N, 384, 512, 448, 1.0, B5, 384, A5, 448, 0.5, Cexp, 384, 14, True, W5)
C5 = C0.clone()
torch.cuda.synchronize()
rc = hip.hipSetDevice(ctypes.c_int(12345))     # fails: leaves hipErrorInvalidDevice pending
out["stale_set"] = bool(rc != 0 and hip.hipPeekAtLastError() != 0)
try:
    C5.addmm_(A5, B5, beta=0.5)                  # -> hipblasDgemm with beta = 0.5
    torch.cuda.synchronize()
    out["stale_beta_bits"] = bool(torch.equal(C5, Cexp))
except RuntimeError as e:                        # torch itself reported the pending error first
    out["stale_exc"] = str(e)[:300]
hip.hipGetLastError()
A = torch.randn(64, 64, dtype=torch.float64, device="cuda", generator=g)
C = A @ A                                        # below the thresholds: forwarded
out["small_relerr"] = float(((C - (A.cpu() @ A.cpu()).cuda()).abs().max() / (A.cpu() @ A.cpu()).abs().max()))
print("RESULT " + json.dumps(out))
'''


def test_torch_matmul_is_emulated():
    assert os.path.exists(HIJACK), "libgemmul8_hijack.so not built"
    env = dict(os.environ, GEMMUL8_INFO="1", GEMMUL8_COMPUTE_MODE="fp64_int8_14")
    r = subprocess.run([sys.executable, "-c", CHILD, HIJACK, os.path.join(ROOT, "mixed-gemmul8_amd")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    log = r.stderr
    assert "[gemmul8] hipblasDgemm m=384 n=512 k=448 -> emulated" in log, log[-2000:]
    assert "[gemmul8] hipblasZgemm m=280 n=300 k=260 -> emulated" in log, log[-2000:]
    assert "m=64 n=64" not in log  # below the intercept thresholds: never reaches the emulator
    assert res["d"]["bits"] and res["z"]["bits"], res
    assert "[gemmul8] hipblasDgemmStridedBatched m=280 n=300 k=260" in log, log[-2000:]
    assert res["bmm_bits"], res
    assert res["d"]["relerr"] < 1e-9 and res["z"]["relerr"] < 1e-9, res
    assert res["small_relerr"] < 1e-12, res
    assert res["graph_bits"], res
    assert res["graph_cold_relerr"] < 1e-9, res
    assert "m=390 n=520 k=450 -> emulated" in log, log[-2000:]  # cold capture: emulated in its own workspace
    assert res["graph_cold_bits"], res
    assert res["capture_own_ws"], res
    assert res["graph_after_grow_bits"], res
    assert res["concurrent_replays_bits"], res
    assert res["threads_same_stream_bits"], res
    assert res["stale_set"], res
    assert res.get("stale_beta_bits"), res
    assert "launch failed" not in log, log[-2000:]
