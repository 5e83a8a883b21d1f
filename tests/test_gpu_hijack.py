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
# the tests below run small shapes: the interposer's default thresholds (1280) would forward them
SMALL_THRESHOLDS = {"GEMMUL8_INTERCEPT_THRESHOLD_M": "128", "GEMMUL8_INTERCEPT_THRESHOLD_N": "128",
                    "GEMMUL8_INTERCEPT_THRESHOLD_K": "128"}

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
    out["stale_still_pending"] = bool(hip.hipPeekAtLastError() != 0)  # not consumed by the emulator
    hip.hipGetLastError()
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


# The Ex and strided-batched forms called directly (no framework uses them for fp64): hipblasGemmEx /
# hipblasGemmStridedBatchedEx with the 64F compute type are emulated, the pedantic compute type is
# forwarded; rocblas_gemm_ex in place (d == c) is emulated, out of place forwarded;
# rocblas_dgemm_strided_batched and rocblas_zgemm_strided_batched are emulated per batch.
CHILD_EX = r'''
import ctypes, json, os, sys
hj = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)
import torch
sys.path.insert(0, sys.argv[2])
import gemmul8 as G
torch.matmul(torch.ones(4, 4, dtype=torch.float64, device="cuda"), torch.ones(4, 4, dtype=torch.float64, device="cuda"))
hb = ctypes.CDLL("libhipblas.so.3", mode=os.RTLD_NOLOAD | os.RTLD_LAZY)
rb = ctypes.CDLL("librocblas.so.5", mode=os.RTLD_NOLOAD | os.RTLD_LAZY)
st = torch.cuda.current_stream().cuda_stream
h = ctypes.c_void_p(); assert hb.hipblasCreate(ctypes.byref(h)) == 0; hb.hipblasSetStream(h, ctypes.c_void_p(st))
r = ctypes.c_void_p(); assert rb.rocblas_create_handle(ctypes.byref(r)) == 0; rb.rocblas_set_stream(r, ctypes.c_void_p(st))
g = torch.Generator(device="cuda").manual_seed(9)
I, P, L = ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong
m, n, k = 384, 320, 448
out = {}
def emu(A, B, dt, Cin=None, beta=0.0, ct=0):
    C = torch.zeros((n, m), dtype=dt, device="cuda") if Cin is None else Cin.clone()
    W = G.alloc_work(m, n, k, 14, ct)
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, beta, C, m, 14, True, W, ct)
    return C
def mats(dt, batch=None):
    sh = lambda a, b: (a, b) if batch is None else (batch, a, b)
    if dt.is_complex:
        mk = lambda a, b: torch.complex(torch.randn(*sh(a, b), dtype=torch.float64, device="cuda", generator=g),
                                        torch.randn(*sh(a, b), dtype=torch.float64, device="cuda", generator=g))
    else:
        mk = lambda a, b: torch.randn(*sh(a, b), dtype=dt, device="cuda", generator=g)
    return mk(k, m), mk(n, k), mk(n, m)
one, half = ctypes.c_double(1.0), ctypes.c_double(0.5)
z1, zh = (ctypes.c_double * 2)(1.0, 0.0), (ctypes.c_double * 2)(0.5, 0.0)
# hipblasGemmEx, HIP_R_64F, HIPBLAS_COMPUTE_64F (7), then _PEDANTIC (8)
A, B, C0 = mats(torch.float64)
for ct, key in ((7, "gemmex"), (8, "gemmex_pedantic")):
    C = C0.clone()
    rc = hj.hipblasGemmEx(h, 111, 111, m, n, k, ctypes.byref(one), P(A.data_ptr()), 1, m, P(B.data_ptr()), 1, k,
                          ctypes.byref(half), P(C.data_ptr()), 1, m, ct, 160)
    torch.cuda.synchronize()
    Cv = C0.clone()
    rcv = -1
    if ct == 8:  # the vendor routine itself (for 64F it would call rocblas_gemm_ex, which is interposed too)
        rcv = hb.hipblasGemmEx(h, 111, 111, m, n, k, ctypes.byref(one), P(A.data_ptr()), 1, m, P(B.data_ptr()), 1, k,
                               ctypes.byref(half), P(Cv.data_ptr()), 1, m, ct, 160)
    torch.cuda.synchronize()
    out[key] = {"rc": rc, "bits": bool(torch.equal(C, emu(A, B, torch.float64, C0, 0.5))),
                "vendor_rc": rcv, "vendor_bits": bool(torch.equal(C, Cv))}
# hipblasGemmStridedBatchedEx, HIP_C_64F, 3 batches
A, B, C0 = mats(torch.complex128, 3)
C = C0.clone()
rc = hj.hipblasGemmStridedBatchedEx(h, 111, 111, m, n, k, z1, P(A.data_ptr()), 5, m, L(k * m), P(B.data_ptr()), 5, k,
                                    L(n * k), zh, P(C.data_ptr()), 5, m, L(n * m), 3, 7, 160)
torch.cuda.synchronize()
out["gemm_sb_ex"] = {"rc": rc, "bits": all(bool(torch.equal(C[i], emu(A[i], B[i], torch.complex128, C0[i], 0.5, 1)))
                                       for i in range(3))}
# rocblas_gemm_ex in place and out of place (f64_r = 152)
A, B, C0 = mats(torch.float64)
C = C0.clone()
rc = hj.rocblas_gemm_ex(r, 111, 111, m, n, k, ctypes.byref(one), P(A.data_ptr()), 152, m, P(B.data_ptr()), 152, k,
                        ctypes.byref(half), P(C.data_ptr()), 152, m, P(C.data_ptr()), 152, m, 152, 0, 0, 0)
torch.cuda.synchronize()
out["rocblas_gemm_ex"] = {"rc": rc, "bits": bool(torch.equal(C, emu(A, B, torch.float64, C0, 0.5)))}
D = torch.zeros_like(C0)
rc = hj.rocblas_gemm_ex(r, 111, 111, m, n, k, ctypes.byref(one), P(A.data_ptr()), 152, m, P(B.data_ptr()), 152, k,
                        ctypes.byref(half), P(C0.data_ptr()), 152, m, P(D.data_ptr()), 152, m, 152, 0, 0, 0)
torch.cuda.synchronize()
out["rocblas_gemm_ex_out_of_place"] = {"rc": rc, "relerr": float(((D - (A.t() @ B.t()).t() - 0.5 * C0).abs().max()
                                                               / D.abs().max()))}
# rocblas_dgemm_strided_batched / rocblas_zgemm_strided_batched
for name, dt, a1, ah, ct in (("rocblas_dgemm_strided_batched", torch.float64, ctypes.byref(one), ctypes.byref(half), 0),
                             ("rocblas_zgemm_strided_batched", torch.complex128, z1, zh, 1)):
    A, B, C0 = mats(dt, 2)
    C = C0.clone()
    rc = getattr(hj, name)(r, 111, 111, m, n, k, a1, P(A.data_ptr()), m, L(k * m), P(B.data_ptr()), k, L(n * k), ah,
                           P(C.data_ptr()), m, L(n * m), 2)
    torch.cuda.synchronize()
    out[name] = {"rc": rc, "bits": all(bool(torch.equal(C[i], emu(A[i], B[i], dt, C0[i], 0.5, ct))) for i in range(2))}
print("RESULT " + json.dumps(out))
'''


def test_ex_and_batched_forms():
    assert os.path.exists(HIJACK), "libgemmul8_hijack.so not built"
    env = dict(os.environ, GEMMUL8_INFO="1", GEMMUL8_COMPUTE_MODE="fp64_int8_14", **SMALL_THRESHOLDS)
    r = subprocess.run([sys.executable, "-c", CHILD_EX, HIJACK, os.path.join(ROOT, "mixed-gemmul8_amd")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][len("RESULT "):])
    log = r.stderr
    assert res["gemmex"]["rc"] == 0 and res["gemmex"]["bits"], res
    assert "[gemmul8] hipblasGemmEx m=384 n=320 k=448 -> emulated" in log, log[-2000:]
    # the pedantic compute type goes to the vendor routine: the same status and C as calling it directly
    # (this hipBLAS answers HIPBLAS_STATUS_NOT_SUPPORTED for it)
    pd = res["gemmex_pedantic"]
    assert pd["rc"] == pd["vendor_rc"] and pd["vendor_bits"], res
    assert log.count("hipblasGemmEx m=384") == 1, log[-2000:]
    assert res["gemm_sb_ex"]["rc"] == 0 and res["gemm_sb_ex"]["bits"], res
    assert log.count("hipblasGemmStridedBatchedEx m=384 n=320 k=448 -> emulated") == 3, log[-2000:]
    assert res["rocblas_gemm_ex"]["rc"] == 0 and res["rocblas_gemm_ex"]["bits"], res
    assert log.count("rocblas_gemm_ex m=384") == 1, log[-2000:]  # out of place: forwarded
    assert res["rocblas_gemm_ex_out_of_place"]["rc"] == 0 and res["rocblas_gemm_ex_out_of_place"]["relerr"] < 1e-13, res
    for name in ("rocblas_dgemm_strided_batched", "rocblas_zgemm_strided_batched"):
        assert res[name]["rc"] == 0 and res[name]["bits"], (name, res)
        assert log.count(f"[gemmul8] {name} m=384 n=320 k=448 -> emulated") == 2, log[-2000:]


def test_torch_matmul_is_emulated():
    assert os.path.exists(HIJACK), "libgemmul8_hijack.so not built"
    env = dict(os.environ, GEMMUL8_INFO="1", GEMMUL8_COMPUTE_MODE="fp64_int8_14", **SMALL_THRESHOLDS)
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


CHILD_DEFAULT = r'''
import ctypes, json, os, sys
hj = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)
import torch
sys.path.insert(0, sys.argv[2])
import gemmul8 as G
g = torch.Generator(device="cuda").manual_seed(3)
out = {}
for s in (512, 1024, 2048):
    A = torch.randn(s, s, dtype=torch.float64, device="cuda", generator=g)
    B = torch.randn(s, s, dtype=torch.float64, device="cuda", generator=g)
    C = torch.matmul(A, B)
    E = G.matmul(B.t().contiguous(), A.t().contiguous(), 14).t()
    out[str(s)] = bool(torch.equal(C, E))
print("RESULT " + json.dumps(out))
'''


def test_default_thresholds_follow_the_crossover():
    """with no threshold set, DGEMMs below the measured MI355X crossover (1280) keep the vendor routine
    (512^3, 1024^3) and larger ones are emulated (2048^3, bit for bit)"""
    assert os.path.exists(HIJACK), "libgemmul8_hijack.so not built"
    env = {k: v for k, v in os.environ.items() if not k.startswith("GEMMUL8_INTERCEPT_THRESHOLD")}
    env.update(GEMMUL8_INFO="1", GEMMUL8_COMPUTE_MODE="fp64_int8_14")
    r = subprocess.run([sys.executable, "-c", CHILD_DEFAULT, HIJACK, os.path.join(ROOT, "mixed-gemmul8_amd")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][len("RESULT "):])
    log = r.stderr
    assert "m=2048 n=2048 k=2048 -> emulated" in log, log[-2000:]
    assert "m=512 " not in log and "m=1024 " not in log, log[-2000:]
    assert res["2048"] and not res["512"], res
