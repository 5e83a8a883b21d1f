"""GPU: the hipBLAS/rocBLAS GEMM interposer (mixed-gemmul8_amd/csrc/hijack.cpp) under an unmodified
PyTorch.  A child process loads libgemmul8_hijack.so into the global symbol scope before torch
(the in-process equivalent of LD_PRELOAD), then calls torch.matmul: float64 / complex128
products at or above the intercept thresholds must be the emulator's result bit for bit, smaller
ones must reach the vendor routine; under CUDA-graph capture the emulator runs where its workspace
already exists and the call is forwarded where it would have to allocate."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIJACK = os.path.join(ROOT, "mixed-gemmul8_amd", "gemmul8", "libgemmul8_hijack.so")

CHILD = r'''
import ctypes, json, sys
ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)
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
# under CUDA-graph capture: a stream whose workspace exists stays emulated inside the graph; a
# stream without one is forwarded to the vendor routine (no allocation inside a capture)
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
    C2 = torch.matmul(A2, B2)
gr2.replay()
torch.cuda.synchronize()
ex2 = A2.cpu() @ B2.cpu()
out["graph_cold_relerr"] = float(((C2.cpu() - ex2).abs() / ex2.abs()).max())
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
    assert "m=390 n=520 k=450 -> emulated" not in log, log[-2000:]
