import sys, json, torch
sys.path.insert(0, "mixed-gemmul8_amd")
import gemmul8 as G
for dt, N, name in ((torch.complex64, 8, "cf N=8"), (torch.complex64, 12, "cf N=12"), (torch.complex128, 12, "cd N=12")):
    m = k = 4096
    A = G.randmat(m, k, dt, 0.5, 123456); B = G.randmat(k, m, dt, 0.5, 654321)
    C = torch.empty((m, m), dtype=dt, device="cuda")
    ct = G.COMPLEX_BIG_MATRIX_ENCODE
    w = G.alloc_work(m, m, k, N, ct)
    call = lambda: G.gemm(G.OP_N, G.OP_N, m, m, k, 1.0, A, m, B, k, 0.0, C, m, N, True, w, ct)
    for _ in range(3): call()
    torch.cuda.synchronize()
    G.timing_enable(True); G.timing_read()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): call()
    e1.record(); torch.cuda.synchronize(); G.timing_enable(False)
    ph, _ = G.timing_read()
    ms = e0.elapsed_time(e1) / 10
    print(name, "ms", round(ms, 4), "TF", round(8 * m**3 / ms / 1e9, 1), "phases", [round(x / 10, 4) for x in ph])
