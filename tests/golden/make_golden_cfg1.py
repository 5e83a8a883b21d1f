#!/usr/bin/env python3
"""Golden fixture for cfg1 (BASELINE.json configs[0]: SGEMM emulation m=n=k=1024, num_moduli=4, fast mode),
generated on an MI355X from the REFERENCE's own HIP build (oracle/_ref/libgemmul8_ref.so).

Run on the GPU box:  python tests/golden/make_golden_cfg1.py <outdir>
Writes <outdir>/cfg1_A.npz (the float32 input A, column-major; B == A as in the reference driver,
seed 123456 of the driver's generator, gemmul8.randmat = testing/make_matrix.hpp:8-21) and
<outdir>/cfg1_ref.json (sha256 of A and of the reference's C, the reference's shift vectors' hashes,
and our library's C hash on the same inputs).  tests/test_oracle_cfg1.py runs the CPU oracle on A
and compares its C bit for bit through the hash.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mixed-gemmul8_amd"), os.path.join(ROOT, "tests", "golden")]
import gemmul8 as G  # noqa: E402
from make_golden import LIB, ref_sft_offsets  # noqa: E402


def sha(x):
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def main():
    outdir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "golden_cfg1")
    os.makedirs(outdir, exist_ok=True)
    m = n = k = 1024
    N = 4
    dA = G.randmat(m, k, torch.float32, 0.5, 123456, "cuda")  # (k, m) tensor = column-major m x k
    dB = G.randmat(k, n, torch.float32, 0.5, 123456, "cuda")
    assert torch.equal(dA, dB)
    lib = ctypes.CDLL(LIB)
    p, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.ref_gemm.argtypes = [i, i, i, i, i, sz, sz, sz, p, p, sz, p, sz, p, p, sz, u, i, i, p, p]
    lib.ref_work_size.restype = sz
    lib.ref_work_size.argtypes = [sz, sz, sz, u, i]
    work = torch.zeros(lib.ref_work_size(m, n, k, N, 0) + 16 * m * k + (1 << 20), dtype=torch.uint8, device="cuda")
    dC = torch.zeros((n, m), dtype=torch.float32, device="cuda")
    al = np.array([1.0], np.float32)
    be = np.array([0.0], np.float32)
    times = (ctypes.c_double * 4)()
    rc = lib.ref_gemm(1, 1, 1, 0, 0, m, n, k, al.ctypes.data, dA.data_ptr(), m, dB.data_ptr(), k, be.ctypes.data,
                      dC.data_ptr(), m, N, 1, 0, work.data_ptr(), times)
    assert rc == 0, rc
    torch.cuda.synchronize()
    C_ref = dC.cpu().numpy()  # (n, m) row-major = column-major m x n bytes
    wsb = work.cpu().numpy()
    oA, oB = ref_sft_offsets(m, n, k, N, False)
    sA = wsb[oA:oA + 2 * m].view(np.int16).copy()
    sB = wsb[oB:oB + 2 * n].view(np.int16).copy()
    # our library on the same inputs
    C2 = torch.empty((n, m), dtype=torch.float32, device="cuda")
    G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, dA, m, dB, k, 0.0, C2, m, N, True, G.alloc_work(m, n, k, N))
    torch.cuda.synchronize()
    A = dA.cpu().numpy()
    ref64 = A.T.astype(np.float64) @ A.T.astype(np.float64)
    rel = np.abs(C_ref.T.astype(np.float64) - ref64) / np.abs(ref64)
    np.savez_compressed(os.path.join(outdir, "cfg1_A.npz"), A_colmajor_as_rows=A)
    meta = {"workload": "cfg1: SGEMM emulation m=n=k=1024, num_moduli=4, fast mode, NN, alpha=1 beta=0, A == B "
                        "(gemmul8.randmat float32, phi 0.5, seed 123456)",
            "sha256_A": sha(A), "sha256_C_reference": sha(C_ref), "sha256_C_gemmul8_amd": sha(C2.cpu().numpy()),
            "sha256_sftA_reference": sha(sA), "sha256_sftB_reference": sha(sB),
            "relerr_max_vs_fp64": float(rel.max()), "relerr_median_vs_fp64": float(np.median(rel)),
            "reference_phase_ns": list(times)}
    json.dump(meta, open(os.path.join(outdir, "cfg1_ref.json"), "w"), indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
