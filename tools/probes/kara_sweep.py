"""Complex GEMM time, Karatsuba sub-products vs the big-matrix product (GEMMUL8_CPLX_PRODUCTS forced
in a child process each), over square and skinny shapes, fast mode N = 12: the measurements behind
the size rule of csrc/oz2_common.hpp kara_default.  Usage: python tools/probes/kara_sweep.py [out.json]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHAPES = [(512, 512, 512), (768, 768, 768), (1024, 1024, 1024), (1536, 1536, 1536), (2048, 2048, 2048),
          (3072, 3072, 3072), (4096, 4096, 4096), (600, 500, 700), (4096, 256, 4096), (256, 4096, 4096),
          (8192, 8192, 1024)]


def child():
    sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
    import torch
    import gemmul8 as G
    out = {}
    for m, n, k in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(1)
        A = torch.randn((k, m), dtype=torch.complex128, device="cuda", generator=g)
        B = torch.randn((n, k), dtype=torch.complex128, device="cuda", generator=g)
        C = torch.empty((n, m), dtype=torch.complex128, device="cuda")
        W = G.alloc_work(m, n, k, 12, G.COMPLEX_BIG_MATRIX_ENCODE)
        f = lambda: G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 12, True, W, G.COMPLEX_BIG_MATRIX_ENCODE)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        it = max(3, min(50, int(2e12 / (8 * m * n * k))))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        out[f"{m}x{n}x{k}"] = {"ms": ms, "tflops": 8 * m * n * k / ms / 1e9, "nsub": G.layout(m, n, k, 12, 1)["nsub"]}
        del W, A, B, C
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        sys.exit(0)
    res = {}
    for tag, env in (("kara", {"GEMMUL8_CPLX_PRODUCTS": "karatsuba"}), ("bigmatrix", {"GEMMUL8_CPLX_PRODUCTS": "bigmatrix"})):
        r = subprocess.run([sys.executable, __file__, "--child"], env=dict(os.environ, **env), capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-3000:])
            sys.exit(r.returncode)
        res[tag] = json.loads(r.stdout.strip().splitlines()[-1])
    for s in res["kara"]:
        a, b = res["kara"][s], res["bigmatrix"][s]
        print(f"{s:>16}  kara {a['ms']:8.4f} ms ({a['tflops']:6.1f} TF)  big {b['ms']:8.4f} ms ({b['tflops']:6.1f} TF)"
              f"  kara/big {a['ms'] / b['ms']:.3f}")
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)
