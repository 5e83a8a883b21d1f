#!/usr/bin/env python3
"""harness.py -- the reference's test drivers (GEMMul8/testing/test_double.cu, test_float.cu,
test_mixed_double.cu, test_mixed_float.cu, test_float_complex.cu) restated over the MI355X library,
with the same sweeps and the same CSV schema, so results line up with the published tables
(GEMMul8/testing/results_in_paper/*.csv).

    python tools/harness.py d accuracy_check flops_check [--out-dir DIR] [--sizes ...]

type   d:   DGEMM emulation (test_double.cu)             f:  SGEMM emulation (test_float.cu)
       dfd: A f64 x B f32 -> C f64 (test_mixed_double.cu) dff: A f64 x B f32 -> C f32 (test_mixed_float.cu)
       fC:  complex f32, COMPLEX_KARATSUBA_MULT (test_float_complex.cu)
       TFLOPS = 2mnk / time for every type, fC included, as the reference's CSVs have it (multiply
       by 4 for complex flops).  The sweep defaults follow each driver (moduli 2..20 and phi 0.5..4 for d / dfd; 2..15 and
       phi 0..1.5 for f / dff / fC).  The reference's "SGEMM-TF32" / "CGEMM-TF32" rows have no
       MI355X counterpart and are not written.
modes  accuracy_check  oz2_results_<t>_accuracy_<device>_<date>.csv
                       "phi,function,2,...,20," rows DGEMM (k=K) / OS2-fast (k=K) / OS2-accu (k=K)
                       of max relative error (test_double.cu:70-200)
       flops_check     oz2_results_<t>_time_<device>_<date>.csv
                       "phi,m,n,k,function,relerr_max,relerr_med,TFLOPS,total_time [sec],
                        conv_64f_2_8i,gpublasGemmEx,conv_32i_2_8u,inverse_scaling," rows INT8-GEMM,
                       DGEMM, OS2-fast-N, OS2-accu-N (test_double.cu:202-496); the phase columns
                       are this build's {scaling, int8 products, 0 (fused), CRT} in seconds
       watt_check      oz2_results_<t>_watt_<device>_<date>.csv (test_double.cu:498-745), when the
                       amdsmi Python module is importable; skipped otherwise
Inputs: the reference generator (make_matrix.hpp:8-71, hiprand XORWOW, seed 123456, A and B from
the same seed); errors against the double-double product for real types (eval.hpp:265-338), against
the FP64 complex product for fC (|C - Cref| / |Cref| with complex abs, eval.hpp:360-379).
"""
import argparse
import datetime
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402

SEED = 123456
PHI = [0.5, 1, 2, 3, 4]
SIZE = [1024, 2048, 4096, 8192]
NUM_MODULI = list(range(2, 21))
# per driver: (A, B, C) dtypes, compute type, vendor routine name, default phi list, default moduli
F64, F32, C64 = torch.float64, torch.float32, torch.complex64
TYPES = {
    "d": ((F64, F64, F64), 0, "DGEMM", PHI, NUM_MODULI),
    "f": ((F32, F32, F32), 0, "SGEMM", [0.0, 0.5, 1, 1.5], list(range(2, 16))),
    "dfd": ((F64, F32, F64), 0, "DGEMM", PHI, NUM_MODULI),
    "dff": ((F64, F32, F32), 0, "SGEMM", [0.0, 0.5, 1, 1.5], list(range(2, 16))),
    "fC": ((C64, C64, C64), 3, "CGEMM", [0.0, 0.5, 1, 1.5], list(range(2, 16))),
}
PHASE_HDR = "conv_64f_2_8i,gpublasGemmEx,conv_32i_2_8u,inverse_scaling,"


def device_name():
    return torch.cuda.get_device_name(0).replace(" ", "_").replace("/", "_").replace("\\", "_")


def sync():
    torch.cuda.synchronize()


def relerr(C, C1, C2):
    """max / median of |C - (C1 + C2)| / |C1 + C2| in double-double (eval.hpp:317-338); complex C
    against the FP64 product C1 (C2 unused): |C - C1| / |C1| (eval.hpp:360-379)"""
    if C.is_complex():
        e = ((C.to(torch.complex128) - C1).abs() / C1.abs()).flatten()
        return float(e.max()), float(e.median())
    return G.relerr_dd(C.to(torch.float64) if C.dtype != torch.float64 else C, C1, C2)


def timed(fn, iters):
    fn()
    sync()
    t = 0.0
    for _ in range(iters):
        sync()
        t0 = time.perf_counter()
        fn()
        sync()
        t += time.perf_counter() - t0
    return t / iters


class Problem:
    """column-major A (m x k), B (k x n) from the reference generator, and the reference product"""

    def __init__(self, t, m, n, k, phi):
        (ta, tb, tc), self.ct, self.vend_name, _, _ = TYPES[t]
        self.m, self.n, self.k = m, n, k
        self.A = G.randmat(m, k, ta, phi, SEED)
        self.B = G.randmat(k, n, tb, phi, SEED)
        self.C = torch.empty((n, m), dtype=tc, device="cuda")
        if tc.is_complex:  # FP64 complex product of the upcast operands (test_float_complex.cu:328)
            self.C1 = torch.matmul(self.A.t().to(torch.complex128), self.B.t().to(torch.complex128)).t().contiguous()
            self.C2 = None
        else:
            self.C1, self.C2 = G.dd_gemm(self.A.to(torch.float64), self.B.to(torch.float64), m, n, k)
        # the vendor routine's operands: DGEMM on B upcast (test_mixed_double.cu:139), SGEMM on A
        # downcast (test_mixed_float.cu:158), else the operands as they are
        self.vA = self.A.to(tc) if tc != ta else self.A
        self.vB = self.B.to(tc) if tc != tb else self.B

    def vendor(self):
        """C = A B through the vendor GEMM (torch.matmul -> hipBLAS), stored column-major"""
        self.C.copy_(torch.matmul(self.vA.t(), self.vB.t()).t())

    def emulate(self, N, fast, work, phases=False):
        return G.gemm(G.OP_N, G.OP_N, self.m, self.n, self.k, 1.0, self.A, self.m, self.B, self.k, 0.0, self.C,
                      self.m, N, fast, work, self.ct, phase_times=phases)

    def work(self, N):
        return G.alloc_work(self.m, self.n, self.k, N, self.ct)


def accuracy_check(t, out, args):
    name = os.path.join(out, f"oz2_results_{t}_accuracy_{device_name()}_{args.stamp}.csv")
    m = n = 1024
    vend = TYPES[t][2]
    with open(name, "w") as f:
        f.write("phi,function," + "".join(f"{N}," for N in args.moduli) + "\n")
        for phi in args.phi:
            for k in args.ksizes:
                P = Problem(t, m, n, k, phi)
                work = P.work(max(args.moduli))
                P.vendor()
                sync()
                emax, _ = relerr(P.C, P.C1, P.C2)
                f.write(f"{phi},{vend} (k={k})," + "".join(f"{emax:e}," for _ in args.moduli) + "\n")
                for fast, lab in ((True, "OS2-fast"), (False, "OS2-accu")):
                    row = []
                    for N in args.moduli:
                        P.emulate(N, fast, work)
                        sync()
                        row.append(relerr(P.C, P.C1, P.C2)[0])
                    f.write(f"{phi:e},{lab} (k={k})," + "".join(f"{e:e}," for e in row) + "\n")
                f.flush()
                print(f"accuracy phi={phi} k={k} done", flush=True)
    return name


def flops_check(t, out, args):
    name = os.path.join(out, f"oz2_results_{t}_time_{device_name()}_{args.stamp}.csv")
    phi = 0.5
    vend = TYPES[t][2]
    with open(name, "w") as f:
        f.write("phi,m,n,k,function,relerr_max,relerr_med,TFLOPS,total_time [sec]," + PHASE_HDR + "\n")
        for s in args.sizes:
            m = n = k = s
            P = Problem(t, m, n, k, phi)
            work = P.work(max(args.moduli))
            flops = 2.0 * m * n * k  # fC too: the reference prints 2mnk (test_float_complex.cu:355)
            # INT8-GEMM: one int8 product of the emulator's own kernel (all-ones operands)
            L = G.layout(m, n, k, 2)
            work[L["offA"]:L["offB"] + L["planeB"] * 2].fill_(1)
            C32 = torch.empty((L["n_pad"], L["m_pad"]), dtype=torch.int32, device="cuda")
            import ctypes
            raw = lambda: G.lib.gemmul8_i8_product_raw(G._stream(), m, n, k, 2, 0, ctypes.c_void_p(work.data_ptr()),
                                                       ctypes.c_void_p(C32.data_ptr()))
            tt = timed(raw, args.iters)
            f.write(f"{phi},{m},{n},{k},INT8-GEMM,,,{flops / tt * 1e-12:e},{tt:e},,,,,\n")
            P.vendor()
            sync()
            emax, emed = relerr(P.C, P.C1, P.C2)
            # the drivers' loop (device sync + host clock around each call) in native code, as the reference's
            # C++ drivers time it: no Python call overhead on either side
            tt = G.time_vendor_gemm(m, n, k, P.vA, P.vB, P.C, args.iters) if args.native_timing else \
                timed(P.vendor, args.iters)
            f.write(f"{phi:e},{m},{n},{k},{vend},{emax:e},{emed:e},{flops / tt * 1e-12:e},{tt:e},,,,,\n")
            for fast, lab in ((True, "OS2-fast"), (False, "OS2-accu")):
                for N in args.moduli:
                    P.emulate(N, fast, work)
                    sync()
                    emax, emed = relerr(P.C, P.C1, P.C2)
                    if args.native_timing:
                        tt, ph = G.time_gemm(G.OP_N, G.OP_N, m, n, k, 1.0, P.A, m, P.B, k, 0.0, P.C, m, N, fast,
                                             work, args.iters, P.ct)
                        ph = [x * 1e-9 for x in ph]
                    else:
                        ph = [0.0] * 4
                        tt = 0.0
                        for _ in range(args.iters):
                            sync()
                            t0 = time.perf_counter()
                            p = P.emulate(N, fast, work, phases=True)
                            sync()
                            tt += time.perf_counter() - t0
                            ph = [a + b for a, b in zip(ph, p)]
                        tt /= args.iters
                        ph = [x / args.iters * 1e-9 for x in ph]
                    f.write(f"{phi:e},{m},{n},{k},{lab}-{N},{emax:e},{emed:e},{flops / tt * 1e-12:e},{tt:e},"
                            + "".join(f"{x:e}," for x in ph) + "\n")
                f.flush()
            print(f"flops n={s} done", flush=True)
    return name


def watt_check(t, out, args):
    try:
        import amdsmi  # noqa: F401
    except Exception:
        print("watt_check skipped: the amdsmi Python module is not importable here", flush=True)
        return None
    import threading
    import amdsmi
    amdsmi.amdsmi_init()
    dev = amdsmi.amdsmi_get_processor_handles()[0]

    def power():
        info = amdsmi.amdsmi_get_power_info(dev)
        avg = info.get("average_socket_power", 0)
        return float(info.get("current_socket_power", avg) if avg in ("N/A", 0) or avg >= 10000 else avg)

    def measure(fn, flops):
        samples, stop = [], [False]

        def sampler():
            while not stop[0]:
                samples.append(power())
                time.sleep(0.01)
        th = threading.Thread(target=sampler)
        th.start()
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < 1.0:
            fn()
            sync()
            reps += 1
        dt = time.perf_counter() - t0
        stop[0] = True
        th.join()
        w = sum(samples) / max(len(samples), 1)
        return w, flops * reps / dt / w * 1e-9

    name = os.path.join(out, f"oz2_results_{t}_watt_{device_name()}_{args.stamp}.csv")
    vend = TYPES[t][2]
    with open(name, "w") as f:
        f.write("phi,m,n,k,function,relerr_max,relerr_med,watt,GFLOPS/watt,\n")
        for s in args.sizes:
            m = n = k = s
            P = Problem(t, m, n, k, 0.5)
            work = P.work(max(args.moduli))
            flops = 2.0 * m * n * k  # fC too: the reference prints 2mnk (test_float_complex.cu:355)
            P.vendor()
            sync()
            emax, emed = relerr(P.C, P.C1, P.C2)
            w, gfw = measure(P.vendor, flops)
            f.write(f"0.5,{m},{n},{k},{vend},{emax:e},{emed:e},{w:e},{gfw:e},\n")
            for fast, lab in ((True, "OS2-fast"), (False, "OS2-accu")):
                for N in args.moduli:
                    P.emulate(N, fast, work)
                    sync()
                    emax, emed = relerr(P.C, P.C1, P.C2)
                    w, gfw = measure(lambda: P.emulate(N, fast, work), flops)
                    f.write(f"0.5,{m},{n},{k},{lab}-{N},{emax:e},{emed:e},{w:e},{gfw:e},\n")
            f.flush()
    return name


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("type", choices=list(TYPES))
    ap.add_argument("modes", nargs="+", choices=["accuracy_check", "flops_check", "watt_check", "all"])
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--sizes", type=int, nargs="+", default=SIZE)
    ap.add_argument("--ksizes", type=int, nargs="+", default=SIZE)
    ap.add_argument("--phi", type=float, nargs="+", default=None, help="default: the driver's list")
    ap.add_argument("--moduli", type=int, nargs="+", default=None, help="default: the driver's list")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--python-timing", action="store_true",
                    help="time each call from Python (per-call binding overhead included) instead of the native loop")
    args = ap.parse_args(argv)
    args.native_timing = not args.python_timing
    args.phi = args.phi or TYPES[args.type][3]
    args.moduli = args.moduli or TYPES[args.type][4]
    args.stamp = datetime.datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    os.makedirs(args.out_dir, exist_ok=True)
    modes = {"accuracy_check", "flops_check", "watt_check"} if "all" in args.modes else set(args.modes)
    out = []
    if "accuracy_check" in modes:
        out.append(accuracy_check(args.type, args.out_dir, args))
    if "flops_check" in modes:
        out.append(flops_check(args.type, args.out_dir, args))
    if "watt_check" in modes:
        out.append(watt_check(args.type, args.out_dir, args))
    for o in out:
        if o:
            print("wrote", o)
    return out


if __name__ == "__main__":
    main()
