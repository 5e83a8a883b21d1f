#!/usr/bin/env python3
"""harness.py -- the reference's test drivers (GEMMul8/testing/test_double.cu, test_float.cu)
restated over the MI355X library, with the same sweeps and the same CSV schema, so results
line up with the published tables (GEMMul8/testing/results_in_paper/*.csv).

    python tools/harness.py d accuracy_check flops_check [--out-dir DIR] [--sizes ...]

type   d: DGEMM emulation (test_double.cu)      f: SGEMM emulation (test_float.cu)
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
Inputs: the reference generator (make_matrix.hpp:8-21, hiprand XORWOW, seed 123456, A and B from
the same seed); errors against the double-double product (eval.hpp:265-338).
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
PHASE_HDR = "conv_64f_2_8i,gpublasGemmEx,conv_32i_2_8u,inverse_scaling,"


def device_name():
    return torch.cuda.get_device_name(0).replace(" ", "_").replace("/", "_").replace("\\", "_")


def sync():
    torch.cuda.synchronize()


def relerr(C, C1, C2):
    """max / median of |C - (C1 + C2)| / |C1 + C2| in double-double (eval.hpp:317-338)"""
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
    """column-major A (m x k), B (k x n) from the reference generator, and the dd product"""

    def __init__(self, t, m, n, k, phi):
        dt = torch.float64 if t == "d" else torch.float32
        self.m, self.n, self.k, self.dt = m, n, k, dt
        self.A = G.randmat(m, k, dt, phi, SEED)
        self.B = G.randmat(k, n, dt, phi, SEED)
        self.C = torch.empty((n, m), dtype=dt, device="cuda")
        self.C1, self.C2 = G.dd_gemm(self.A.to(torch.float64), self.B.to(torch.float64), m, n, k)

    def vendor(self):
        """C = A B through the vendor GEMM (torch.matmul -> hipBLAS), stored column-major"""
        self.C.copy_(torch.matmul(self.A.t(), self.B.t()).t())

    def emulate(self, N, fast, work, phases=False):
        return G.gemm(G.OP_N, G.OP_N, self.m, self.n, self.k, 1.0, self.A, self.m, self.B, self.k, 0.0, self.C,
                      self.m, N, fast, work, phase_times=phases)


def accuracy_check(t, out, args):
    name = os.path.join(out, f"oz2_results_{t}_accuracy_{device_name()}_{args.stamp}.csv")
    m = n = 1024
    vend = "DGEMM" if t == "d" else "SGEMM"
    with open(name, "w") as f:
        f.write("phi,function," + "".join(f"{N}," for N in args.moduli) + "\n")
        for phi in args.phi:
            for k in args.ksizes:
                P = Problem(t, m, n, k, phi)
                work = G.alloc_work(m, n, k, max(args.moduli))
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
    vend = "DGEMM" if t == "d" else "SGEMM"
    with open(name, "w") as f:
        f.write("phi,m,n,k,function,relerr_max,relerr_med,TFLOPS,total_time [sec]," + PHASE_HDR + "\n")
        for s in args.sizes:
            m = n = k = s
            P = Problem(t, m, n, k, phi)
            work = G.alloc_work(m, n, k, max(args.moduli))
            flops = 2.0 * m * n * k
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
            tt = timed(P.vendor, args.iters)
            f.write(f"{phi:e},{m},{n},{k},{vend},{emax:e},{emed:e},{flops / tt * 1e-12:e},{tt:e},,,,,\n")
            for fast, lab in ((True, "OS2-fast"), (False, "OS2-accu")):
                for N in args.moduli:
                    P.emulate(N, fast, work)
                    sync()
                    emax, emed = relerr(P.C, P.C1, P.C2)
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
    vend = "DGEMM" if t == "d" else "SGEMM"
    with open(name, "w") as f:
        f.write("phi,m,n,k,function,relerr_max,relerr_med,watt,GFLOPS/watt,\n")
        for s in args.sizes:
            m = n = k = s
            P = Problem(t, m, n, k, 0.5)
            work = G.alloc_work(m, n, k, max(args.moduli))
            flops = 2.0 * m * n * k
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
    ap.add_argument("type", choices=["d", "f"])
    ap.add_argument("modes", nargs="+", choices=["accuracy_check", "flops_check", "watt_check", "all"])
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--sizes", type=int, nargs="+", default=SIZE)
    ap.add_argument("--ksizes", type=int, nargs="+", default=SIZE)
    ap.add_argument("--phi", type=float, nargs="+", default=PHI)
    ap.add_argument("--moduli", type=int, nargs="+", default=NUM_MODULI)
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args(argv)
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
