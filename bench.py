#!/usr/bin/env python3
"""bench.py -- emulated DGEMM throughput of the MI355X Ozaki-II emulator (BASELINE.json metric).

Workload (BASELINE.json configs[1], "cfg2"): DGEMM emulation, m = n = k = 8192,
num_moduli = 14, fast mode, NN, alpha = 1, beta = 0, inputs from the reference
driver's generator (hiprand XORWOW, (U - 0.5) * exp(0.5 * N(0,1)), seed 123456,
A and B identical as in GEMMul8/testing/test_double.cu:273-274).

One "step" = one gemmul8 DGEMM call (scaling -> N int8 products -> CRT) with the
operands resident in HBM.  TFLOP/s = 2*m*n*k / time (test_double.cu:440).

Multi-GPU (torchrun, one process per GPU, RCCL), --partition:
  rows (default)  weak scaling by output row blocks -- rank r computes the 8192-row
                  block r of C = A * B for an (8192*N) x 8192 x 8192 product; B is
                  replicated, no data-path collective (fast-mode shifts of a row depend
                  only on that row, so the blocks are bit-identical to a single-GPU run
                  of the whole product; gemmul8/dist.py).
  moduli          strong scaling of ONE m=n=k=size product: rank r computes the residue
                  planes of its moduli and sends them to rank 0 (P2P over xGMI), which
                  runs the CRT (gemmul8.dist.matmul_moduli).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
import sys  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))

INT8_PEAK_TOPS = 2048 * 4 * 256 * 2.4e9 / 1e12  # v_mfma_i32_32x32x32_i8: 2048 ops/clk/SIMD, 4 SIMD x 256 CU @ 2.4 GHz
HBM_PEAK_GBS = 8000.0
GH200_PUBLISHED_TFLOPS = 72.13  # OS2-fast-14 8192 on GH200 (R/...GH200...csv:192)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--moduli", type=int, default=14)
    ap.add_argument("--accurate", action="store_true")
    ap.add_argument("--partition", choices=["rows", "moduli"], default="rows")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-accuracy", action="store_true")
    ap.add_argument("--no-dgemm", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="CPU baseline size (default: auto)")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # one GPU per rank; GEMMUL8_BENCH_BACKEND=gloo (with ranks sharing a device) rehearses the
        # multi-rank flow on a one-GPU box -- timing from such a run means nothing
        backend = os.environ.get("GEMMUL8_BENCH_BACKEND", "nccl")
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(size_hint):
    """The oracle (CPU restatement, OpenMP) timed on a bounded sample of the same workload."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    threads = O.num_threads()
    n = size_hint or 5120  # about 14 s of the oracle on 16 host threads (6.9 s at 4096)
    rng = np.random.default_rng(123456)
    A = np.asfortranarray((1.0 - rng.random((n, n)) - 0.5) * np.exp(0.5 * rng.standard_normal((n, n))))
    t0 = time.perf_counter()
    O.gemm(A, A, 14, True)
    dt = time.perf_counter() - t0
    model = "unknown CPU"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": 2.0 * n ** 3 / dt / 1e12, "unit": "TFLOP/s", "cores": threads, "kind": "port",
            "sample": f"DGEMM emulation m=n=k={n}, num_moduli=14, fast mode, one call ({dt:.1f} s) of the "
                      f"oracle/oz2_oracle.c restatement with {threads} OpenMP threads on {model} "
                      f"({os.cpu_count()} logical CPUs visible)"}


def traffic_from_profile(shape):
    """PMC bytes per product launch, from the committed --pmc passes; only for the shape they measured
    (m, n, k, num_moduli planes per launch, fast mode), else None"""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        t = json.load(open(p))
    except Exception:
        return None
    if tuple(t.get("shape", ())) != tuple(shape):
        return None
    return t.get("gemm_hbm_bytes_per_launch")


def main():
    args = parse()
    world, rank = dist_setup(args)
    import gemmul8 as G

    m = n = k = args.size
    N = args.moduli
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.partition == "moduli" and world > 1:
        from gemmul8 import dist as GD
        # row-major m x k / k x n operands (randmat(k, m) is the column-major k x m matrix)
        Arm = G.randmat(k, m, torch.float64, 0.5, 123456, dev)
        Brm = G.randmat(n, k, torch.float64, 0.5, 654321, dev)
        A = B = None

        def step():
            GD.matmul_moduli(Arm, Brm, N, not args.accurate)
    else:
        # inputs (column-major; the (k, m) row-major tensor holds the column-major m x k matrix)
        seed = 123456 + rank
        A = G.randmat(m, k, torch.float64, 0.5, seed, dev)
        B = G.randmat(k, n, torch.float64, 0.5, 123456, dev)
        C = torch.empty((n, m), dtype=torch.float64, device=dev)
        work = G.alloc_work(m, n, k, N, G.REAL_DEFAULT, dev)

        def step():
            G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, not args.accurate, work)

        if args.accurate and world > 1:
            # accurate mode couples B's column shifts to every row block: one MAX all-reduce of
            # the bound product's column maxima per call (gemmul8.dist.matmul_rows)
            from gemmul8 import dist as GD
            Arm = G.randmat(k, m, torch.float64, 0.5, seed, dev)
            Brm = G.randmat(n, k, torch.float64, 0.5, 123456, dev)
            A = B = None

            def step():
                GD.matmul_rows(Arm, Brm, N, False)

    for _ in range(args.warmup):
        step()
    G.timing_enable(True)
    G.timing_read()  # reset
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier(world)
    dt = time.perf_counter() - t0
    G.timing_enable(False)
    phase_ms, _ = G.timing_read()
    dt = max_over_ranks(dt, world)
    ms_per_step = dt / args.steps * 1e3
    flops = 2.0 * m * n * k
    strong = args.partition == "moduli" and world > 1
    value = flops * (1 if strong else world) * args.steps / dt / 1e12

    out = None
    if rank == 0:
        # per step: one gemm call (single GPU, row blocks) or, in the modulus partition, one product
        # launch per owned plane (gemmul8.dist.matmul_moduli; its split and CRT go through the phase
        # entry points, which time the products only)
        avg = [x / args.steps for x in phase_ms]
        # dominant kernel: the int8 products (all of this rank's moduli per step)
        gemm_ms = avg[1]
        planes = N
        if strong:
            from gemmul8 import dist as GD
            a, b = GD.moduli_partition(N, world)[0]
            planes = b - a  # rank 0's share of the moduli
        ops = 2.0 * m * n * k * planes
        achieved = ops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
        roofline = {"bound": "mfma", "achieved": round(achieved, 1), "peak": round(INT8_PEAK_TOPS, 1),
                    "unit": "TFLOP/s", "frac": round(achieved / INT8_PEAK_TOPS, 4), "traffic": traffic_from_profile((m, n, k, planes, not args.accurate)),
                    "kernel": "gemm_i8_persistent_kernel (residue products; int8 ops counted as FLOP, 2*m*n*k*num_moduli per launch)",
                    "avg_launch_ms": round(gemm_ms, 4)}
        # measured live after the timed region: the same MFMA alone on uniformly random operand bytes
        # (the residue distribution) in registers -- the clock the chip holds under that load bounds
        # any int8 GEMM on such data
        ceiling = G.mfma_ceiling()
        if ceiling > 0:
            roofline["data_bound_ceiling"] = round(ceiling, 1)
            roofline["frac_of_data_bound_ceiling"] = round(achieved / ceiling, 4)
        extra = {"phase_ms": {"scaling": round(avg[0], 4), "int8_products": round(avg[1], 4),
                              "inverse_scaling": round(avg[3], 4)}}
        if not args.no_accuracy and A is not None:
            # accuracy against a double-double reference (testing/eval.hpp semantics)
            step()
            torch.cuda.synchronize()
            C1, C2 = G.dd_gemm(A, B, m, n, k)
            emax, emed = G.relerr_dd(C, C1, C2)
            extra["relerr_max"] = emax
            extra["relerr_median"] = emed
            del C1, C2
        if not args.no_dgemm and A is not None:
            Ar = A.t()  # logical m x k view
            Br = B.t()
            for _ in range(2):
                torch.matmul(Ar, Br)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            reps = 5
            for _ in range(reps):
                torch.matmul(Ar, Br)
            torch.cuda.synchronize()
            dg = flops * reps / (time.perf_counter() - t1) / 1e12
            extra["rocblas_dgemm_tflops"] = round(dg, 2)
            extra["vs_rocblas_dgemm"] = round(value / world / dg, 3)
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(args.cpu_sample)
        out = {
            "metric": "emulated DGEMM TFLOP/s + max rel-error, m=n=k=8192 num_moduli=14",
            "value": round(value, 3),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": round(value / world / GH200_PUBLISHED_TFLOPS, 3),
            "vs_baseline_ref": "GH200 published OS2-fast-14 8192 (72.13 TFLOP/s, BASELINE.md); per-GPU ratio",
            "dtype": "i8",
            "io_dtype": "f64",
            "data": "synthetic: hiprand XORWOW (U-0.5)*exp(0.5*N(0,1)), seed 123456 (rank r: A seed 123456+r), "
                    "A == B at N=1 as in the reference driver",
            "config": {"workload": "cfg2: DGEMM emulation m=n=k=8192, num_moduli=14, fast mode, NN, alpha=1 beta=0"
                       if (m == 8192 and N == 14 and not args.accurate) else
                       f"DGEMM emulation m=n=k={m}, num_moduli={N}, {'accurate' if args.accurate else 'fast'} mode",
                       "m": m, "n": n, "k": k, "num_moduli": N, "fastmode": not args.accurate,
                       "parallelism": (f"{args.partition} x{world}" if world > 1 else "single")},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        out.update(extra)
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
