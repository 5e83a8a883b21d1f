#!/usr/bin/env python3
"""bench.py -- emulated DGEMM throughput of the MI355X Ozaki-II emulator (BASELINE.json metric).

Workloads (BASELINE.json configs):
  cfg2 (default at --gpus 1)  DGEMM emulation m = n = k = 8192, num_moduli = 14, fast mode, 1 GPU
  cfg3 (default at --gpus N>1) DGEMM emulation m = n = k = 16384, num_moduli = 14, fast mode, the
                               (modulus, column block) units sharded over N GPUs: strong scaling of ONE product,
                               C left distributed.  --partition auto (default): at an even N >= 4 the 2-D unit
                               grid (gemmul8.dist.gemm_moduli_grid: 2 row blocks, each a (modulus, column block)
                               partition of its rows over N / 2 ranks), else gemmul8.dist.gemm_moduli over all N;
                               the other one is timed among the variants
  cfg4                         mixed FP64 * FP32 -> FP64, 8192^3, num_moduli = 10, accurate mode, 1 GPU
  cfg5                         complex DGEMM (COMPLEX_BIG_MATRIX_ENCODE), 4096^3, num_moduli = 12, 1 GPU
Inputs come from the reference driver's generator (hiprand XORWOW, (U - 0.5) * exp(0.5 * N(0,1)),
seed 123456, A and B identical for square shapes as in GEMMul8/testing/test_double.cu:273-274),
NN, alpha = 1, beta = 0.  One "step" = one emulated GEMM with the operands resident in HBM.
TFLOP/s = 2 m n k / time (8 m n k complex; test_double.cu:440).

--gpus N without a torchrun environment re-launches itself under torch.distributed.run with N
ranks (one process per GPU, RCCL) before touching the GPU.  --partition rows selects the weak-scaling
row-block partition instead (rank r: the 8192-row block r of an (8192 N) x 8192 x 8192 product).

Prints ONE JSON line on rank 0.
"""
import argparse
import datetime
import hashlib
import json
import os
import socket
import subprocess
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))

INT8_PEAK_TOPS = 2048 * 4 * 256 * 2.4e9 / 1e12  # v_mfma_i32_32x32x32_i8: 2048 ops/clk/SIMD, 4 SIMD x 256 CU @ 2.4 GHz
HBM_PEAK_GBS = 8000.0
GH200_PUBLISHED_TFLOPS = 72.13  # OS2-fast-14 8192 on GH200 (R/...GH200...csv:192)
BASELINE_METRIC = "emulated DGEMM TFLOP/s + max rel-error, m=n=k=8192 num_moduli=14"

WORKLOADS = {
    "cfg2": dict(size=8192, moduli=14, accurate=False, kind="d",
                 text="cfg2: DGEMM emulation m=n=k=8192, num_moduli=14, fast mode, NN, alpha=1 beta=0"),
    "cfg3": dict(size=16384, moduli=14, accurate=False, kind="d",
                 text="cfg3: DGEMM emulation m=n=k=16384, num_moduli=14, fast mode, moduli sharded over the GPUs"),
    "cfg4": dict(size=8192, moduli=10, accurate=True, kind="dfd",
                 text="cfg4: mixed FP64*FP32->FP64 m=n=k=8192, num_moduli=10, accurate mode"),
    "cfg5": dict(size=4096, moduli=12, accurate=False, kind="z",
                 text="cfg5: complex DGEMM (COMPLEX_BIG_MATRIX_ENCODE) m=n=k=4096, num_moduli=12, fast mode"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None,
                    help="default: cfg2 on one GPU, cfg3 on more")
    ap.add_argument("--size", type=int, default=None, help="override m = n = k")
    ap.add_argument("--moduli", type=int, default=None)
    ap.add_argument("--accurate", action="store_true")
    ap.add_argument("--partition", choices=["auto", "moduli", "grid", "rows"], default="auto",
                    help="multi-GPU: auto = grid (gemm_moduli_grid, 2 row blocks) for fast mode on an even W >= 4 whose "
                         "sub-groups exist, else moduli (gemm_moduli); rows = the weak-scaling row partition")
    ap.add_argument("--order", choices=["moduli", "columns"], default="moduli",
                    help="moduli partition: unit order of gemmul8.dist.ShardPlan")
    ap.add_argument("--gather", action="store_true", help="moduli partition: collect C on rank 0 in the step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-accuracy", action="store_true")
    ap.add_argument("--no-dgemm", action="store_true")
    ap.add_argument("--no-cfg3-1gpu", action="store_true", help="N = 1: skip timing cfg3's shape on the one GPU")
    ap.add_argument("--no-power", action="store_true", help="no amdsmi power / clock sampling during the timed steps")
    ap.add_argument("--no-variants", action="store_true", help="sharded runs: skip timing the other partitions")
    ap.add_argument("--cpu-sample", type=int, default=0, help="CPU baseline size (default: auto)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline OpenMP threads (default: OMP_NUM_THREADS, the host's CPU share for this job)")
    ap.add_argument("--no-single-gpu", action="store_true",
                    help="sharded runs: skip timing the same call on one GPU after the timed region")
    return ap.parse_args(argv)


# The line's dicts (extra, its variants, roofline) change after the timed region while the watchdog thread
# may serialise them (an optional phase got stuck): every such change and every serialisation takes this lock,
# and nothing that can block runs under it.
STATE_LOCK = threading.Lock()


def put(d, key, value):
    with STATE_LOCK:
        d[key] = value


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_command(args, argv):
    """the torch.distributed.run command line of a --gpus N > 1 run started outside torchrun (None: run here)"""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)


def maybe_launch(args):
    """--gpus N > 1 outside torchrun: run N ranks under torch.distributed.run as a child (no GPU touched
    in this process) and exit with its status."""
    cmd = launch_command(args, sys.argv[1:])
    if cmd is None:
        return
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    if world > 1:
        import torch.distributed as dist
        # one GPU per rank; GEMMUL8_BENCH_BACKEND=gloo (with ranks sharing a device) rehearses the
        # multi-rank flow on a one-GPU box -- timing from such a run means nothing
        backend = os.environ.get("GEMMUL8_BENCH_BACKEND", "nccl")
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        # stdout carries rank 0's one JSON line only: what the communication libraries print while they
        # connect (gloo announces its peers on fd 1) goes to stderr, and so does everything of the other ranks
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        # explicit communicator timeout: a peer that never arrives fails the run in minutes, not at the
        # default watchdog's limit (GEMMUL8_DIST_TIMEOUT seconds, default 300)
        tmo = datetime.timedelta(seconds=float(os.environ.get("GEMMUL8_DIST_TIMEOUT", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        if world >= 4 and world % 2 == 0 and os.environ.get("GEMMUL8_BENCH_NO_GRID") is None:
            # the sub-groups of the 2-D grid variant, created now: the communication libraries announce new
            # groups on fd 1 (gloo does), and stdout must carry rank 0's one JSON line only
            sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
            from gemmul8 import dist as GD
            ok = 1
            try:
                GD.grid_groups(world, 2)
            except Exception as e:  # the variant then reports its failure; the measured line does not depend on it
                print(f"bench: grid sub-groups: {type(e).__name__}: {str(e)[:200]}", file=sys.stderr, flush=True)
                ok = 0
            # every rank skips the variant if any rank failed: a rank entering the sub-group collectives alone
            # would stall the variant phase until the watchdog (MIN over ranks of a success flag)
            flag = torch.tensor([ok], dtype=torch.int32, device=f"cuda:{local}" if backend == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag.item()) == 0:
                os.environ["GEMMUL8_BENCH_NO_GRID"] = "1"
        dist.barrier()  # the connections are up before stdout is given back
        world = dist.get_world_size()
        rank = dist.get_rank()
        if rank == 0:
            os.dup2(saved, 1)
        os.close(saved)
    else:
        torch.cuda.set_device(0)
    return world, rank, backend


class StepPower:
    """Board power and clocks of this process's GPU while a loop of steps runs (sampled in
    process): the SMU's gpu_metrics table read through amdsmi every `period` s by a thread (tools/power_trace.py's
    sampler), and the energy accumulator across the loop.  Any failure (no amdsmi, no permission) leaves the line
    without the field."""

    def __init__(self, period=0.005):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import amdsmi
        import power_trace as PT
        amdsmi.amdsmi_init()
        self.smi, self.PT, self.period = amdsmi, PT, period
        self.dev, _ = PT.find_device(amdsmi)
        cap = amdsmi.amdsmi_get_power_cap_info(self.dev)
        self.cap_w = cap.get("power_cap", 0) / 1e6 if isinstance(cap, dict) else None
        self.sampler, self.e0 = None, None

    def _energy(self):
        e = self.smi.amdsmi_get_energy_count(self.dev)
        self.res = float(e.get("counter_resolution") or 15.259)  # microjoules per count
        return e["energy_accumulator"] * self.res * 1e-6, time.perf_counter()

    def begin(self):
        self.e0 = self._energy()
        self.sampler = self.PT.Sampler(self.smi, self.dev, self.period)
        self.sampler.phase = "steps"
        self.sampler.start()

    def end(self, steps, settle=0.0):
        e1 = self._energy()
        self.sampler.stop_ev.set()
        self.sampler.join()
        rows = self.sampler.rows[int(len(self.sampler.rows) * settle):]
        mean = lambda key: round(sum(r[key] for r in rows if r.get(key) is not None) /
                                 max(1, sum(1 for r in rows if r.get(key) is not None)), 1)
        clk = [sum(r[f"gfxclk{i}"] for i in range(8)) / 8 for r in rows if all(r.get(f"gfxclk{i}") for i in range(8))]
        out = {"samples": len(rows), "period_ms": self.period * 1e3, "power_cap_W": self.cap_w,
               "socket_power_W_mean": mean("current_socket_power"),
               "gfxclk_MHz_mean_8xcd": round(sum(clk) / len(clk), 1) if clk else None,
               "hotspot_C_mean": mean("temperature_hotspot")}
        total = e1[1] - self.e0[1]
        a, b = (rows[0], rows[-1]) if len(rows) >= 2 else (None, None)
        if a and a.get("energy_accumulator") is not None and b.get("energy_accumulator") is not None and total > 0:
            # over the settled window, from the samples' own accumulator readings (the step rate is the loop's)
            joules, dt = (b["energy_accumulator"] - a["energy_accumulator"]) * self.res * 1e-6, b["t"] - a["t"]
            if dt > 0 and joules > 0:
                out["energy_per_step_J"] = round(joules / (steps * dt / total), 4)
                out["power_from_energy_W"] = round(joules / dt, 1)
        if a and a.get("ppt_residency_acc") is not None and b.get("accumulation_counter") and \
                b["accumulation_counter"] > a["accumulation_counter"]:
            out["ppt_limiter_residency"] = round((b["ppt_residency_acc"] - a["ppt_residency_acc"]) /
                                                 (b["accumulation_counter"] - a["accumulation_counter"]), 3)
        out["loop_ms_per_step"] = round(total / steps * 1e3, 4) if steps else None
        try:
            self.smi.amdsmi_shut_down()
        except Exception:
            pass
        return out


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def reduce_max(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _physical_cores():
    """distinct (socket, core) pairs in /proc/cpuinfo (the whole host), or None"""
    try:
        cores, phys = set(), None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":", 1)[1].strip()))
        return len(cores) or None
    except OSError:
        return None


def cpu_baseline(size_hint, dev, gpu_C=None, threads_req=0):
    """The oracle (CPU restatement, OpenMP) timed on a bounded sample of the cfg2 workload (same generator,
    fast mode, N = 14) and cfg1 (SGEMM emulation 1024^3, N = 4, fast) in full, both on this host.
    gpu_C: the GPU line's C of the same call (column-major, (n, m) tensor): the oracle's C is compared with it
    byte for byte, and its error is measured against the double-double reference GEMM (eval.hpp semantics)."""
    import numpy as np
    import gemmul8 as G
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    # threads: every CPU this job is allotted.  On the GPU pool a one-GPU job's share is 16 CPUs of the host
    # (the harness exports OMP_NUM_THREADS=16 and bounds worker pools to that share) although the affinity mask
    # lists all of the host's CPUs; --cpu-threads overrides it on a dedicated host
    if threads_req > 0:
        O.set_num_threads(threads_req)
    threads = O.num_threads()
    # the full cfg2 size (full size when it fits the time budget): the oracle's int8 products run
    # blocked on AVX-512 VNNI where the host has it (about 4 s at 4096 on 8 threads of this container)
    n = size_hint or 8192
    A = G.randmat(n, n, torch.float64, 0.5, 123456, dev).cpu().numpy().T  # column-major n x n (F order)
    t0 = time.perf_counter()
    C = O.gemm(A, A, 14, True)
    dt = time.perf_counter() - t0
    affinity = len(os.sched_getaffinity(0))
    out = {"value": 2.0 * n ** 3 / dt / 1e12, "unit": "TFLOP/s", "cores": threads, "kind": "port",
           "sample": f"cfg2 workload at m=n=k={n} (DGEMM emulation, num_moduli=14, fast mode, reference "
                     f"generator seed 123456, A == B), one call ({dt:.1f} s) of the oracle/oz2_oracle.c "
                     f"restatement (int8 products on AVX-512 VNNI: {O.vnni()}) with {threads} OpenMP threads on "
                     f"{_cpu_model()} ({affinity} CPUs in this process's affinity mask, "
                     f"{os.cpu_count()} logical CPUs in the machine)",
           "threads": threads, "affinity_cpus": affinity, "logical_cpus_machine": os.cpu_count(),
           "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
           "threads_policy": ("--cpu-threads" if threads_req > 0 else
                              "OpenMP default = OMP_NUM_THREADS (the CPUs allotted to a one-GPU job on the GPU pool; "
                              "the affinity mask shows the whole host, which other jobs share)")}
    dA = torch.from_numpy(np.ascontiguousarray(A.T)).to(dev)
    C1, C2 = G.dd_gemm(dA, dA, n, n, n)
    dC = torch.from_numpy(np.ascontiguousarray(C.T)).to(dev)
    emax, emed = G.relerr_dd(dC, C1, C2)
    out["relerr_max"], out["relerr_median"] = emax, emed  # against the double-double GEMM, as the GPU line
    if gpu_C is not None and tuple(gpu_C.shape) == (n, n):
        out["bit_identical_to_gpu_C"] = bool(torch.equal(gpu_C.view(torch.uint8), dC.view(torch.uint8)))
    del C1, C2, dA, dC
    # how the port scales with threads (a 2048^3 sample of the same workload at 1, 2, 4, ... threads up to the
    # count above), so the rate on a host's every core can be read off without running there
    A2 = G.randmat(2048, 2048, torch.float64, 0.5, 123456, dev).cpu().numpy().T
    scaling = {}
    t = 1
    while t <= threads:
        O.set_num_threads(t)
        t0 = time.perf_counter()
        O.gemm(A2, A2, 14, True)
        scaling[str(t)] = round(2.0 * 2048 ** 3 / (time.perf_counter() - t0) / 1e12, 5)
        t = t * 2 if t * 2 <= threads or t == threads else threads
    O.set_num_threads(threads)
    out["thread_scaling_2048_tflops"] = scaling
    # not measured: the value above scaled linearly from its thread count to every physical core of the host (an
    # upper bound for the port there; the sample above shows how far below linear it scales up to 16 threads)
    phys = _physical_cores()
    if phys:
        out["physical_cores_machine"] = phys
        out["all_physical_cores_linear_bound"] = {
            "value": round(out["value"] * phys / threads, 4), "unit": "TFLOP/s", "cores": phys,
            "basis": f"extrapolated, not measured: value x {phys} / {threads} threads"}
    # cfg1 in full: SGEMM emulation 1024^3, N = 4, fast mode (BASELINE.json configs[0])
    A1 = G.randmat(1024, 1024, torch.float32, 0.5, 123456, dev).cpu().numpy().T
    t0 = time.perf_counter()
    C1 = O.gemm(A1, A1, 4, True)
    dt1 = time.perf_counter() - t0
    r1 = A1.astype(np.float64) @ A1.astype(np.float64)
    rel1 = np.abs(C1.astype(np.float64) - r1) / np.abs(r1)
    cfg1 = {"workload": "cfg1: SGEMM emulation m=n=k=1024, num_moduli=4, fast mode (CPU, full size)",
            "seconds": round(dt1, 3), "tflops": 2.0 * 1024 ** 3 / dt1 / 1e12, "threads": threads,
            "relerr_max_vs_fp64": float(rel1.max()), "relerr_median_vs_fp64": float(np.median(rel1)),
            "sha256_C": hashlib.sha256(np.asfortranarray(C1).tobytes(order="F")).hexdigest()}
    fx = os.path.join(ROOT, "tests", "golden", "cfg1_ref.json")
    if os.path.exists(fx):
        ref1 = json.load(open(fx))
        cfg1["matches_reference_build"] = cfg1["sha256_C"] == ref1.get("sha256_C_reference")
    out["cfg1"] = cfg1
    return out


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


def make_operands(kind, m, n, k, seed_a, dev):
    """column-major operands ((cols, rows) tensors) of the workload kind"""
    import gemmul8 as G
    if kind == "z":
        return (G.randmat(m, k, torch.complex128, 0.5, seed_a, dev), G.randmat(k, n, torch.complex128, 0.5, 123456, dev),
                torch.complex128)
    tb = torch.float32 if kind == "dfd" else torch.float64
    return G.randmat(m, k, torch.float64, 0.5, seed_a, dev), G.randmat(k, n, tb, 0.5, 123456, dev), torch.float64


def time_variants(G, GD, A, B, m, n, k, N, fast, world, rank, args, ops, arm=lambda name: None, out=None):
    """SURVEY.md 8(e)'s partitions side by side, after the timed region, same operands (a few steps each):
    the default (modulus, column block) units with C gathered on the root; whole moduli per rank with the residue
    planes sent to the root and the root's CRT (variant (i)); row blocks of C, all moduli per rank, no exchange
    (variant (ii), strong scaling); its 2-D form (output blocks on a near-square rank grid); and the north star's
    reduce of FP64 partial CRT sums (gemm_moduli_reduce: two m x n double accumulators to the root; C within a
    few ulp, not bit-identical).  Each result goes into `out` as soon as it is measured, so a line printed after a
    later variant got stuck still carries it."""
    steps, warm = 3, 1
    out = {} if out is None else out
    flops = 2.0 * m * n * k

    stall = os.environ.get("GEMMUL8_BENCH_REHEARSE_STALL")  # rehearsal of the fail-soft path

    def timed(name, fn):
        arm(name)
        if stall == name and rank == world - 1:
            time.sleep(1e9)  # the last rank never arrives: the others' collectives of this variant wait on it
        try:
            for _ in range(warm):
                fn()
            barrier(world)
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            barrier(world)
        except Exception as e:  # a variant must not cost the main line (e.g. a collective the backend lacks)
            put(out, name, f"failed: {type(e).__name__}: {str(e)[:200]}")
            return
        v = reduce_max(time.perf_counter() - t0, world) / steps * 1e3
        put(out, name, {"ms_per_step": round(v, 3), "tflops": round(flops / (v * 1e-3) / 1e12, 1)})

    timed("moduli_columns",  # gemm_moduli over all W ranks, C distributed (the headline where the grid is not)
        lambda: GD.gemm_moduli(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, fast, torch.float64, ops=ops, order=args.order))
    timed("moduli_columns_gathered",
        lambda: GD.gemm_moduli(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, fast, torch.float64, gather=True, ops=ops))
    timed("moduli_whole_planes_to_root",
        lambda: GD.gemm_moduli_planes_to_root(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, fast, torch.float64, ops=ops))
    r0, r1 = GD.blocks(m, world)[rank]
    if r1 > r0:
        wr = G.alloc_work(r1 - r0, n, k, N, G.REAL_DEFAULT, A.device)
        Cr = torch.empty((n, r1 - r0), dtype=torch.float64, device=A.device)
        Ar = A[:, r0:]  # rows r0.. of the column-major A (lda = m)
        rows = lambda: G.gemm(G.OP_N, G.OP_N, r1 - r0, n, k, 1.0, Ar, m, B, k, 0.0, Cr, r1 - r0, N, fast, wr)
    else:
        rows = lambda: None
    timed("row_blocks_all_moduli", rows)
    if r1 > r0:
        del wr, Cr
    # 2-D output blocks, all moduli per rank (grid R x Q = W with R, Q closest to sqrt(W)): each rank reads and
    # encodes 1/R of A and 1/Q of B; fast-mode shifts need no exchange, so nothing crosses the fabric
    R = max(d for d in range(1, int(world ** 0.5) + 1) if world % d == 0)
    Q = world // R
    (a0, a1), (b0, b1) = GD.blocks(m, R)[rank // Q], GD.blocks(n, Q)[rank % Q]
    if fast and a1 > a0 and b1 > b0:
        wb = G.alloc_work(a1 - a0, b1 - b0, k, N, G.REAL_DEFAULT, A.device)
        Cb = torch.empty((b1 - b0, a1 - a0), dtype=torch.float64, device=A.device)
        Ab, Bb = A[:, a0:], B[b0:]
        blk = lambda: G.gemm(G.OP_N, G.OP_N, a1 - a0, b1 - b0, k, 1.0, Ab, m, Bb, k, 0.0, Cb, a1 - a0, N, fast, wb)
    else:
        blk = lambda: None
    timed(f"output_blocks_{R}x{Q}_all_moduli", blk)
    if fast and a1 > a0 and b1 > b0:
        del wb, Cb
    # the 2-D unit grid (gemm_moduli_grid): two row blocks of W / 2 ranks, each a (modulus, column block)
    # partition of its rows over its own sub-group -- each rank reads half of A and exchanges within its row block
    # (GEMMUL8_BENCH_NO_GRID=1, or sub-groups that could not be created at setup: not timed)
    if fast and world >= 4 and world % 2 == 0 and os.environ.get("GEMMUL8_BENCH_NO_GRID") is None:
        gops = GD.HipShardOps()
        timed(f"moduli_grid_2x{world // 2}",
              lambda: GD.gemm_moduli_grid(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, fast, torch.float64, row_blocks=2,
                                          ops=gops, order=args.order))
        GD.release_workspaces(gops)
        torch.cuda.empty_cache()
    # the north star's partition as built (gemm_moduli_reduce): whole moduli per rank, partial FP64 CRT sums,
    # one sum-reduce of the two m x n planes to the root, the root's finishing CRT (C within ulps, not bit-identical)
    timed("moduli_partial_sums_reduce",
        lambda: GD.gemm_moduli_reduce(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, fast, torch.float64, ops=ops))
    torch.cuda.empty_cache()
    return out


def select_workload(args, world):
    """the configuration this run measures: --workload, else cfg2 on one GPU and cfg3 (the moduli-sharded
    BASELINE config) on more; --size / --moduli / --accurate make it a custom one"""
    name = args.workload or ("cfg3" if (world > 1 and args.partition != "rows") else "cfg2")
    wl = WORKLOADS[name]
    m = args.size or wl["size"]
    N = args.moduli or wl["moduli"]
    fast = not (args.accurate or wl["accurate"])
    custom = m != wl["size"] or N != wl["moduli"] or fast == wl["accurate"]
    return {"name": name, "wl": wl, "m": m, "N": N, "fast": fast, "kind": wl["kind"], "custom": custom}


def source_sha16():
    """the first 16 hex digits of the sha256 of the host sources that decide a line (bench.py, gemmul8/dist.py,
    gemmul8/__init__.py): a committed line can be checked against the revision under test"""
    out = {}
    for rel in ("bench.py", "mixed-gemmul8_amd/gemmul8/dist.py", "mixed-gemmul8_amd/gemmul8/__init__.py"):
        try:
            with open(os.path.join(ROOT, rel), "rb") as f:
                out[os.path.basename(rel) if rel != "mixed-gemmul8_amd/gemmul8/__init__.py" else "gemmul8/__init__.py"] = \
                    hashlib.sha256(f.read()).hexdigest()[:16]
        except OSError:
            pass
    return out


def resolve_partition(args, world, fast):
    """the partition of a multi-GPU run: --partition, or for auto the 2-D unit grid (gemm_moduli_grid: 2 row blocks
    of W / 2 ranks, each a (modulus, column block) partition of its rows) where it applies -- fast mode, an even
    W >= 4, sub-groups created at setup -- else the (modulus, column block) units over all W ranks.  The grid is
    the headline because the cfg3 per-rank replay measured it faster by more than the run-to-run spread
    (profiles/r06/cfg3_partitions/: slowest rank 6.070 / 6.063 ms against 6.194 / 6.179 ms, one box)"""
    if world <= 1:
        return "single"
    if args.partition != "auto":
        return args.partition
    grid_ok = fast and world >= 4 and world % 2 == 0 and os.environ.get("GEMMUL8_BENCH_NO_GRID") is None
    return "grid" if grid_ok else "moduli"


def labels(W):
    """(config.workload, metric) of a run: BASELINE.json's metric string only for the cfg2 workload itself"""
    cplx, m, N, fast = W["kind"] == "z", W["m"], W["N"], W["fast"]
    if W["custom"]:
        workload = (f"{'complex ' if cplx else ''}{'mixed ' if W['kind'] == 'dfd' else ''}DGEMM emulation m=n=k={m}, "
                    f"num_moduli={N}, {'fast' if fast else 'accurate'} mode")
    else:
        workload = W["wl"]["text"]
    if W["name"] == "cfg2" and not W["custom"]:
        metric = BASELINE_METRIC
    else:
        metric = (f"emulated {'ZGEMM' if cplx else 'DGEMM'} TFLOP/s + max rel-error, m=n=k={m} num_moduli={N}" +
                  ("" if fast else " accurate") + (f" ({W['name']})" if not W["custom"] else ""))
    return workload, metric


def algorithmic_work(m, n, k, N, kind, fast, L):
    """SURVEY.md 8(d)'s algorithmic work of one call: int8 ops of the products this build runs (2 m n k per
    plane; complex: 4 m n k big matrix, 3 m n k Karatsuba; accurate mode: one bound plane more) and the fused-
    minimum HBM bytes per phase -- operands read once, slices written once and read once by the products,
    residues written once and read once by the CRT, C written once (beta = 0).  Slice and residue bytes are
    the padded planes of this build's layout (gemmul8.layout)."""
    cplx = kind == "z"
    eA, eB, eC = {"d": (8, 8, 8), "dfd": (8, 4, 8), "z": (16, 16, 16)}[kind]
    fmac = (3.0 if L["nsub"] == 3 else 4.0) if cplx else 1.0
    planes = N + (0 if fast else 1)
    ops = 2.0 * fmac * m * n * k * planes
    slices = N * (L["planeA"] + L["planeB"])
    resid = N * L["planeR"]
    split = m * k * eA + k * n * eB + slices + (0 if fast else L["planeA"] + L["planeB"])
    prod = slices + resid + (0 if fast else L["planeA"] + L["planeB"])
    crt = resid + m * n * eC
    return {"int8_ops": ops, "bytes": {"split": split, "products": prod, "crt": crt,
                                       "total": split + prod + crt}}


def composite_roofline(work, ms_per_step, phase_ms=None, world=1):
    """(int8_ops / P_int8 + bytes_alg / B_hbm) / t_step (world > 1: over W GPUs' peaks),
    plus each memory-bound phase's algorithmic GB/s from its measured time"""
    t = ms_per_step * 1e-3
    t_mfma = work["int8_ops"] / (INT8_PEAK_TOPS * 1e12 * world)
    t_hbm = work["bytes"]["total"] / (HBM_PEAK_GBS * 1e9 * world)
    out = {"int8_ops": work["int8_ops"], "bytes_alg": work["bytes"]["total"],
           "t_mfma_bound_ms": round(t_mfma * 1e3, 4), "t_hbm_bound_ms": round(t_hbm * 1e3, 4),
           "frac": round((t_mfma + t_hbm) / t, 4),
           "formula": "(int8_ops/P_int8 + bytes_alg/B_hbm)/t_step" + (f" with P, B x {world} GPUs" if world > 1 else "")}
    if phase_ms:
        gbs = {}
        for name, key in (("split", "scaling"), ("crt", "inverse_scaling")):
            if phase_ms.get(key, 0) > 0:
                gbs[name] = {"bytes_alg": work["bytes"][name], "ms": phase_ms[key],
                             "GBps": round(work["bytes"][name] / (phase_ms[key] * 1e-3) / 1e9, 1),
                             "frac_of_hbm_peak": round(work["bytes"][name] / (phase_ms[key] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        out["phases"] = gbs
    return out


def main():
    args = parse()
    maybe_launch(args)
    world, rank, backend = dist_setup()
    import gemmul8 as G
    from gemmul8 import dist as GD

    wd = None
    if world > 1:
        # fail fast: a phase that outlives its limit ends this rank with the stage and peers it was at
        wd = GD.StageWatchdog(float(os.environ.get("GEMMUL8_DIST_WATCHDOG_S", "240")), rank)
    arm = (lambda ph, on_fire=None: wd.arm(ph, on_fire)) if wd else (lambda ph, on_fire=None: None)

    W = select_workload(args, world)
    wl_name, wl, m, N, fast, kind, custom = W["name"], W["wl"], W["m"], W["N"], W["fast"], W["kind"], W["custom"]
    n = k = m
    cplx = kind == "z"
    ct = G.COMPLEX_BIG_MATRIX_ENCODE if cplx else G.REAL_DEFAULT
    flop_per = (8.0 if cplx else 2.0) * m * n * k
    dev = torch.device("cuda", torch.cuda.current_device())
    part = resolve_partition(args, world, fast)
    sharded = part in ("moduli", "grid")
    grid = part == "grid"
    rows_accurate = world > 1 and not sharded and not fast
    seed = 123456 + (rank if (world > 1 and not sharded) else 0)
    arm("setup")
    A, B, tc = make_operands(kind, m, n, k, seed, dev)
    L = G.layout(m, n, k, N, ct)
    trace = None
    # the rows [r0, r1) of C this rank's units cover and its index in the plan (grid: its row block's sub-plan)
    r0, r1, prank = 0, m, rank
    if grid:
        Gs = world // 2
        hblk, prank = divmod(rank, Gs)
        r0, r1 = GD.blocks(m, 2)[hblk]
    if sharded:
        ops = GD.HipShardOps()
        plan = GD.ShardPlan(r1 - r0, n, N, world // 2 if grid else world, order=args.order)
        trace = []

        if grid:
            def step(tr=None):
                return GD.gemm_moduli_grid(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, fast, tc, ct, row_blocks=2,
                                           gather=args.gather, ops=ops, order=args.order, trace=tr)
        else:
            def step(tr=None):
                return GD.gemm_moduli(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, fast, tc, ct, gather=args.gather,
                                      ops=ops, trace=tr, order=args.order)
    elif rows_accurate:
        # accurate row blocks: B's column shifts come from the bound product over ALL rows of A, so the ranks
        # MAX-combine its column maxima (gemmul8.dist.matmul_rows); row-major operands: op T on both
        Arm, Brm = A.t().contiguous(), B.t().contiguous()
        row_ops = GD.HipOps()

        def step(tr=None):
            return GD.matmul_rows(Arm, Brm, N, False, tc, ops=row_ops)
    else:
        C = torch.empty((n, m), dtype=tc, device=dev)
        work = G.alloc_work(m, n, k, N, ct, dev)

        def step(tr=None):
            G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, work, ct)
            return C

    arm("warmup")
    for _ in range(args.warmup):
        step()
    G.timing_enable(True)
    G.timing_read()  # reset
    barrier(world)
    arm("timed steps")
    # the K steps are timed with HIP events on the stream, recorded inside the barrier +
    # synchronize bracket: the GPU timeline of the steps, idle time between calls included.  The host wall time of
    # the bracket is reported beside it (ms_per_step_wall); it also holds the host's return from the closing
    # synchronize (profiles/r04/final4: wall steps 0.01-0.5 ms above the summed kernel phases; tools/probes/gap_probe.py,
    # in git history at ae0caaa)
    e_start, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e_start.record()
    for _ in range(args.steps):
        step(trace)
    e_end.record()
    barrier(world)
    wall = time.perf_counter() - t0
    G.timing_enable(False)
    phase_ms, _ = G.timing_read()
    dt = reduce_max(e_start.elapsed_time(e_end) * 1e-3, world)
    wall = reduce_max(wall, world)
    ms_per_step = dt / args.steps * 1e3
    # strong scaling (one product over all ranks) or weak (row partition: one product per rank)
    value = flop_per * (1 if (sharded or world == 1) else world) * args.steps / dt / 1e12

    avg = [x / args.steps for x in phase_ms]
    extra = {}
    # int8 MACs per output element and modulus relative to m n k: 1 real, 4 complex big matrix, 3 Karatsuba
    fmac = (3.0 if L["nsub"] == 3 else 4.0) if cplx else 1.0
    work_alg = algorithmic_work(m, n, k, N, kind, fast, L)
    if sharded:
        # dominant kernel: the int8 products of rank 0's units (one products_cols launch per merged unit)
        ops_step = sum(2.0 * (r1 - r0) * (c1 - c0) * k * fmac * (j1 - j0) for j0, j1, c0, c1 in plan.launches[prank])
        planes = sum((c1 - c0) * (j1 - j0) for j0, j1, c0, c1 in plan.launches[prank]) / n
        seg = {}
        for i in range(0, len(trace), 6):
            evs = trace[i:i + 6]
            for (a, ea), (b, eb) in zip(evs, evs[1:]):
                seg[b] = seg.get(b, 0.0) + ea.elapsed_time(eb)
        extra["step_phases_ms_rank0"] = {kk: round(v / args.steps, 4) for kk, v in seg.items()}
        extra["launches_rank0"] = [list(u) for u in plan.launches[prank]]
    else:
        ops_step = 2.0 * fmac * m * n * k * N
        planes = N
    gemm_ms = avg[1]
    achieved = ops_step / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
    roofline = {"bound": "mfma", "achieved": round(achieved, 1), "peak": round(INT8_PEAK_TOPS, 1), "unit": "TFLOP/s",
                "frac": round(achieved / INT8_PEAK_TOPS, 4),
                "traffic": traffic_from_profile((m, n, k, planes, fast)) if not cplx else None,
                "kernel": G.last_products_kernel() + " (residue products; int8 ops counted as FLOP, "
                          "2*m'*n'*k' per plane and launch" + (", rank 0's units)" if sharded else ")"),
                "avg_launch_ms": round(gemm_ms, 4)}
    if sharded:
        # every unit of the plan runs exactly once: all ranks' int8 ops over W GPUs' peak and the step time
        # (accurate mode: the bound product is split by column blocks too)
        roofline["aggregate"] = {"int8_ops_all_ranks": work_alg["int8_ops"],
                                 "frac": round(work_alg["int8_ops"] / (world * INT8_PEAK_TOPS * 1e12 * ms_per_step * 1e-3), 4),
                                 "formula": "sum over ranks of int8 ops / (W * P_int8 * t_step)"}

    if not sharded and not rows_accurate:
        extra["phase_ms"] = {"scaling": round(avg[0], 4), "int8_products": round(avg[1], 4),
                             "inverse_scaling": round(avg[3], 4)}
        roofline["composite"] = composite_roofline(work_alg, ms_per_step, extra["phase_ms"])
    elif sharded:
        roofline["composite"] = composite_roofline(work_alg, ms_per_step, None, world)
    report = {"cpu": None}

    def line(incomplete=None):
        """rank 0's JSON line from what has been measured so far"""
        workload, metric = labels(W)
        out = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "ms_per_step_wall": round(wall / args.steps * 1e3, 4),
            "timing": "HIP events on the stream over the K steps, max over ranks (ms_per_step_wall: host clock of the "
                      "barrier + synchronize bracket)",
            "higher_is_better": True,
            "scaling": "strong" if sharded else ("weak" if world > 1 else "single"),
            "vs_baseline": round(value / world / GH200_PUBLISHED_TFLOPS, 3) if (wl_name == "cfg2" and not custom) else None,
            "vs_baseline_ref": "GH200 published OS2-fast-14 8192 (72.13 TFLOP/s, BASELINE.md); per-GPU ratio",
            "dtype": "i8",
            "io_dtype": {"d": "f64", "dfd": "f64*f32->f64", "z": "c128"}[kind],
            "data": "synthetic: hiprand XORWOW (U-0.5)*exp(0.5*N(0,1)), seed 123456, A == B as in the reference "
                    "driver" + (" (row partition: rank r's A seed 123456+r)" if (world > 1 and not sharded) else ""),
            "config": {"workload": workload, "m": m, "n": n, "k": k, "num_moduli": N, "fastmode": fast,
                       "parallelism": ((f"row blocks 2 x (moduli x column blocks) x{world // 2}" if grid else
                                        "moduli x column blocks" if sharded else "rows") + f" x{world}")
                       if world > 1 else "single",
                       "partition": part,
                       "world_size": world, "backend": backend or "none",
                       "output": ("C gathered on rank 0" if args.gather else "C distributed by column blocks")
                       if sharded else "C on each rank"},
            "roofline": roofline,
            "cpu_baseline": report["cpu"],
            "source_sha16": source_sha16(),
        }

        if sharded:
            out["config"]["unit_order"] = args.order
            out["config"]["dist_side_stream"] = GD.side_stream_enabled() and backend == "nccl"
            out["config"]["dist_timeout_s"] = float(os.environ.get("GEMMUL8_DIST_TIMEOUT", "300"))
        out.update(dict(extra))
        if incomplete:
            # a phase after the timed region outlived the watchdog: the timed steps above stand, the fields
            # that phase and the later ones would have added are missing
            out["incomplete"] = incomplete
        return out

    # the phases after the timed region are optional: if one of them gets stuck (a collective of a variant
    # whose peer failed, say), rank 0 prints the line measured so far and every rank exits with status 0
    if rank == 0:
        def soft(msg):
            with STATE_LOCK:
                text = json.dumps(line(msg))
            print(text, flush=True)
    else:
        def soft(msg):
            pass

    # accuracy against a double-double reference (testing/eval.hpp semantics); sharded: each rank checks
    # its own output columns, the max is combined
    if not args.no_accuracy and not cplx and kind == "d":
        arm("accuracy", soft)
        Cout = step()
        torch.cuda.synchronize()
        if sharded:
            c0, c1 = plan.cols[prank]
            if args.gather:
                Cout = None if rank else Cout[c0:c1, r0:r1]
            if c1 > c0 and r1 > r0 and Cout is not None:
                Ab = A if not grid else A[:, r0:r1].contiguous()  # (the rows of this rank's row block)
                C1, C2 = G.dd_gemm(Ab, B[c0:c1], r1 - r0, c1 - c0, k)
                emax, emed = G.relerr_dd(Cout, C1, C2)
                del C1, C2
            else:
                emax, emed = 0.0, 0.0
            emax = reduce_max(emax, world)
            put(extra, "relerr_max", emax)
            put(extra, "relerr_median_rank0_columns", emed)
        elif world == 1 or rank == 0:
            C1, C2 = G.dd_gemm(A, B, m, n, k)
            emax, emed = G.relerr_dd(Cout, C1, C2)
            put(extra, "relerr_max", emax)
            put(extra, "relerr_median", emed)
            del C1, C2
            if world == 1:
                # a second, independent seed pair (A 123456, B 654321) beside the reference's A == B
                B2 = G.randmat(k, n, torch.float64, 0.5, 654321, dev)
                C2o = torch.empty((n, m), dtype=tc, device=dev)
                G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B2, k, 0.0, C2o, m, N, fast, work, ct)
                C1, C2 = G.dd_gemm(A, B2, m, n, k)
                emax2, emed2 = G.relerr_dd(C2o, C1, C2)
                put(extra, "relerr_seed_pair_123456_654321", {"max": emax2, "median": emed2})
                del C1, C2, B2, C2o

    if sharded and not args.no_single_gpu:
        # the same call on ONE GPU (rank 0, after the timed region; the other ranks wait at the barrier): the
        # strong-scaling efficiency of this line is single_gpu_ms / (W * ms_per_step)
        arm("single-GPU baseline", soft)
        GD.release_workspaces(ops)
        torch.cuda.empty_cache()
        if rank == 0:
            C1g = torch.empty((n, m), dtype=tc, device=dev)
            w1 = G.alloc_work(m, n, k, N, ct, dev)
            one = lambda: G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C1g, m, N, fast, w1, ct)
            one()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 3
            e0.record()
            for _ in range(reps):
                one()
            e1.record()
            torch.cuda.synchronize()
            single_ms = e0.elapsed_time(e1) / reps
            put(extra, "single_gpu_ms", round(single_ms, 4))
            put(extra, "single_gpu_tflops", round(flop_per / (single_ms * 1e-3) / 1e12, 2))
            put(extra, "strong_scaling_efficiency", round(single_ms / (world * ms_per_step), 4))
            del w1, C1g
            torch.cuda.empty_cache()
        barrier(world)

    if sharded and kind == "d" and not args.no_variants:
        # last of the collective phases: each variant is a phase of its own for the watchdog
        put(extra, "variants", {})
        time_variants(G, GD, A, B, m, n, k, N, fast, world, rank, args, ops,
                      arm=lambda name: arm(f"variants: {name}", soft), out=extra["variants"])

    if rank == 0:
        arm("report", soft)
        # measured live after the timed region: the same MFMA alone on uniformly random operand bytes
        # (the residue distribution) in registers -- the clock the chip holds under that load bounds
        # any int8 GEMM on such data
        ceiling = G.mfma_ceiling()
        if ceiling > 0:
            put(roofline, "data_bound_ceiling", round(ceiling, 1))
            put(roofline, "frac_of_data_bound_ceiling", round(achieved / ceiling, 4))
        if world == 1 and not args.no_power:
            # the box's power state on this step, after the timed region: the SMU averages over longer than the
            # K timed steps, so the same step runs back to back for about a second while amdsmi is sampled every
            # 5 ms (the first 30 % of the window dropped while the clock settles); the power-capped clock differs
            # from device to device, and this is what a line from a slow box shows
            try:
                sp = StepPower()
                sp.begin()
                t_p, calls = time.perf_counter(), 0
                while time.perf_counter() - t_p < 1.0:
                    for _ in range(4):
                        step()
                    calls += 4
                    torch.cuda.synchronize()
                put(extra, "power_steady_state", sp.end(calls, settle=0.3))
            except Exception as e:  # (fail-soft: the line goes without the field)
                print(f"bench: no power sample: {type(e).__name__}: {str(e)[:120]}", file=sys.stderr, flush=True)
        if not args.no_dgemm and kind == "d" and (world == 1 or sharded):
            # the vendor DGEMM of the same shape on ONE GPU (rocBLAS through torch)
            Ar, Br = A.t(), B.t()
            for _ in range(2):
                torch.matmul(Ar, Br)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            reps = 5 if m <= 8192 else 2
            for _ in range(reps):
                torch.matmul(Ar, Br)
            torch.cuda.synchronize()
            dg = 2.0 * m * n * k * reps / (time.perf_counter() - t1) / 1e12
            put(extra, "rocblas_dgemm_tflops_1gpu", round(dg, 2))
            put(extra, "vs_rocblas_dgemm_1gpu", round(value / dg, 3))
        if world == 1 and wl_name == "cfg2" and not custom and not args.no_cfg3_1gpu:
            # the multi-GPU lines measure cfg3 (16384^3): its one-GPU time here, so that a 1 -> N curve assembled
            # from N = 1 (cfg2) and N > 1 (cfg3) lines can also be read against the same workload
            n3 = WORKLOADS["cfg3"]["size"]
            A3 = G.randmat(n3, n3, torch.float64, 0.5, 123456, dev)
            C3 = torch.empty((n3, n3), dtype=torch.float64, device=dev)
            w3 = G.alloc_work(n3, n3, n3, 14, G.REAL_DEFAULT, dev)
            one3 = lambda: G.gemm(G.OP_N, G.OP_N, n3, n3, n3, 1.0, A3, n3, A3, n3, 0.0, C3, n3, 14, True, w3)
            one3()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                one3()
            e1.record()
            torch.cuda.synchronize()
            ms3 = e0.elapsed_time(e1) / 3
            put(extra, "cfg3_workload_1gpu", {"workload": WORKLOADS["cfg3"]["text"].split(",")[0] + " on ONE GPU",
                                              "ms_per_step": round(ms3, 3),
                                              "tflops": round(2.0 * n3 ** 3 / (ms3 * 1e-3) / 1e12, 2)})
            del A3, C3, w3
            torch.cuda.empty_cache()
        gpu_C = C if (world == 1 and kind == "d" and fast and N == 14) else None
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args.cpu_sample, dev, gpu_C, args.cpu_threads)
        put(report, "cpu", cpu)
        if wd:
            # no fire between here and the print: a fire already in progress ends the process inside disarm()
            # (the watchdog holds its lock while it reports), so exactly one line is printed either way
            wd.disarm()
        with STATE_LOCK:
            text = json.dumps(line())
        print(text, flush=True)
    if world > 1:
        import torch.distributed as dist
        arm("teardown", lambda msg: None)  # the line is out (rank 0) or not this rank's to print
        try:
            dist.barrier()
            GD.release_grid_groups()
            dist.destroy_process_group()
        except Exception as e:  # a peer that left after a stuck optional phase: the line stands
            print(f"bench: teardown: {type(e).__name__}: {str(e)[:200]}", file=sys.stderr, flush=True)
    if wd:
        wd.disarm()
        wd.close()


if __name__ == "__main__":
    main()
