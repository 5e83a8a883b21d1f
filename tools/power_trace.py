#!/usr/bin/env python3
"""power_trace.py -- board power, clocks and memory-controller activity of the cfg2 loop.

Runs, back to back on one GPU, each for about --seconds:
  idle        nothing (the baseline draw)
  gemm        the bench step: gemmul8 gemm at cfg2 (8192^3, N = 14, fast mode), calls back to back
  products    the product kernel alone (gemmul8.products on a workspace the split filled once)
  mfma        the int8 MFMA alone on random operand bytes in registers (gemmul8.mfma_ceiling)
  hbm_read    torch.sum over a 4 GiB float64 tensor (every byte from HBM: beyond the 256 MiB Infinity Cache)
  mall_read   torch.sum over a 128 MiB tensor (beyond the 32 MiB of L2, inside the Infinity Cache)
while a sampler thread reads the SMU's gpu_metrics table (amdsmi) every --period ms: socket power, the
eight XCDs' gfx clocks, UMC (HBM controller) activity, the energy accumulator and the throttle
residency counters (PPT = package power tracking, thermal).  Per phase it reports mean power, mean
clock, the energy per call from the accumulator, and the throttle residencies' growth.

The two read loops calibrate UMC activity against known HBM bytes: the product kernel's HBM bytes per
launch are estimated as (its UMC activity / hbm_read's) x hbm_read's byte rate x the launch time,
beside its memory-side (L2 miss) bytes from the PMC passes.  Writes go to --out (summary.json,
samples.csv).  Usage: python3 tools/power_trace.py --out gpurun_out/power [--seconds 2.5]
"""
import argparse
import csv
import json
import os
import statistics
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))

FIELDS = ["current_socket_power", "average_socket_power", "average_gfxclk_frequency", "current_uclk",
          "average_umc_activity", "average_gfx_activity", "energy_accumulator", "throttle_status",
          "indep_throttle_status", "ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc",
          "hbm_thm_residency_acc", "prochot_residency_acc", "accumulation_counter", "mem_activity_acc",
          "gfx_activity_acc", "temperature_hotspot", "temperature_mem", "voltage_gfx"]


def _num(x):
    try:
        return float(x)
    except (TypeError, ValueError):
        return None


class Sampler(threading.Thread):
    def __init__(self, smi, dev, period):
        super().__init__(daemon=True)
        self.smi, self.dev, self.period = smi, dev, period
        self.rows, self.stop_ev, self.phase = [], threading.Event(), "start"
        self.errors = 0

    def run(self):
        while not self.stop_ev.is_set():
            t = time.perf_counter()
            try:
                m = self.smi.amdsmi_get_gpu_metrics_info(self.dev)
            except Exception:
                self.errors += 1
                time.sleep(self.period)
                continue
            row = {"t": t, "phase": self.phase}
            for f in FIELDS:
                row[f] = _num(m.get(f))
            clks = m.get("current_gfxclks")
            if isinstance(clks, list):
                for i, c in enumerate(clks[:8]):
                    row[f"gfxclk{i}"] = _num(c)
            self.rows.append(row)
            dt = self.period - (time.perf_counter() - t)
            if dt > 0:
                time.sleep(dt)


def find_device(smi):
    """the amdsmi handle of torch's cuda:0 (by PCI bus id; the box may list every GPU of the host)"""
    p = torch.cuda.get_device_properties(0)
    handles = smi.amdsmi_get_processor_handles()
    for h in handles:
        try:
            bdf = smi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
            dom, bus = int(bdf.split(":")[0], 16), int(bdf.split(":")[1], 16)
            if bus == p.pci_bus_id and dom == p.pci_domain_id:
                return h, bdf
        except Exception:
            continue
    return handles[0], "unmatched (first handle)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/power")
    ap.add_argument("--seconds", type=float, default=2.5)
    ap.add_argument("--period", type=float, default=0.01)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--moduli", type=int, default=14)
    ap.add_argument("--cfg", type=int, default=2, choices=[2, 4, 5],
                    help="workload of the gemm / products loops: 2 (default), 4 (d x s -> d, N = 10, accurate) or 5 "
                         "(complex 4096^3, N = 12, Karatsuba products)")
    ap.add_argument("--no-calibration", action="store_true", help="skip the mfma / hbm_read / mall_read loops")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)

    import amdsmi as smi
    import gemmul8 as G
    smi.amdsmi_init()
    torch.cuda.set_device(0)
    dev, bdf = find_device(smi)
    info = {"bdf": bdf}
    for name, fn in (("power_cap", smi.amdsmi_get_power_cap_info), ("energy_count", smi.amdsmi_get_energy_count)):
        try:
            info[name] = fn(dev)
        except Exception as e:
            info[name] = f"unavailable: {e}"
    res = info["energy_count"].get("counter_resolution") if isinstance(info["energy_count"], dict) else None
    uj_per_count = float(res) if res else 15.259  # microjoules per accumulator count

    d = torch.device("cuda", 0)
    ta, tb, ct, fast = torch.float64, torch.float64, G.REAL_DEFAULT, True
    m = n = k = args.size
    N = args.moduli
    if args.cfg == 4:
        tb, N, fast = torch.float32, 10, False
    elif args.cfg == 5:
        ta = tb = torch.complex128
        ct, N, m = G.COMPLEX_BIG_MATRIX_ENCODE, 12, 4096
        n = k = m
    A = G.randmat(m, k, ta, 0.5, 123456, d)
    B = A if tb == ta else G.randmat(k, n, tb, 0.5, 123456, d)
    C = torch.empty((n, m), dtype=ta, device=d)
    work = G.alloc_work(m, n, k, N, ct, d)
    gemm = lambda: G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, work, ct)
    prods = lambda: G.products(m, n, k, N, work, computeType=ct)
    L = G.layout(m, n, k, N, ct)
    fmac = (3.0 if L["nsub"] == 3 else 4.0) if args.cfg == 5 else 1.0
    big = torch.ones(512 * 1024 * 1024 if not args.no_calibration else 1, dtype=torch.float64, device=d)  # 4 GiB
    mall = torch.ones(16 * 1024 * 1024 if not args.no_calibration else 1, dtype=torch.float64, device=d)  # 128 MiB
    for f in (gemm, prods, lambda: big.sum(), lambda: mall.sum()):
        f()
    torch.cuda.synchronize()

    sampler = Sampler(smi, dev, args.period)
    sampler.start()
    phases = {}

    def run(name, fn, per_call=None):
        """fn back to back for about --seconds (per_call: (int8 ops, bytes) per call)"""
        torch.cuda.synchronize()
        sampler.phase = name
        t0 = time.perf_counter()
        calls = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        while time.perf_counter() - t0 < args.seconds:
            for _ in range(8):
                fn()
            calls += 8
            torch.cuda.synchronize()  # bounds the host's run-ahead
        e1.record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        phases[name] = {"t0": t0, "t1": t1, "calls": calls, "gpu_ms": e0.elapsed_time(e1),
                        "ms_per_call": e0.elapsed_time(e1) / max(calls, 1), "per_call": per_call}
        sampler.phase = "gap"
        time.sleep(0.3)

    ops = 2.0 * fmac * m * n * k * N
    sampler.phase = "idle"
    t0 = time.perf_counter()
    time.sleep(args.seconds)
    phases["idle"] = {"t0": t0, "t1": time.perf_counter(), "calls": 0}
    run("gemm", gemm, {"int8_ops": ops + (0 if fast else 2.0 * fmac * m * n * k),
                       "emulated_flop": (8.0 if args.cfg == 5 else 2.0) * m * n * k})
    run("products", prods, {"int8_ops": ops})
    if not args.no_calibration:
        iters = 100000
        # ops per call: 2 forms x (iters / 4 + 1 + iters) iterations x 64 MFMAs x 2 * 32^3 ops x 2 * CUs * 4 waves
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        mops = 2 * (iters // 4 + 1 + iters) * 64 * 2.0 * 32 ** 3 * 2 * cus * 4
        run("mfma", lambda: G.mfma_ceiling(iters), {"int8_ops": mops, "note": "two launches of each MFMA form per call"})
        run("hbm_read", lambda: big.sum(), {"bytes": big.numel() * 8})
        run("mall_read", lambda: mall.sum(), {"bytes": mall.numel() * 8})
    sampler.stop_ev.set()
    sampler.join()

    rows = sampler.rows
    with open(os.path.join(args.out, "samples.csv"), "w", newline="") as f:
        keys = sorted({kk for r in rows for kk in r}, key=lambda s: (s != "t", s != "phase", s))
        w = csv.DictWriter(f, fieldnames=keys)
        w.writeheader()
        for r in rows:
            w.writerow(r)

    summary = {"device": info, "workload": f"cfg{args.cfg}: m={m} n={n} k={k} N={N} {'fast' if fast else 'accurate'}",
               "period_s": args.period, "samples": len(rows), "sampler_errors": sampler.errors,
               "uj_per_energy_count": uj_per_count, "phases": {}}
    for name, ph in phases.items():
        # samples strictly inside the phase (skip the first 20 %: clocks settle after a load change)
        span = ph["t1"] - ph["t0"]
        inside = [r for r in rows if ph["t0"] + 0.2 * span <= r["t"] <= ph["t1"]]
        out = {"seconds": round(span, 3), "calls": ph["calls"], "samples": len(inside)}
        if ph.get("gpu_ms"):
            out["ms_per_call"] = round(ph["ms_per_call"], 4)
        for f_ in ["current_socket_power", "average_gfxclk_frequency", "average_umc_activity", "average_gfx_activity",
                   "temperature_hotspot", "voltage_gfx", "current_uclk"] + [f"gfxclk{i}" for i in range(8)]:
            vals = [r[f_] for r in inside if r.get(f_) is not None]
            if vals:
                out[f_ + "_mean"] = round(statistics.fmean(vals), 2)
                out[f_ + "_min"] = round(min(vals), 2)
                out[f_ + "_max"] = round(max(vals), 2)
        clk = [statistics.fmean([r[f"gfxclk{i}"] for i in range(8) if r.get(f"gfxclk{i}") is not None])
               for r in inside if r.get("gfxclk0") is not None]
        if clk:
            out["gfxclk_8xcd_mean_MHz"] = round(statistics.fmean(clk), 1)
        # accumulators over the whole phase window (first and last sample inside [t0, t1])
        win = [r for r in rows if ph["t0"] <= r["t"] <= ph["t1"]]
        if len(win) >= 2:
            a, b = win[0], win[-1]
            dt = b["t"] - a["t"]
            for acc in ("energy_accumulator", "ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc",
                        "hbm_thm_residency_acc", "prochot_residency_acc", "accumulation_counter", "mem_activity_acc",
                        "gfx_activity_acc"):
                if a.get(acc) is not None and b.get(acc) is not None:
                    out[acc + "_delta"] = b[acc] - a[acc]
            if out.get("energy_accumulator_delta") is not None and dt > 0:
                joules = out["energy_accumulator_delta"] * uj_per_count * 1e-6
                out["energy_J"] = round(joules, 3)
                out["power_from_energy_W"] = round(joules / dt, 1)
                if ph["calls"] and ph.get("gpu_ms"):
                    # energy per call over the window the accumulator covered
                    calls_in = ph["calls"] * dt / span
                    out["energy_per_call_J"] = round(joules / calls_in, 5)
                    pc = ph.get("per_call") or {}
                    if pc.get("int8_ops"):
                        out["pJ_per_int8_op"] = round(joules / calls_in / pc["int8_ops"] * 1e12, 4)
            if out.get("ppt_residency_acc_delta") is not None and out.get("accumulation_counter_delta"):
                out["ppt_residency_frac"] = round(out["ppt_residency_acc_delta"] / out["accumulation_counter_delta"], 4)
        pc = ph.get("per_call") or {}
        if pc.get("int8_ops") and ph.get("ms_per_call"):
            out["TOPS"] = round(pc["int8_ops"] / (ph["ms_per_call"] * 1e-3) / 1e12, 1)
        if pc.get("bytes") and ph.get("ms_per_call"):
            out["read_GBps"] = round(pc["bytes"] / (ph["ms_per_call"] * 1e-3) / 1e9, 1)
        summary["phases"][name] = out
    # UMC-activity calibration: bytes/s per % of UMC activity on the HBM-bound read
    P = summary["phases"]
    h, mr, pr = P.get("hbm_read", {}), P.get("mall_read", {}), P.get("products", {})
    if h.get("average_umc_activity_mean") and h.get("read_GBps"):
        gbps_per_pct = h["read_GBps"] / h["average_umc_activity_mean"]
        est = {"GBps_per_umc_pct (hbm_read)": round(gbps_per_pct, 2),
               "mall_read_umc_pct": mr.get("average_umc_activity_mean")}
        if pr.get("average_umc_activity_mean") is not None and pr.get("ms_per_call"):
            rate = pr["average_umc_activity_mean"] * gbps_per_pct
            est["products_hbm_GBps_est"] = round(rate, 1)
            est["products_hbm_GB_per_launch_est"] = round(rate * pr["ms_per_call"] * 1e-3, 3)
        summary["umc_calibration"] = est
    with open(os.path.join(args.out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1, default=str)
    print(json.dumps(summary, default=str))
    smi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
