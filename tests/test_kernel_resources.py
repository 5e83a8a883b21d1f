"""Register / LDS budgets of the hot gfx950 kernels, read from the built library's code-object metadata
(tools/kernel_resources.py; no GPU needed).  A source change elsewhere in a kernel can push it across an
occupancy step without any visible sign: in round 3 the reference-epilogue code took the Karatsuba CRT from
164 to 172 VGPRs, 3 -> 2 waves per SIMD, and cfg5's CRT from 0.202 to 0.231 ms.  The floors below are the
occupancies the measured timings in DESIGN.md were taken at."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(not shutil.which("llvm-readelf", path="/opt/rocm/llvm/bin"),
                                reason="ROCm LLVM tools absent")

# demangled-name prefix -> minimum waves per SIMD
FLOORS = {
    "oz2::gemm_i8_persistent_pg_kernel<false, 1, 0>": 2,  # cfg2/3/4 products: 512 threads, 160 KiB LDS, 1 block per CU
    "oz2::gemm_i8_persistent_pg_kernel<true, 1, 0>": 2,   # cfg5 (Karatsuba sub-products)
    "oz2::gemm_i8_persistent_kernel<false, 1, 0, 0>": 2,  # the block-epilogue form (GEMMUL8_PG_EPILOGUE=0)
    "oz2::gemm_i8_small_kernel<0, false>": 2,       # small launches: 256 threads, 64 KiB LDS, 2 blocks per CU
    "oz2::gemm_i8_small_kernel<1, false>": 2,       # the accurate-mode bound product of small problems
    "oz2::crt_kernel<0, false, 14u, false, 4, false>": 5,    # cfg2/3 CRT (4 rows per lane, the default)
    "oz2::crt_kernel<0, false, 14u, false, 8, false>": 5,    # GEMMUL8_CRT_ROWS=8
    "oz2::crt_kernel<0, false, 14u, false, 8, true>": 4,     # ... with 4 columns per block and prefetch
    "oz2::crt_kernel<0, false, 10u, false, 8, false>": 5,    # cfg4 CRT
    "oz2::crt_kernel<2, false, 12u, true, 8, false>": 3,     # cfg5 CRT (Karatsuba residues)
    "oz2::stats_pair_kernel<16, true>": 8,             # cfg2 shifts
    "oz2::encode_pair_kernel<double, false, false, true, true, false>": 4,  # cfg2 slices
    "oz2::split_fused_kernel<1024, 4, 256, false, true, false, false, 1>": 4,  # small problems: shifts and slices at once
    "oz2::encode_kernel<double, true, false, false, 0, true>": 2,    # cfg5 slices
}


@pytest.fixture(scope="module")
def table():
    import kernel_resources as K
    lib = K.LIB
    assert os.path.exists(lib), "build first: make -C mixed-gemmul8_amd"
    res = K.resources(lib)
    dm = K.demangled(sorted(res))
    return {dm[n]: v for n, v in res.items()}


def test_occupancy_formula():
    """waves per SIMD: 512 registers per lane in granules of 8, 160 KiB of LDS per CU over 4 SIMDs, at most 8"""
    import kernel_resources as K
    assert K.occupancy(81, 0, 16384, 256) == 5      # the real CRT: 88 registers -> 5
    assert K.occupancy(156, 0, 32768, 256) == 3     # the Karatsuba CRT
    assert K.occupancy(172, 0, 32768, 256) == 2     # ... as it had drifted
    assert K.occupancy(238, 0, 163840, 512) == 2    # the product kernel: one 512-thread block per CU
    assert K.occupancy(62, 0, 19328, 256) == 8      # the stats pair kernel
    assert K.occupancy(260, 4, 16640, 128) == 1     # 264 registers: one wave
    assert K.occupancy(102, 0, 16640, 128) == 4     # 128-thread blocks: LDS allows 9 blocks = 18 waves / 4


def test_no_kernel_uses_scratch(table):
    bad = {n: v["scratch"] for n, v in table.items() if v["scratch"] or v["vgpr_spill"]}
    assert not bad, bad


@pytest.mark.parametrize("prefix", sorted(FLOORS))
def test_hot_kernel_occupancy(table, prefix):
    hits = {n: v for n, v in table.items() if n.startswith("void " + prefix + "(")}
    assert hits, f"{prefix} not in the library"
    for n, v in hits.items():
        assert v["occupancy"] >= FLOORS[prefix], (n, v)


@pytest.mark.parametrize("prefix,loads,stores,load_op", [
    ("oz2::gemm_i8_persistent_pg_kernel<false, 1, 0>(", 0, 8, "dwordx2"),  # residue stores (LDS-DMA loads: buffer ops)
    ("oz2::gemm_i8_persistent_pg_kernel<true, 1, 0>(", 0, 8, "dwordx2"),
    ("oz2::gemm_i8_persistent_kernel<false, 1, 0, 0>(", 0, 8, "dwordx2"),
    ("oz2::crt_kernel<0, false, 14u, false, 4, false>(", 14, 2, "dword"),  # 14 residue planes (4 rows: one dword
                                                                            # each), C stored in 16-byte vectors
    ("oz2::crt_kernel<0, false, 14u, false, 8, false>(", 14, 4, "dwordx2"),
    ("oz2::crt_kernel<2, false, 12u, true, 8, false>(", 36, 8, "dwordx2"),  # 3 Karatsuba sub-planes x 12 moduli
])
def test_streaming_memory_ops(prefix, loads, stores, load_op):
    """the streams read or written once per call stay out of the caches (non-temporal), and the
    CRT's residue loads are global, not flat (a flat load also counts in lgkmcnt, so scalar and LDS waits would
    wait for the residues in flight)"""
    import re
    import kernel_resources as K
    (body,) = K.disassembly(prefix)
    ops = [ln.split("//")[0] for ln in body.splitlines() if re.search(r"\s(global|flat)_(load|store)", ln)]
    assert not [o for o in ops if "flat_load_dwordx2" in o], "residue loads through flat addresses"
    assert sum(o.split()[0] == "global_load_" + load_op and o.rstrip().endswith(" nt") for o in ops) == loads
    assert sum("global_store_dwordx4" in o and o.rstrip().endswith(" nt") for o in ops) == stores
