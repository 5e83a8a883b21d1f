#!/usr/bin/env python3
"""Register, LDS and scratch use of every gfx950 kernel in the built library, and the occupancy that follows.

Reads the HIP fat binary of mixed-gemmul8_amd/gemmul8/libgemmul8_amd.so (or an object file): each translation
unit's clang offload bundle holds one gfx950 code object, whose AMDGPU metadata note lists every kernel's
.vgpr_count / .agpr_count / .sgpr_count / .group_segment_fixed_size / .private_segment_fixed_size.  Occupancy
(waves per SIMD) = min(8, VGPR limit, LDS limit): 512 unified registers per lane per SIMD in granules of 8, and
160 KiB of LDS per CU shared by the blocks resident on its 4 SIMDs.

A code change can move a kernel across an occupancy step without changing its source (round 3: the Karatsuba
CRT went from 3 to 2 waves per SIMD, +18 % time); tests/test_kernel_resources.py pins the hot kernels.

    python tools/kernel_resources.py [library or object] [name filter]"""
import os
import shutil
import struct
import subprocess
import sys
import tempfile

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mixed-gemmul8_amd", "gemmul8", "libgemmul8_amd.so")
LLVM = "/opt/rocm/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
LDS_PER_CU = 160 * 1024


def _section(path, name=".hip_fatbin"):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sec.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f"{name}={out}", path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        return open(out, "rb").read()


def _code_objects(blob, target="gfx950"):
    """the gfx950 code objects of every offload bundle in the section"""
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(target):
                yield blob[pos + off:pos + off + size]
        pos = blob.find(MAGIC, pos + 32)


def _kernels(code_object):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code_object)
        f.flush()
        txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], check=True,
                             capture_output=True, text=True).stdout
    doc = txt[txt.index("---") + 3:]
    doc = doc[:doc.index("\n...")] if "\n..." in doc else doc
    meta = yaml.safe_load(doc)
    return meta["amdhsa.kernels"]


def occupancy(vgpr, agpr, lds, wg):
    """waves per SIMD on gfx950"""
    regs = vgpr if not agpr else -(-vgpr // 4) * 4 + agpr
    regs = max(8, -(-regs // 8) * 8)
    by_regs = 512 // regs
    waves_per_block = -(-wg // 64)
    by_lds = 8 if lds == 0 else (LDS_PER_CU // lds) * waves_per_block // 4
    return max(0, min(8, by_regs, by_lds))


def resources(path=LIB):
    out = {}
    for co in _code_objects(_section(path)):
        for k in _kernels(co):
            vg, ag = k.get(".vgpr_count", 0), k.get(".agpr_count", 0)
            lds, wg = k.get(".group_segment_fixed_size", 0), k.get(".max_flat_workgroup_size", 256)
            out[k[".name"]] = {"vgpr": vg, "agpr": ag, "sgpr": k.get(".sgpr_count", 0), "lds": lds,
                               "scratch": k.get(".private_segment_fixed_size", 0),
                               "vgpr_spill": k.get(".vgpr_spill_count", 0), "wg": wg,
                               "occupancy": occupancy(vg, ag, lds, wg)}
    return out


def demangled(names):
    tool = shutil.which("llvm-cxxfilt", path="/opt/rocm/lib/llvm/bin:" + LLVM) or shutil.which("c++filt")
    if tool is None:
        return {n: n for n in names}
    r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True)
    return dict(zip(names, r.stdout.splitlines())) if r.returncode == 0 else {n: n for n in names}


def disassembly(prefix, path=LIB):
    """gfx950 instructions of the kernel(s) whose demangled name starts with `prefix` (one string per kernel)"""
    out = []
    for co in _code_objects(_section(path)):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", "--demangle", f.name],
                                 check=True, capture_output=True, text=True).stdout
        for block in txt.split("\n\n"):
            head = block.lstrip("\n").split("\n", 1)[0]  # "<address> <void name(args)>:"
            if head.endswith(">:") and (("<" + prefix) in head or ("<void " + prefix) in head):
                out.append(block)
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else LIB
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    res = resources(path)
    dm = demangled(sorted(res))
    print(f"{'kernel':90s} {'vgpr':>4s} {'agpr':>4s} {'lds':>6s} {'scr':>4s} {'occ':>3s}")
    for n in sorted(res, key=lambda x: dm[x]):
        if flt in dm[n]:
            r = res[n]
            print(f"{dm[n][:90]:90s} {r['vgpr']:4d} {r['agpr']:4d} {r['lds']:6d} {r['scratch']:4d} {r['occupancy']:3d}")


if __name__ == "__main__":
    main()
