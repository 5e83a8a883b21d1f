"""GPU: the reference's C++ API (include/gemmul8.hpp: workSize + gemm<TA,TB,TC> with a hipBLAS
handle) used from C++ exactly as code written for the reference would use it (tests/cpp/api_check.cpp,
compiled here with hipcc and linked against libgemmul8_amd.so): bit-identical to the C ABI, the
handle's stream honoured, invalid compute types rejected with {0,0,0,0}, and a call captured into a
HIP graph on the handle's stream replays bit-identically."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "mixed-gemmul8_amd", "gemmul8")


def test_cpp_api_drop_in(tmp_path):
    exe = str(tmp_path / "api_check")
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++20", "-O1", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "api_check.cpp"), "-L" + LIBDIR, "-lgemmul8_amd", "-lhipblas",
           "-Wl,-rpath," + LIBDIR, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def test_cpp_api_async_switch(tmp_path):
    """GEMMUL8_TIMERS=0: gemmul8::gemm returns {0,0,0,0} while its kernels are still queued (hipStreamQuery right
    after two back-to-back 4096^3 calls reports not ready); without it the call returns after its own completion
    with phase times.  Both runs bit-identical to the C ABI."""
    exe = str(tmp_path / "api_check")
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++20", "-O1", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "api_check.cpp"), "-L" + LIBDIR, "-lgemmul8_amd", "-lhipblas",
           "-Wl,-rpath," + LIBDIR, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ)
    env["GEMMUL8_TIMERS"] = "0"
    r = subprocess.run([exe, "async"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "async OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
    env.pop("GEMMUL8_TIMERS")
    r = subprocess.run([exe, "sync"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "sync OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
