"""Test helpers: tiled-layout decode, reference input generation, comparisons."""
import numpy as np


def untile(plane_bytes, vpad, kpad):
    """Decode one int8 slice plane of the MFMA panel layout into a (vpad, kpad) matrix
    (layout documented in mixed-gemmul8_amd/csrc/oz2_common.hpp)."""
    a = np.frombuffer(plane_bytes, dtype=np.int8)
    a = a.reshape(vpad // 256, kpad // 64, 2, 8, 2, 32, 16)  # vt, ks, s, blk, h, r, b
    a = a.transpose(0, 3, 5, 1, 2, 4, 6)  # vt, blk, r, ks, s, h, b
    return a.reshape(vpad, kpad)


def tile(mat, vpad, kpad):
    """Inverse of untile: (vpad, kpad) int8 -> plane bytes."""
    a = np.asarray(mat, dtype=np.int8).reshape(vpad // 256, 8, 32, kpad // 64, 2, 2, 16)
    a = a.transpose(0, 3, 4, 1, 5, 2, 6)
    return np.ascontiguousarray(a).reshape(-1)


def randmat_np(rng, m, n, phi=0.5, dtype=np.float64):
    """(U(0,1] - 0.5) * exp(phi * N(0,1)) as in testing/make_matrix.hpp:8-21 (numpy stream)."""
    if np.issubdtype(dtype, np.complexfloating):
        rd = np.float64 if dtype == np.complex128 else np.float32
        re = randmat_np(rng, m, n, phi, rd)
        im = randmat_np(rng, m, n, phi, rd)
        return np.asfortranarray((re + 1j * im).astype(dtype))
    u = 1.0 - rng.random((m, n))
    x = (u - 0.5) * np.exp(rng.standard_normal((m, n)).astype(dtype) * dtype(phi))
    return np.asfortranarray(x.astype(dtype))


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()
