// crt.hip -- CRT recombination ("inverse scaling") for gfx950.
//
// Per output element: C = sum_i w_i * r_i (double, or the hi/lo double-double
// pair for numM = 2), q = -rint(C / M), t = C + q*M, scaled by 2^(sftA+sftB),
// then the BLAS epilogue.  Operation order restates
// GEMMul8/src/inverse_scaling.hpp:35-62 (numM = 1) and :138-172 (numM = 2), so
// the result is bit-identical to the reference for the same residues.
// Each thread reads one 4-byte word from every residue plane (4 consecutive rows
// of one column, coalesced across the wave) and writes 4 consecutive outputs;
// the weights arrive as kernel arguments (the reference uploads them to
// __constant__ on every call, gemmul8.cu:236-241).
#include "oz2_split.hpp"

namespace oz2 {

struct CrtArgs {
    const uint8_t *R;
    size_t planeR, ldr;
    size_t m, n;
    size_t imag_off;  // complex: rows of the imaginary part (= m), else 0
    const int16_t *sftA, *sftB;
    void *C;
    size_t ldc;
    double ar, ai, br, bi;
    CrtParams cp;
};

template <bool NUMM1>
__device__ __forceinline__ double crt_value(const CrtParams &cp, const uint32_t *w, int e) {
    const unsigned N = cp.N;
    // loops are unrolled to OZ2_MAX_MODULI with a uniform guard so w[] stays in VGPRs
    if (NUMM1) {
        double C = 0.0;
#pragma unroll
        for (unsigned i = 0; i < OZ2_MAX_MODULI; ++i)
            if (i < N) C = __builtin_fma(cp.w_hi[i], (double)((w[i] >> (8 * e)) & 0xffu), C);
        const double quot = -__builtin_rint(C * cp.invM);
        return __builtin_fma(quot, cp.M1, C);
    } else {
        double C1 = 0.0, C2 = 0.0;
#pragma unroll
        for (unsigned i = 0; i < OZ2_MAX_MODULI; ++i) {
            if (i >= N) break;
            const double r = (double)((w[i] >> (8 * e)) & 0xffu);
            C1 = __builtin_fma(cp.w_hi[i], r, C1);
            C2 = __builtin_fma(cp.w_lo[i], r, C2);
        }
        const double quot = -__builtin_rint(__builtin_fma(C1, cp.invM, C2 * cp.invM));
        const double t1 = __builtin_fma(quot, cp.M1, C1) + C2;
        return __builtin_fma(quot, cp.M2, t1);
    }
}

__device__ __forceinline__ void load_words(const CrtArgs &a, size_t off, bool aligned, size_t rows_left, uint32_t *w) {
    const unsigned N = a.cp.N;
    if (aligned && rows_left >= 4) {
#pragma unroll
        for (unsigned i = 0; i < OZ2_MAX_MODULI; ++i)
            w[i] = i < N ? *reinterpret_cast<const uint32_t *>(a.R + i * a.planeR + off) : 0u;
    } else {
#pragma unroll
        for (unsigned i = 0; i < OZ2_MAX_MODULI; ++i) {
            if (i >= N) { w[i] = 0; continue; }
            uint32_t x = 0;
            for (int e = 0; e < 4; ++e)
                if ((size_t)e < rows_left) x |= (uint32_t)a.R[i * a.planeR + off + e] << (8 * e);
            w[i] = x;
        }
    }
}

// BLAS epilogue; the reference's alpha==1/beta==1 special cases are kept
// (inverse_scaling.hpp:823-948), its non-BLAS variants (:417, :682, :736, :763) are not.
__device__ __forceinline__ double epi_d(double v, double c, double al, double be) {
    if (be == 0.0) return al == 1.0 ? v : al * v;  // C is not read (BLAS)
    if (al == 1.0) {
        if (be == 1.0) return c + v;
        return __builtin_fma(be, c, v);
    }
    if (be == 1.0) return __builtin_fma(al, v, c);
    return __builtin_fma(be, c, al * v);
}
__device__ __forceinline__ float epi_f(float v, float c, float al, float be) {
    if (be == 0.0f) return al == 1.0f ? v : al * v;
    if (al == 1.0f) {
        if (be == 1.0f) return c + v;
        return __builtin_fmaf(be, c, v);
    }
    if (be == 1.0f) return __builtin_fmaf(al, v, c);
    return __builtin_fmaf(be, c, al * v);
}

template <int OT, bool NUMM1>
__global__ __launch_bounds__(256) void crt_kernel(CrtArgs a) {
    const size_t r0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (r0 >= a.m) return;
    const size_t rows_left = a.m - r0;
    const int nr = rows_left >= 4 ? 4 : (int)rows_left;
    for (size_t col = blockIdx.y; col < a.n; col += gridDim.y) {
        uint32_t w[OZ2_MAX_MODULI], wi[OZ2_MAX_MODULI];
        const size_t off = col * a.ldr + r0;
        load_words(a, off, true, rows_left, w);
        if (OT >= 2) load_words(a, off + a.imag_off, (a.imag_off & 3) == 0, rows_left, wi);
        const int sB = a.sftB[col];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (e < nr) {
            const size_t row = r0 + e;
            const int sft = (int)a.sftA[row] + sB;
            const double vr = scalbn(crt_value<NUMM1>(a.cp, w, e), sft);
            const size_t o = col * a.ldc + row;
            if (OT == 0) {
                double *C = static_cast<double *>(a.C);
                C[o] = epi_d(vr, a.br == 0.0 ? 0.0 : C[o], a.ar, a.br);
            } else if (OT == 1) {
                float *C = static_cast<float *>(a.C);
                const float al = (float)a.ar, be = (float)a.br;
                C[o] = epi_f(__double2float_rn(vr), be == 0.0f ? 0.0f : C[o], al, be);
            } else {
                const double vi = scalbn(crt_value<NUMM1>(a.cp, wi, e), sft);
                const bool plain = a.ar == 1.0 && a.ai == 0.0 && a.br == 0.0 && a.bi == 0.0;
                const bool zb = a.br == 0.0 && a.bi == 0.0;
                if (OT == 2) {
                    double2 *C = static_cast<double2 *>(a.C);
                    if (plain) {
                        C[o] = make_double2(vr, vi);
                    } else {
                        const double2 c = zb ? make_double2(0.0, 0.0) : C[o];
                        const double tr = __builtin_fma(a.ar, vr, -a.ai * vi), ti = __builtin_fma(a.ar, vi, a.ai * vr);
                        C[o] = make_double2(__builtin_fma(a.br, c.x, __builtin_fma(-a.bi, c.y, tr)),
                                            __builtin_fma(a.br, c.y, __builtin_fma(a.bi, c.x, ti)));
                    }
                } else {
                    float2 *C = static_cast<float2 *>(a.C);
                    const float fr = __double2float_rn(vr), fi = __double2float_rn(vi);
                    if (plain) {
                        C[o] = make_float2(fr, fi);
                    } else {
                        const float2 c = zb ? make_float2(0.0f, 0.0f) : C[o];
                        const float arf = (float)a.ar, aif = (float)a.ai, brf = (float)a.br, bif = (float)a.bi;
                        const float tr = __builtin_fmaf(arf, fr, -aif * fi), ti = __builtin_fmaf(arf, fi, aif * fr);
                        C[o] = make_float2(__builtin_fmaf(brf, c.x, __builtin_fmaf(-bif, c.y, tr)),
                                           __builtin_fmaf(brf, c.y, __builtin_fmaf(bif, c.x, ti)));
                    }
                }
            }
            }
        }
    }
}

void crt_inverse(const uint8_t *R, const Layout &L, const int16_t *sftA, const int16_t *sftB, const CrtParams &CP,
                 OutType ot, const void *alpha, const void *beta, void *C, size_t ldc, hipStream_t st) {
    CrtArgs a{};
    a.R = R;
    a.planeR = L.planeR;
    a.ldr = L.m_pad;
    a.m = L.m;
    a.n = L.n;
    a.imag_off = L.cplx ? L.m : 0;
    a.sftA = sftA;
    a.sftB = sftB;
    a.C = C;
    a.ldc = ldc;
    switch (ot) {
    case OutType::F64: a.ar = *(const double *)alpha; a.br = *(const double *)beta; break;
    case OutType::F32: a.ar = *(const float *)alpha; a.br = *(const float *)beta; break;
    case OutType::C64:
        a.ar = ((const double *)alpha)[0]; a.ai = ((const double *)alpha)[1];
        a.br = ((const double *)beta)[0]; a.bi = ((const double *)beta)[1];
        break;
    default:
        a.ar = ((const float *)alpha)[0]; a.ai = ((const float *)alpha)[1];
        a.br = ((const float *)beta)[0]; a.bi = ((const float *)beta)[1];
        break;
    }
    a.cp = CP;
    const unsigned gx = (unsigned)((L.m + 1023) / 1024);
    const unsigned gy = (unsigned)(L.n < 65535 ? L.n : 65535);
    dim3 grid(gx, gy);
#define OZ2_CRT(ot_, nm) crt_kernel<ot_, nm><<<grid, dim3(256), 0, st>>>(a)
    const bool nm1 = CP.numM1 != 0;
    switch (ot) {
    case OutType::F64: if (nm1) OZ2_CRT(0, true); else OZ2_CRT(0, false); break;
    case OutType::F32: OZ2_CRT(1, true); break;
    case OutType::C64: if (nm1) OZ2_CRT(2, true); else OZ2_CRT(2, false); break;
    default: OZ2_CRT(3, true); break;
    }
#undef OZ2_CRT
}

}  // namespace oz2
