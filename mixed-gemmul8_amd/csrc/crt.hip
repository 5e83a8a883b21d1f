// crt.hip -- CRT recombination ("inverse scaling") for gfx950.
//
// Per output element: C = sum_i w_i * r_i (double, or the hi/lo double-double
// pair for numM = 2), q = -rint(C / M), t = C + q*M, scaled by 2^(sftA+sftB),
// then the BLAS epilogue.  Operation order restates
// GEMMul8/src/inverse_scaling.hpp:35-62 (numM = 1) and :138-172 (numM = 2), so
// the result is bit-identical to the reference for the same residues.
//
// HBM-bound streaming kernel: each thread owns 8 consecutive rows of one column,
// reads one 8-byte word from each of the N residue planes (coalesced across the
// wave: 512 B per plane per wave instruction) and writes 8 outputs.  N is a
// template parameter (19 instantiations) so every plane load is unguarded and
// the accumulation fully unrolled; the weights are compile-time constants of the
// instantiation (the reference uploads them to __constant__ on every call,
// gemmul8.cu:236-241).  Complex outputs read the real and imaginary residues from rows r and
// r + m of the big-matrix planes, or combine them from the three Karatsuba sub-planes (KARA).
#include <utility>

#include "oz2_split.hpp"

namespace oz2 {

constexpr int CRT_ROWS = 8;

struct CrtArgs {
    const uint8_t *R;
    size_t planeR, ldr;
    size_t m, n;
    size_t imag_off;  // complex big matrix: rows of the imaginary part (= m), else 0
    size_t sub;       // Karatsuba complex: stride of the sub-planes P1, P2, P3 within a plane
    const int16_t *sftA, *sftB;
    void *C;
    size_t ldc;
    double ar, ai, br, bi;
    int ref_epi;  // 1: the reference's epilogue kernels including their non-BLAS variants (gemmul8_set_epilogue)
};

// CRT value of one element (inverse_scaling.hpp:35-62 numM = 1, :138-172 numM = 2) with the weights
// and M as compile-time constants of (N, NUMM1), the table make_crt_params reads: passed as kernel
// arguments the 2N weights overflowed the SGPRs and were parked in VGPR lanes.  Each of C1 and C2
// accumulates i = 0..N-1 in order, as the reference does.
template <unsigned N, bool NUMM1, unsigned I> __device__ __forceinline__ constexpr double w_hi() {
    if constexpr (NUMM1) return oz2_NMi_1[N - 2][I];
    else if constexpr (N >= 8) return oz2_NMi_2[N - 8][I][0];
    else return 0.0;
}
template <unsigned N, unsigned I> __device__ __forceinline__ constexpr double w_lo() {
    if constexpr (N >= 8) return oz2_NMi_2[N - 8][I][1];
    else return 0.0;
}
template <unsigned N, bool NUMM1, unsigned... I>
__device__ __forceinline__ double crt_value_const(const uint8_t (&r)[N], std::integer_sequence<unsigned, I...>) {
    constexpr double invM = oz2_invM[N - 2], M1 = oz2_M_hi[N - 2], M2 = oz2_M_lo[N - 2];
    if constexpr (NUMM1) {
        double C = 0.0;
        ((C = __builtin_fma(w_hi<N, true, I>(), (double)r[I], C)), ...);
        const double quot = -__builtin_rint(C * invM);
        return __builtin_fma(quot, M1, C);
    } else {
        double C1 = 0.0, C2 = 0.0;
        ((C1 = __builtin_fma(w_hi<N, false, I>(), (double)r[I], C1)), ...);
        ((C2 = __builtin_fma(w_lo<N, I>(), (double)r[I], C2)), ...);
        const double quot = -__builtin_rint(__builtin_fma(C1, invM, C2 * invM));
        const double t1 = __builtin_fma(quot, M1, C1) + C2;
        return __builtin_fma(quot, M2, t1);
    }
}

// The same values for the CRT_ROWS rows of a lane at once, moduli outermost: each weight pair is used for the
// lane's rows right after it is materialised, so only one pair is live (per row the fma chains run i ascending,
// as in crt_value_const: the same bits).  With the rows innermost the compiler kept all 2N weights live across
// the row loop and parked most of them in VGPR lanes.
// An f64 constant materialised in an SGPR pair where it is used: the two moves are volatile, so they are
// not hoisted out of the column loop (hoisted, the 2N weights overflow the SGPRs and are spilled to VGPR lanes)
template <uint64_t BITS> __device__ __forceinline__ double sconst() {
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)BITS));
    asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(BITS >> 32)));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <unsigned N, bool NUMM1, int R, typename W, unsigned... I>
__device__ __forceinline__ void crt_rows_const(const W (&w)[N], double (&out)[R], std::integer_sequence<unsigned, I...>) {
    constexpr double invM = oz2_invM[N - 2], M1 = oz2_M_hi[N - 2], M2 = oz2_M_lo[N - 2];
    double C1[R] = {}, C2[R] = {};
    auto step = [&](auto ic) {
        constexpr unsigned i = decltype(ic)::value;
        const W x = w[i];
        const double hi = sconst<__builtin_bit_cast(uint64_t, w_hi<N, NUMM1, i>())>();
        const double lo = NUMM1 ? 0.0 : sconst<__builtin_bit_cast(uint64_t, w_lo<N, i>())>();
#pragma unroll
        for (int e = 0; e < R; ++e) {
            const double r = (double)(uint8_t)(x >> (8 * e));
            C1[e] = __builtin_fma(hi, r, C1[e]);
            if constexpr (!NUMM1) C2[e] = __builtin_fma(lo, r, C2[e]);
        }
    };
    (step(std::integral_constant<unsigned, I>{}), ...);
#pragma unroll
    for (int e = 0; e < R; ++e) {
        if constexpr (NUMM1) {
            const double quot = -__builtin_rint(C1[e] * invM);
            out[e] = __builtin_fma(quot, M1, C1[e]);
        } else {
            const double quot = -__builtin_rint(__builtin_fma(C1[e], invM, C2[e] * invM));
            const double t1 = __builtin_fma(quot, M1, C1[e]) + C2[e];
            out[e] = __builtin_fma(quot, M2, t1);
        }
    }
}
#ifndef OZ2_CRT_MODOUTER
#define OZ2_CRT_MODOUTER 1  // A/B builds: 0 = the per-row chains (crt_value_const) in the Karatsuba CRT
#endif
#ifndef OZ2_CRT_MODOUTER_ALL
#define OZ2_CRT_MODOUTER_ALL 0  // A/B builds: 1 = the same order in the real and big-matrix complex CRT (the
                                // real CRT is bound by HBM: same time; N = 10 then needs 135 VGPRs)
#endif
#ifndef OZ2_CRT_MODOUTER_MIN_N
#define OZ2_CRT_MODOUTER_MIN_N 15  // ... and from this N on regardless: with the rows innermost the real CRT parks
                                   // 244-820 weight words in VGPR lanes at N = 16-20 (90 at N = 14)
#endif
#ifndef OZ2_KARA_ROWS
#define OZ2_KARA_ROWS 8  // rows per lane of the Karatsuba CRT (A/B builds: 4 -- 127 VGPRs and 4 waves per SIMD
                         // instead of 155 and 3, the same time: profiles/r04/j/lib_ab.txt)
#endif
// residue word of R consecutive rows of one plane (one byte per row)
template <int R> using RowWord = std::conditional_t<R == 8, uint64_t, uint32_t>;

#ifndef OZ2_CRT_NT
// 1 = non-temporal residue loads, 2 = non-temporal C stores, 3 = both (default): the residues are read once and C is
// not re-read by the next call, so neither needs the caches; the dirty C lines otherwise leave the caches during the
// next call.  Same bits; tools/probes/lib_ab.py, 4 interleaved rounds, profiles/r05/nt_store_ab/: whole call cfg2
// -0.2 %, cfg5 -0.6 %, 8192^2 x 1024 -1.1 % against 0 (the CRT phase alone: loads -2.5 %, stores +2-3 %)
#define OZ2_CRT_NT 3
#endif
// residues of rows [off, off+8) of every plane; the fast path is one 8-byte load per plane
template <unsigned N, typename W = uint64_t>
__device__ __forceinline__ void load_rows(const CrtArgs &a, size_t off, bool fast, int nr, W (&w)[N]) {
    if (fast) {
        // one per-lane pointer stepped plane by plane (N scalar plane bases would spill the SGPRs); a global
        // (address space 1) pointer, so the opaque step keeps global_load: a generic one made the compiler emit flat
        // loads, which also count in lgkmcnt, so every scalar or LDS wait waited for the residues in flight too
        typedef const __attribute__((address_space(1))) uint8_t *GP;
        typedef const __attribute__((address_space(1))) W *GW;
        GP q = (GP)(a.R + off);
#pragma unroll
        for (unsigned i = 0; i < N; ++i) {
            if (OZ2_CRT_NT & 1) w[i] = __builtin_nontemporal_load((GW)q);
            else w[i] = *(GW)q;
            q += a.planeR;
            asm volatile("" : "+v"(q));
        }
    } else {
#pragma unroll
        for (unsigned i = 0; i < N; ++i) {
            W x = 0;
            for (int e = 0; e < nr; ++e) x |= (W)a.R[i * a.planeR + off + e] << (8 * e);
            w[i] = x;
        }
    }
}

// BLAS epilogue; the reference's alpha==1/beta==1 special cases are kept
// (inverse_scaling.hpp:823-948).  Its non-BLAS variants only with ref (the reference-epilogue mode):
// _1b / _2_1b compute beta*AB + C (:417, :682), _2_a1 alpha*C + AB (:736, :763; two-level moduli only,
// numM2), and _ab reads C at beta = 0 (fma(0, C, alpha*AB): NaN / Inf in C propagate, :522, :791).
__device__ __forceinline__ double epi_d(double v, double c, double al, double be, bool ref, bool numM1) {
    if (be == 0.0 && !(ref && al != 1.0)) return al == 1.0 ? v : al * v;  // C is not read (BLAS)
    if (al == 1.0) {
        if (be == 1.0) return c + v;
        return ref ? __builtin_fma(be, v, c) : __builtin_fma(be, c, v);
    }
    if (be == 1.0) return (ref && !numM1) ? __builtin_fma(al, c, v) : __builtin_fma(al, v, c);
    return __builtin_fma(be, c, al * v);
}
__device__ __forceinline__ float epi_f(float v, float c, float al, float be, bool ref) {
    if (be == 0.0f && !(ref && al != 1.0f)) return al == 1.0f ? v : al * v;
    if (al == 1.0f) {
        if (be == 1.0f) return c + v;
        return ref ? __builtin_fmaf(be, v, c) : __builtin_fmaf(be, c, v);
    }
    if (be == 1.0f) return __builtin_fmaf(al, v, c);
    return __builtin_fmaf(be, c, al * v);
}

// intra-wave LDS handoff (the whole wave takes part; no block-level barrier is needed)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int OT> struct OutElem;
template <> struct OutElem<0> { using T = double; };
template <> struct OutElem<1> { using T = float; };
template <> struct OutElem<2> { using T = double2; };
template <> struct OutElem<3> { using T = float2; };

// f<NUMM1>: the complex forms depend on the reference kernel's moduli level (below)
template <int OT> struct BlasEpi;
template <> struct BlasEpi<0> {
    template <bool NUMM1>
    static __device__ __forceinline__ double f(double v, double c, const CrtArgs &a) {
        return epi_d(v, c, a.ar, a.br, a.ref_epi != 0, NUMM1);
    }
};
template <> struct BlasEpi<1> {
    template <bool NUMM1>
    static __device__ __forceinline__ float f(float v, float c, const CrtArgs &a) {
        return epi_f(v, c, (float)a.ar, (float)a.br, a.ref_epi != 0);
    }
};
// Complex outputs: the reference's kernels operation for operation (inverse_scaling.hpp:268-948), with
// hip_complex.h's hipCmul / hipCfma as clang contracts them in its build (pinned on the reference's own
// full-precision outputs, tools/probes/epi_dump2.py, and pinned by tests/golden/ref_golden_epilogue.npz):
//   alpha = 1, beta = 0: v (_10);  alpha = beta = 1: C + v per component (CAdd, _11);
//   beta = 1: hipCfma(alpha, v, C) (_a1);  otherwise hipCfma(beta, C, hipCmul(alpha, v)) (_ab).
// Two departures, both BLAS semantics: beta = 0 does not read C (the reference's _ab does),
// and alpha = 1 with another beta is hipCfma(beta, C, v) (the reference's _1b computes beta*AB + C, 10.3).
// ref (the reference-epilogue mode) takes the reference's kernels there too, and its _2_a1 form
// hipCfma(alpha, C, v) for beta = 1 at two moduli levels (NUMM2).
template <typename R, typename R2, bool IM_PXQY> struct CplxEpi {
    static __device__ __forceinline__ R fma_(R a, R b, R c) {
        if constexpr (sizeof(R) == 8) return __builtin_fma(a, b, c);
        else return __builtin_fmaf(a, b, c);
    }
    static __device__ __forceinline__ R2 mk(R x, R y) { return R2{x, y}; }
    static __device__ __forceinline__ R2 cmul(R pr, R pi, R qr, R qi) {  // hipCmul(p, q)
        // which product of the imaginary part clang fused differs between the reference's kernels
        if constexpr (IM_PXQY) return mk(fma_(pr, qr, -(pi * qi)), fma_(pr, qi, pi * qr));
        else return mk(fma_(pr, qr, -(pi * qi)), fma_(pi, qr, pr * qi));
    }
    static __device__ __forceinline__ R2 cfma(R pr, R pi, R qr, R qi, R rr, R ri) {  // hipCfma(p, q, r)
        R re = fma_(pr, qr, rr), im = fma_(qr, pi, ri);
        return mk(fma_(-pi, qi, re), fma_(pr, qi, im));
    }
    static __device__ __forceinline__ R2 f(R2 v, R2 c, R ar, R ai, R br, R bi, bool ref, bool numM1) {
        const bool a1 = ar == R(1) && ai == R(0);
        if (br == R(0) && bi == R(0) && !(ref && !a1)) return a1 ? v : cmul(ar, ai, v.x, v.y);
        if (br == R(1) && bi == R(0)) {
            if (a1) return mk(c.x + v.x, c.y + v.y);
            return (ref && !numM1) ? cfma(ar, ai, c.x, c.y, v.x, v.y) : cfma(ar, ai, v.x, v.y, c.x, c.y);
        }
        if (a1 && ref) return cfma(br, bi, v.x, v.y, c.x, c.y);  // _1b: beta * AB + C
        const R2 x = a1 ? v : cmul(ar, ai, v.x, v.y);
        return cfma(br, bi, c.x, c.y, x.x, x.y);
    }
};
// hipCmul's imaginary part: p.x*q.y fused in the two-level (numM = 2) complex-double kernels
// (inverse_scaling_2_*_bigmatrix), p.y*q.x in the one-level ones and in every complex-float kernel
template <> struct BlasEpi<2> {
    template <bool NUMM1>
    static __device__ __forceinline__ double2 f(double2 v, double2 c, const CrtArgs &a) {
        return CplxEpi<double, double2, !NUMM1>::f(v, c, a.ar, a.ai, a.br, a.bi, a.ref_epi != 0, NUMM1);
    }
};
template <> struct BlasEpi<3> {
    template <bool NUMM1>
    static __device__ __forceinline__ float2 f(float2 v, float2 c, const CrtArgs &a) {
        return CplxEpi<float, float2, false>::f(v, c, (float)a.ar, (float)a.ai, (float)a.br, (float)a.bi,
                                                a.ref_epi != 0, true);
    }
};

// Karatsuba complex: the residues of Re = P1 - P2 and Im = P3 - P1 - P2 modulo p, for 8 bytes at once.
// Bytes go to 16-bit lanes (even / odd bytes of each dword); in a lane d = b1 - b2 wraps mod 2^16 when
// negative, so (d, d + p) holds exactly one value below p, the residue; likewise (q, q + p, q + 2p) for
// q = b3 - b1 - b2 in (-2p, p).  Packed u16 add / sub / min (v_pk_*_u16): about 6 ops per byte pair.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
template <int P>
__device__ __forceinline__ void kara_dword(uint32_t x1, uint32_t x2, uint32_t x3, uint32_t &re, uint32_t &im) {
    const u16x2 p1 = {(unsigned short)P, (unsigned short)P}, p2 = {(unsigned short)(2 * P), (unsigned short)(2 * P)};
    auto lanes = [&](uint32_t a1, uint32_t a2, uint32_t a3, uint32_t &r, uint32_t &t) {
        const u16x2 e1 = __builtin_bit_cast(u16x2, a1), e2 = __builtin_bit_cast(u16x2, a2), e3 = __builtin_bit_cast(u16x2, a3);
        const u16x2 d = e1 - e2;
        r = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(d, d + p1));
        const u16x2 q = e3 - (e1 + e2);
        t = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_elementwise_min(q, q + p1), q + p2));
    };
    constexpr uint32_t LO = 0x00ff00ffu;
    uint32_t rE, tE, rO, tO;
    lanes(x1 & LO, x2 & LO, x3 & LO, rE, tE);
    lanes((x1 >> 8) & LO, (x2 >> 8) & LO, (x3 >> 8) & LO, rO, tO);
    re = rE | (rO << 8);
    im = tE | (tO << 8);
}
// The same residues in two steps, so that only two sub-planes' words are live at a time: from P1 and P2,
// Re = (b1 - b2) mod p and S = (b1 + b2) mod p (b1 + b2 < 2p, so (e, e - p) holds exactly one value below p);
// later Im = (b3 - S) mod p, which equals (b3 - b1 - b2) mod p.
template <int P>
__device__ __forceinline__ void kara_pair_dword(uint32_t x1, uint32_t x2, uint32_t &re, uint32_t &sum) {
    const u16x2 p1 = {(unsigned short)P, (unsigned short)P};
    auto lanes = [&](uint32_t a1, uint32_t a2, uint32_t &r, uint32_t &t) {
        const u16x2 e1 = __builtin_bit_cast(u16x2, a1), e2 = __builtin_bit_cast(u16x2, a2);
        const u16x2 d = e1 - e2, e = e1 + e2;
        r = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(d, d + p1));
        t = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(e, e - p1));
    };
    constexpr uint32_t LO = 0x00ff00ffu;
    uint32_t rE, tE, rO, tO;
    lanes(x1 & LO, x2 & LO, rE, tE);
    lanes((x1 >> 8) & LO, (x2 >> 8) & LO, rO, tO);
    re = rE | (rO << 8);
    sum = tE | (tO << 8);
}
template <int P> __device__ __forceinline__ uint32_t kara_sub_dword(uint32_t x3, uint32_t sum) {
    const u16x2 p1 = {(unsigned short)P, (unsigned short)P};
    auto lanes = [&](uint32_t a3, uint32_t s) {
        const u16x2 d = __builtin_bit_cast(u16x2, a3) - __builtin_bit_cast(u16x2, s);
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(d, d + p1));
    };
    constexpr uint32_t LO = 0x00ff00ffu;
    return lanes(x3 & LO, sum & LO) | (lanes((x3 >> 8) & LO, (sum >> 8) & LO) << 8);
}
template <unsigned N, typename W, unsigned... I>
__device__ __forceinline__ void kara_pair_words(const W (&w1)[N], const W (&w2)[N], W (&re)[N], W (&sum)[N],
                                                std::integer_sequence<unsigned, I...>) {
    auto one = [&](auto ic) {
        constexpr unsigned i = decltype(ic)::value;
        uint32_t r0, s0;
        kara_pair_dword<oz2_p[i]>((uint32_t)w1[i], (uint32_t)w2[i], r0, s0);
        if constexpr (sizeof(W) == 8) {
            uint32_t r1, s1;
            kara_pair_dword<oz2_p[i]>((uint32_t)(w1[i] >> 32), (uint32_t)(w2[i] >> 32), r1, s1);
            re[i] = (uint64_t)r0 | ((uint64_t)r1 << 32);
            sum[i] = (uint64_t)s0 | ((uint64_t)s1 << 32);
        } else {
            re[i] = r0;
            sum[i] = s0;
        }
        asm volatile("" : "+v"(re[i]), "+v"(sum[i]));  // computed here, so P1's and P2's words die here
    };
    (one(std::integral_constant<unsigned, I>{}), ...);
}
template <unsigned N, typename W, unsigned... I>
__device__ __forceinline__ void kara_sub_words(const W (&w3)[N], W (&sum_im)[N], std::integer_sequence<unsigned, I...>) {
    auto one = [&](auto ic) {
        constexpr unsigned i = decltype(ic)::value;
        const uint32_t lo = kara_sub_dword<oz2_p[i]>((uint32_t)w3[i], (uint32_t)sum_im[i]);
        if constexpr (sizeof(W) == 8) {
            const uint32_t hi = kara_sub_dword<oz2_p[i]>((uint32_t)(w3[i] >> 32), (uint32_t)(sum_im[i] >> 32));
            sum_im[i] = (uint64_t)lo | ((uint64_t)hi << 32);
        } else {
            sum_im[i] = lo;
        }
        asm volatile("" : "+v"(sum_im[i]));
    };
    (one(std::integral_constant<unsigned, I>{}), ...);
}
template <unsigned N, unsigned... I>
__device__ __forceinline__ void kara_words(const uint64_t (&w1)[N], const uint64_t (&w2)[N], const uint64_t (&w3)[N],
                                           uint64_t (&re)[N], uint64_t (&im)[N], std::integer_sequence<unsigned, I...>) {
    auto one = [&](auto ic) {
        constexpr unsigned i = decltype(ic)::value;
        uint32_t r0, i0, r1, i1;
        kara_dword<oz2_p[i]>((uint32_t)w1[i], (uint32_t)w2[i], (uint32_t)w3[i], r0, i0);
        kara_dword<oz2_p[i]>((uint32_t)(w1[i] >> 32), (uint32_t)(w2[i] >> 32), (uint32_t)(w3[i] >> 32), r1, i1);
        re[i] = (uint64_t)r0 | ((uint64_t)r1 << 32);
        im[i] = (uint64_t)i0 | ((uint64_t)i1 << 32);
    };
    (one(std::integral_constant<unsigned, I>{}), ...);
}

// One wave covers 512 consecutive rows of a column: lane l recombines rows 8l..8l+7
// (one 8-byte load per plane), parks the scaled values in LDS, and the wave then
// writes them back as 16-byte vectors in lane order so the C stream (the larger
// one) is fully coalesced.  The BLAS epilogue runs after the transpose, on the
// coalesced C read when beta != 0.  KARA (complex outputs): the residues of the real and
// imaginary parts come from the three Karatsuba sub-planes instead of rows r and r + m.
// LDS slot of row e of lane l in a wave's transpose buffer: l * 8 + (e ^ sw(l)), with sw(l) a multiple of
// EPV (so the EPV consecutive rows of one 16-byte read stay adjacent and in order) that differs between
// the lanes whose 8-row groups share a 256-byte LDS row; unswizzled, the 8-byte (f64) writes of a wave
// hit the same banks 16 ways (complex f64: 32 ways), swizzled 4 ways
template <typename E, int R = CRT_ROWS> __device__ __forceinline__ int crt_slot(int l, int e) {
    constexpr int EPV = 16 / sizeof(E);
    constexpr int LPR = 256 / (R * (int)sizeof(E));  // lanes per 256-byte row
    constexpr int SH = LPR >= 8 ? 3 : LPR >= 4 ? 2 : LPR >= 2 ? 1 : 0;
    return l * R + (e ^ ((EPV * (l >> SH)) & (R - 1)));
}

template <int OT, bool NUMM1, unsigned N, bool KARA = false, int R = CRT_ROWS, bool PFC = false>
__global__ __launch_bounds__(256) void crt_kernel(CrtArgs a) {
    static_assert(R == CRT_ROWS || R == 4, "rows per lane: 8 or 4");
    using W = RowWord<R>;
    using E = typename OutElem<OT>::T;
    constexpr int EPV = 16 / sizeof(E);  // elements per 16-byte vector
    __shared__ E buf[4][64 * R];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t wrow0 = ((size_t)blockIdx.x * 256 + wv * 64) * R;
    if (wrow0 >= a.m) return;  // whole wave beyond the last row (no block-level sync below)
    const size_t r0 = wrow0 + (size_t)lane * R;
    const int nr = r0 >= a.m ? 0 : (a.m - r0 >= R ? R : (int)(a.m - r0));
    const bool plain_ab = a.ar == 1.0 && a.ai == 0.0 && a.br == 0.0 && a.bi == 0.0;
    // C is not read at beta = 0 (BLAS), except by the reference's _ab kernels (reference-epilogue mode)
    const bool zero_beta = a.br == 0.0 && a.bi == 0.0 && !(a.ref_epi && !(a.ar == 1.0 && a.ai == 0.0));
    int16_t sa[R];
#pragma unroll
    for (int e = 0; e < R; ++e) sa[e] = e < nr ? a.sftA[r0 + e] : 0;
    E *wb = buf[wv];
    // real outputs with several columns per block (PF): the next column's residue words are loaded before this
    // column's CRT, so they are in flight under its arithmetic and stores
    constexpr bool PF = PFC && !KARA && OT < 2;
    W wpf[PF ? N : 1];
    if constexpr (PF) {
        if (nr > 0 && blockIdx.y < a.n) load_rows<N>(a, blockIdx.y * a.ldr + r0, nr == R, nr, wpf);
    }
    for (size_t col = blockIdx.y; col < a.n; col += gridDim.y) {
        const int sB = a.sftB[col];
        if (nr > 0) {
            W w[N], wi[N];
            const size_t off = col * a.ldr + r0;
            if constexpr (PF) {
#pragma unroll
                for (unsigned i = 0; i < N; ++i) w[i] = wpf[i];
                const size_t nxt = col + gridDim.y;
                if (nxt < a.n) load_rows<N>(a, nxt * a.ldr + r0, nr == R, nr, wpf);
            }
            if constexpr (KARA) {
                // real parts from P1, P2 first, then the imaginary parts with P3: two sub-planes' words
                // live at a time instead of three (occupancy; the residues are the same bytes)
                W w1[N], w2[N];
                load_rows<N>(a, off, nr == R, nr, w1);
                load_rows<N>(a, off + a.sub, nr == R, nr, w2);
                kara_pair_words<N>(w1, w2, w, wi, std::make_integer_sequence<unsigned, N>{});
                // P3's loads go out after that (an opaque dependency on the last combined word keeps the
                // compiler from merging them with P1's and P2's), in flight under the real parts
                size_t off3 = off + 2 * a.sub;
                asm volatile("" : "+v"(off3) : "v"(wi[N - 1]));
                W w3[N];
                load_rows<N>(a, off3, nr == R, nr, w3);
                if constexpr (OZ2_CRT_MODOUTER) {
                    double v[R];
                    crt_rows_const<N, NUMM1, R>(w, v, std::make_integer_sequence<unsigned, N>{});
#pragma unroll
                    for (int e = 0; e < R; ++e) {
                        const double vr = scalbn(v[e], (int)sa[e] + sB);
                        if constexpr (OT == 2) wb[crt_slot<E, R>(lane, e)].x = vr;
                        else wb[crt_slot<E, R>(lane, e)].x = __double2float_rn(vr);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < R; ++e) {
                        uint8_t r[N];
#pragma unroll
                        for (unsigned i = 0; i < N; ++i) r[i] = (uint8_t)(w[i] >> (8 * e));
                        const double vr = scalbn(crt_value_const<N, NUMM1>(r, std::make_integer_sequence<unsigned, N>{}),
                                                 (int)sa[e] + sB);
                        if constexpr (OT == 2) wb[crt_slot<E, R>(lane, e)].x = vr;
                        else wb[crt_slot<E, R>(lane, e)].x = __double2float_rn(vr);
                    }
                }
                asm volatile("" ::: "memory");  // the real parts go to LDS now (no merging with the imaginary ones)
                kara_sub_words<N>(w3, wi, std::make_integer_sequence<unsigned, N>{});
                if constexpr (OZ2_CRT_MODOUTER) {
                    double v[R];
                    crt_rows_const<N, NUMM1, R>(wi, v, std::make_integer_sequence<unsigned, N>{});
#pragma unroll
                    for (int e = 0; e < R; ++e) {
                        const double vi = scalbn(v[e], (int)sa[e] + sB);
                        if constexpr (OT == 2) wb[crt_slot<E, R>(lane, e)].y = vi;
                        else wb[crt_slot<E, R>(lane, e)].y = __double2float_rn(vi);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < R; ++e) {
                        uint8_t r[N];
#pragma unroll
                        for (unsigned i = 0; i < N; ++i) r[i] = (uint8_t)(wi[i] >> (8 * e));
                        const double vi = scalbn(crt_value_const<N, NUMM1>(r, std::make_integer_sequence<unsigned, N>{}),
                                                 (int)sa[e] + sB);
                        if constexpr (OT == 2) wb[crt_slot<E, R>(lane, e)].y = vi;
                        else wb[crt_slot<E, R>(lane, e)].y = __double2float_rn(vi);
                    }
                }
            } else if constexpr (!PF) {
                load_rows<N>(a, off, nr == R, nr, w);
                if (OT >= 2) load_rows<N>(a, off + a.imag_off, nr == R && (a.imag_off & 7) == 0, nr, wi);
            }
            constexpr bool MO = OZ2_CRT_MODOUTER_ALL || N >= OZ2_CRT_MODOUTER_MIN_N;
            if constexpr (!KARA && MO) {
                double vr[R], vi[R];
                crt_rows_const<N, NUMM1, R>(w, vr, std::make_integer_sequence<unsigned, N>{});
                if constexpr (OT >= 2) crt_rows_const<N, NUMM1, R>(wi, vi, std::make_integer_sequence<unsigned, N>{});
#pragma unroll
                for (int e = 0; e < R; ++e) {
                    const int sft = (int)sa[e] + sB;
                    const double x = scalbn(vr[e], sft);
                    if constexpr (OT == 0) wb[crt_slot<E, R>(lane, e)] = x;
                    else if constexpr (OT == 1) wb[crt_slot<E, R>(lane, e)] = __double2float_rn(x);
                    else if constexpr (OT == 2) wb[crt_slot<E, R>(lane, e)] = make_double2(x, scalbn(vi[e], sft));
                    else wb[crt_slot<E, R>(lane, e)] = make_float2(__double2float_rn(x), __double2float_rn(scalbn(vi[e], sft)));
                }
            }
#pragma unroll
            for (int e = 0; e < (KARA || MO ? 0 : R); ++e) {
                uint8_t r[N];
#pragma unroll
                for (unsigned i = 0; i < N; ++i) r[i] = (uint8_t)(w[i] >> (8 * e));
                const int sft = (int)sa[e] + sB;
                const double vr = scalbn(crt_value_const<N, NUMM1>(r, std::make_integer_sequence<unsigned, N>{}), sft);
                if constexpr (OT == 0) {
                    wb[crt_slot<E, R>(lane, e)] = vr;
                } else if constexpr (OT == 1) {
                    wb[crt_slot<E, R>(lane, e)] = __double2float_rn(vr);
                } else {
#pragma unroll
                    for (unsigned i = 0; i < N; ++i) r[i] = (uint8_t)(wi[i] >> (8 * e));
                    const double vi = scalbn(crt_value_const<N, NUMM1>(r, std::make_integer_sequence<unsigned, N>{}), sft);
                    if constexpr (OT == 2) wb[crt_slot<E, R>(lane, e)] = make_double2(vr, vi);
                    else wb[crt_slot<E, R>(lane, e)] = make_float2(__double2float_rn(vr), __double2float_rn(vi));
                }
            }
        }
        wave_sync();
        E *Cc = static_cast<E *>(a.C) + col * a.ldc + wrow0;
        const bool vec_ok = (reinterpret_cast<uintptr_t>(Cc) & 15) == 0;
#pragma unroll
        for (int j = 0; j < R / EPV; ++j) {
            const int idx = j * 64 * EPV + lane * EPV;
            E v[EPV];
            *reinterpret_cast<int4 *>(v) = *reinterpret_cast<const int4 *>(wb + crt_slot<E, R>(idx / R, idx % R));
            if (vec_ok && wrow0 + idx + EPV <= a.m) {
                if (!plain_ab) {
                    E c[EPV];
                    if (zero_beta) {
#pragma unroll
                        for (int q = 0; q < EPV; ++q) c[q] = E{};
                    } else {
                        *reinterpret_cast<int4 *>(c) = *reinterpret_cast<const int4 *>(Cc + idx);
                    }
#pragma unroll
                    for (int q = 0; q < EPV; ++q) v[q] = BlasEpi<OT>::template f<NUMM1>(v[q], c[q], a);
                }
                if (OZ2_CRT_NT & 2) {
                    typedef int i4v __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(*reinterpret_cast<const i4v *>(v), reinterpret_cast<i4v *>(Cc + idx));
                } else {
                    *reinterpret_cast<int4 *>(Cc + idx) = *reinterpret_cast<const int4 *>(v);
                }
            } else {
#pragma unroll
                for (int q = 0; q < EPV; ++q) {
                    if (wrow0 + idx + q < a.m) {
                        E x = v[q];
                        if (!plain_ab) x = BlasEpi<OT>::template f<NUMM1>(x, zero_beta ? E{} : Cc[idx + q], a);
                        Cc[idx + q] = x;
                    }
                }
            }
        }
        wave_sync();
    }
}

// rows per lane of the real CRT: 4 (twice the waves of 8; every wave of a block busy at m = 1024; measured
// faster at every size) without the next-column prefetch (it costs 8% at cfg2 with 4 rows; it pays with
// 8); GEMMUL8_CRT_ROWS=8 (the round-6 kernel) and GEMMUL8_CRT_PF=0/1 (read once) are the A/B switches
static int crt_env(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}
static int crt_rows_real() {
    static const int v = crt_env("GEMMUL8_CRT_ROWS", 4) == 8 ? 8 : 4;
    return v;
}
static bool crt_prefetch(int rows) {
    static const int v = crt_env("GEMMUL8_CRT_PF", -1);
    return v < 0 ? rows == 8 : v != 0;
}
template <int OT, bool NUMM1, unsigned N, bool KARA, int R>
static void launch_crt_r(const CrtArgs &a, dim3 grid, hipStream_t st) {
    grid.x = (unsigned)((a.m + 256 * R - 1) / (256 * R));
    if (!KARA && OT < 2 && grid.y < a.n && crt_prefetch(R))
        launch(crt_kernel<OT, NUMM1, N, KARA, R, true>, grid, dim3(256), st, a);
    else
        launch(crt_kernel<OT, NUMM1, N, KARA, R>, grid, dim3(256), st, a);
}
template <int OT, bool NUMM1, unsigned N, bool KARA>
static void launch_crt_n(const CrtArgs &a, dim3 grid, hipStream_t st) {
    if (!KARA && OT < 2 && crt_rows_real() == 4) launch_crt_r<OT, NUMM1, N, KARA, 4>(a, grid, st);
    else launch_crt_r<OT, NUMM1, N, KARA, KARA ? OZ2_KARA_ROWS : CRT_ROWS>(a, grid, st);
}

template <int OT, bool NUMM1, bool KARA = false>
static void launch_crt(const CrtArgs &a, unsigned N, dim3 grid, hipStream_t st) {
    switch (N) {
#define OZ2_N(n) case n: launch_crt_n<OT, NUMM1, n, KARA>(a, grid, st); break;
        OZ2_N(2) OZ2_N(3) OZ2_N(4) OZ2_N(5) OZ2_N(6) OZ2_N(7) OZ2_N(8) OZ2_N(9) OZ2_N(10) OZ2_N(11)
        OZ2_N(12) OZ2_N(13) OZ2_N(14) OZ2_N(15) OZ2_N(16) OZ2_N(17) OZ2_N(18) OZ2_N(19) OZ2_N(20)
#undef OZ2_N
    default: break;
    }
}

void crt_inverse(const uint8_t *R, const Layout &L, const int16_t *sftA, const int16_t *sftB, const CrtParams &CP,
                 OutType ot, const void *alpha, const void *beta, void *C, size_t ldc, hipStream_t st, int ref_epi) {
    CrtArgs a{};
    a.ref_epi = ref_epi;
    a.R = R;
    a.planeR = L.planeR;
    a.ldr = L.ldr;
    a.m = L.m;
    a.n = L.n;
    a.imag_off = L.cplx && !L.kara ? L.m : 0;
    a.sub = L.kara ? L.subR : 0;
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
    const unsigned gx = (unsigned)((L.m + 256 * CRT_ROWS - 1) / (256 * CRT_ROWS));
    // columns per block of the real CRT: the next column's residues are prefetched under the current one's
    // arithmetic (crt_kernel, PF).  4 from n = 4096 (cfg2 CRT 0.2622 -> 0.2593 ms, 8192^2 x 1024 0.2679 ->
    // 0.2651 ms, three interleaved rounds, same bits: profiles/r06/crt_cols/); GEMMUL8_CRT_COLS (read once) forces it
    static const int cols_forced = [] {
        const char *e = getenv("GEMMUL8_CRT_COLS");
        const int v = e ? atoi(e) : 0;
        return v >= 1 && v <= 64 ? v : 0;
    }();
    const unsigned cpb = (ot == OutType::F64 || ot == OutType::F32) ? (cols_forced ? (unsigned)cols_forced : L.n >= 4096 ? 4u : 1u) : 1u;
    const size_t gyn = (L.n + cpb - 1) / cpb;
    const unsigned gy = (unsigned)(gyn < 65535 ? gyn : 65535);
    dim3 grid(gx, gy);
    const bool nm1 = CP.numM1 != 0;
    switch (ot) {
    case OutType::F64: if (nm1) launch_crt<0, true>(a, CP.N, grid, st); else launch_crt<0, false>(a, CP.N, grid, st); break;
    case OutType::F32: launch_crt<1, true>(a, CP.N, grid, st); break;
    case OutType::C64:
        if (L.kara) { if (nm1) launch_crt<2, true, true>(a, CP.N, grid, st); else launch_crt<2, false, true>(a, CP.N, grid, st); }
        else { if (nm1) launch_crt<2, true>(a, CP.N, grid, st); else launch_crt<2, false>(a, CP.N, grid, st); }
        break;
    default: if (L.kara) launch_crt<3, true, true>(a, CP.N, grid, st); else launch_crt<3, true>(a, CP.N, grid, st); break;
    }
}

// ---------------------------------------------------------------------------------------------
// Partial CRT sums of a moduli range and the CRT finished from summed partials: the north star's
// multi-GPU form (BASELINE.json: "a single RCCL reduce of partial FP64 accumulators"), gemmul8/dist.py
// gemm_moduli_reduce.  A rank that holds the residue planes of moduli [j0, j1) writes per element
// C1_g = sum hi_i r_i and C2_g = sum lo_i r_i over its range (the reference's fma chains of
// inverse_scaling.hpp:138-172 restricted to it, i ascending; numM = 1: C_g = sum NMi_i r_i and C2_g = 0);
// the ranks sum the two planes (RCCL reduce) and one finish applies the reference's tail: quot, the two-
// step reduction, the scaling and the BLAS epilogue.  C1 is exact in any order (every term and partial sum
// is a multiple of 2^tz below 2^(53+tz)), so C1 equals the single call's; C2 (the low words) and numM = 1
// at N = 6, 7 are rounded sums whose order the reduce changes: C is then within a few ulp of the single
// call's, not bit-identical (tests/test_gpu_phases.py measures it).  Real outputs only.
struct CrtPartialArgs {
    const uint8_t *R;
    size_t planeR, ldr, m, n;
    unsigned j0, j1;
    int numM1;
    double whi[OZ2_MAX_MODULI], wlo[OZ2_MAX_MODULI];
    double *S;
    size_t lds;
};

__global__ __launch_bounds__(256) void crt_partial_kernel(CrtPartialArgs a) {
    const size_t r0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * CRT_ROWS;
    if (r0 >= a.m) return;
    const int nr = a.m - r0 >= CRT_ROWS ? CRT_ROWS : (int)(a.m - r0);
    for (size_t col = blockIdx.y; col < a.n; col += gridDim.y) {
        double c1[CRT_ROWS] = {}, c2[CRT_ROWS] = {};
        const uint8_t *q = a.R + col * a.ldr + r0;
        for (unsigned j = a.j0; j < a.j1; ++j) {
            uint64_t w = 0;
            if (nr == CRT_ROWS) w = *reinterpret_cast<const uint64_t *>(q + j * a.planeR);
            else
                for (int e = 0; e < nr; ++e) w |= (uint64_t)q[j * a.planeR + e] << (8 * e);
            const double hi = a.whi[j], lo = a.wlo[j];
#pragma unroll
            for (int e = 0; e < CRT_ROWS; ++e) {
                const double r = (double)(uint8_t)(w >> (8 * e));
                c1[e] = __builtin_fma(hi, r, c1[e]);
                if (!a.numM1) c2[e] = __builtin_fma(lo, r, c2[e]);
            }
        }
        double *s1 = a.S + col * a.lds + r0, *s2 = s1 + a.n * a.lds;
        for (int e = 0; e < nr; ++e) {
            s1[e] = c1[e];
            s2[e] = c2[e];
        }
    }
}

struct CrtFinishArgs {
    const double *S;
    size_t lds, m, n;
    const int16_t *sftA, *sftB;
    void *C;
    size_t ldc;
    int f32, numM1, ref_epi;
    double invM, M1, M2, ar, br;
};

__global__ __launch_bounds__(256) void crt_finish_kernel(CrtFinishArgs a) {
    const size_t row = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (row >= a.m) return;
    const int sA = a.sftA[row];
    for (size_t col = blockIdx.y; col < a.n; col += gridDim.y) {
        const double C1 = a.S[col * a.lds + row], C2 = a.S[(a.n + col) * a.lds + row];
        double v;
        if (a.numM1) {
            const double quot = -__builtin_rint(C1 * a.invM);
            v = __builtin_fma(quot, a.M1, C1);
        } else {
            const double quot = -__builtin_rint(__builtin_fma(C1, a.invM, C2 * a.invM));
            const double t1 = __builtin_fma(quot, a.M1, C1) + C2;
            v = __builtin_fma(quot, a.M2, t1);
        }
        v = scalbn(v, sA + (int)a.sftB[col]);
        const bool zero_beta = a.br == 0.0 && !(a.ref_epi && a.ar != 1.0);
        if (a.f32) {
            float *C = static_cast<float *>(a.C) + col * a.ldc + row;
            const float x = __double2float_rn(v);
            *C = (a.ar == 1.0 && a.br == 0.0) ? x : epi_f(x, zero_beta ? 0.f : *C, (float)a.ar, (float)a.br, a.ref_epi != 0);
        } else {
            double *C = static_cast<double *>(a.C) + col * a.ldc + row;
            *C = (a.ar == 1.0 && a.br == 0.0) ? v : epi_d(v, zero_beta ? 0.0 : *C, a.ar, a.br, a.ref_epi != 0, a.numM1 != 0);
        }
    }
}

void crt_partial(const uint8_t *R, const Layout &L, unsigned N, bool numM1, unsigned j0, unsigned j1, double *S,
                 size_t lds, hipStream_t st) {
    CrtPartialArgs a{};
    a.R = R;
    a.planeR = L.planeR;
    a.ldr = L.ldr;
    a.m = L.m;
    a.n = L.n;
    a.j0 = j0;
    a.j1 = j1;
    a.numM1 = numM1 ? 1 : 0;
    for (unsigned j = 0; j < N; ++j) {
        a.whi[j] = numM1 ? oz2_NMi_1[N - 2][j] : oz2_NMi_2[N - 8][j][0];
        a.wlo[j] = numM1 ? 0.0 : oz2_NMi_2[N - 8][j][1];
    }
    a.S = S;
    a.lds = lds;
    const dim3 grid((unsigned)((L.m + 256 * CRT_ROWS - 1) / (256 * CRT_ROWS)), (unsigned)(L.n < 65535 ? L.n : 65535));
    launch(crt_partial_kernel, grid, dim3(256), st, a);
}

void crt_finish(const double *S, size_t lds, const Layout &L, unsigned N, bool numM1, const int16_t *sftA,
                const int16_t *sftB, bool f32, const void *alpha, const void *beta, void *C, size_t ldc,
                hipStream_t st, int ref_epi) {
    CrtFinishArgs a{};
    a.S = S;
    a.lds = lds;
    a.m = L.m;
    a.n = L.n;
    a.sftA = sftA;
    a.sftB = sftB;
    a.C = C;
    a.ldc = ldc;
    a.f32 = f32 ? 1 : 0;
    a.numM1 = numM1 ? 1 : 0;
    a.ref_epi = ref_epi;
    a.invM = oz2_invM[N - 2];
    a.M1 = oz2_M_hi[N - 2];
    a.M2 = oz2_M_lo[N - 2];
    a.ar = f32 ? (double)*(const float *)alpha : *(const double *)alpha;
    a.br = f32 ? (double)*(const float *)beta : *(const double *)beta;
    const dim3 grid((unsigned)((L.m + 255) / 256), (unsigned)(L.n < 65535 ? L.n : 65535));
    launch(crt_finish_kernel, grid, dim3(256), st, a);
}

}  // namespace oz2
