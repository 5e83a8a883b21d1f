// split.hip -- slice extraction and residue encoding for gfx950 ("scaling" stage).
//
// Two passes per operand, both HBM-streaming:
//   1. stats:  per vector (row of op(A) / column of op(B)) amax and the round-up
//              sum of squares, reduced in exactly the order the reference reduces
//              them on gfx950 (thread-strided partials of `VT` threads, wave64
//              __shfl_down tree, lane-1 group pickup -- GEMMul8/src/scaling.hpp:155-213),
//              then the shift (vecnorm::compute_sft, scaling.hpp:3373-3383).  The
//              partials are computed from coalesced loads: a strided (column-major
//              row) vector is swept 16 rows at a time, so every wave load is a
//              contiguous run of rows instead of the reference's lda-strided walk
//              or its stair_kernel copy (scaling.hpp:232-239, 3703-3710).
//   2. encode: 64-vector x 64-element tiles staged through LDS, trunc(x*2^sft),
//              N residues per element (mod_8i, scaling.hpp:215-230), written as
//              16-byte chunks straight into the MFMA-ready panel layout.
// Accurate mode adds the 6-bit magnitude extraction (scaling.hpp:1897-1941,
// 2215-2260) whose bound product runs on the int8 GEMM kernel (gemm_i8.hip).
#include <climits>

#include "oz2_split.hpp"
#include <cstdlib>

namespace oz2 {

enum : int { ENC_CONJ = 1, ENC_BTAIL = 2, ENC_KFIRST = 4, ENC_KARA = 8 };

// (a + b) mod p as the symmetric representative of an int8 slice, for residues a, b of mod_8i
// (|a|, |b| <= p/2; p = 256: any byte of a + b is the residue)
__device__ __forceinline__ int center_sum(int a, int b, int p) {
    const int h = (p - 1) >> 1;
    int s = a + b;
    s -= s > h ? p : 0;
    s += s < -h ? p : 0;
    return s;
}
#ifndef OZ2_ENC_ABLATE
#define OZ2_ENC_ABLATE 0  // probe builds only (tools/probes/enc_probe.hip, fused_probe.hip)
#endif
#ifndef OZ2_ENC_NTS
#define OZ2_ENC_NTS 0  // probe builds only: 1 = non-temporal slice stores (real operands)
#endif

// f64 residues in groups of moduli.  mod_8i (scaling.hpp:215-223) reduces the integer-valued x
// with one f64 step per modulus (x - rint(x/p)*p) and finishes in f32.  Both steps are exact, so
// the result is THE symmetric residue of x (for p = 256 the two ties +-128 are the same byte).
// Here x is reduced once modulo the product P of a group in f64, and each p of the group then
// finishes in f32 from that value:
//   pairs (N <= 17): P < 2^16, |x| < 2^72 (fast: log2M_fast[N] < 65; accurate: 6 + log2M_accu[N] < 72),
//     so the f64 step leaves |t| <= P/2 + |x| 2^-52 < 2^21, exact in f32, and ONE f32 step is exact
//     (rint(t*fl(1/p)) is off from t/p by < 2^-23 |t/p| < 2^-9, less than the 1/(2p) separating t/p
//     from a half-integer when p is odd; p = 256: exact product, a tie gives +-128, one byte);
//   triples (N >= 18): P < 2^24, two f32 steps (the reference's own two).
// Same residues as mod_8i either way (tools/probes/modcheck.py checks both forms against exact
// integers over the magnitude range); per element, 7 f64 steps and 14 packed f32 steps at N = 14.
// f32 operands: mod_8i<float> (scaling.hpp:225-230) takes four f32 steps from x itself.  For
// |x| < 2^46 the first step's quotient errs by < 2^23/p, so its fma result is an exact integer
// below 2^24 and the remaining steps end at THE symmetric residue; |x| < 2^(6 + log2M_accu[N]) <=
// 2^45.2 holds for N <= 10 in both modes, and there the f64 group form (x converted exactly)
// gives the same bytes.  Above N = 10 the four f32 steps are kept as they are, rounding included.
struct ModGroups {
    int ng;
    int steps;      // f32 steps per modulus (1: pairs, 2: triples)
    int f32_exact;  // f32 operands: mod_8i<float>'s four f32 steps are exact (N <= 10), so the f64 form applies
    int bytes;      // pair form straight to bytes (plane_bytes); GEMMUL8_ENC_BYTES=0 keeps the convert-and-pack form
    int start[OZ2_MAX_MODULI + 1];
    double P[OZ2_MAX_MODULI];
    double rP[OZ2_MAX_MODULI];
};
static ModGroups make_groups(const ModParams &MP, unsigned Ncall) {
    ModGroups G{};
    static const bool triples = [] {  // GEMMUL8_ENC_TRIPLES=1: the triple form at every N (A-B runs)
        const char *e = getenv("GEMMUL8_ENC_TRIPLES");
        return e && atoi(e) != 0;
    }();
    const unsigned gs = (Ncall <= 17 && !triples) ? 2 : 3;
    G.steps = gs == 2 ? 1 : 2;
    G.f32_exact = Ncall <= 10 && !triples;
    static const bool no_bytes = [] {
        const char *e = getenv("GEMMUL8_ENC_BYTES");
        return e && atoi(e) == 0;
    }();
    G.bytes = !no_bytes;
    unsigned j = 0;
    while (j < MP.N) {
        const unsigned e = j + gs < MP.N ? j + gs : MP.N;
        double P = 1.0;
        for (unsigned i = j; i < e; ++i) P *= (double)(MP.p[i] > 0 ? MP.p[i] : 256);
        G.start[G.ng] = (int)j;
        G.P[G.ng] = P;
        G.rP[G.ng] = 1.0 / P;
        ++G.ng;
        j = e;
    }
    G.start[G.ng] = (int)MP.N;
    return G;
}

template <typename R> __device__ __forceinline__ R add_ru(R a, R b);
template <> __device__ __forceinline__ double add_ru<double>(double a, double b) { return __dadd_ru(a, b); }
template <> __device__ __forceinline__ float add_ru<float>(float a, float b) { return __fadd_ru(a, b); }

#ifndef OZ2_STATS_XCD
#define OZ2_STATS_XCD 1  // A/B builds: 0 = strided stats blocks in dispatch order (no XCD renumbering)
#endif
// loads in flight per thread in the stats passes (probe builds vary them: tools/probes/stats_probe.hip, in git
// history at ae0caaa)
#ifndef OZ2_STRIDED_LOADS
#define OZ2_STRIDED_LOADS 16
#endif
#ifndef OZ2_CONTIG_LOADS
#define OZ2_CONTIG_LOADS 8
#endif

// reference wave tree: __shfl_down width 64, steps 16..1 (inner_warp_sum on wave64)
template <typename R> __device__ __forceinline__ R ref_wave_sum(R v) {
#pragma unroll
    for (int d = 16; d >= 1; d >>= 1) v = add_ru<R>(v, __shfl_down(v, d));
    return v;
}
template <typename R> __device__ __forceinline__ R wave_max(R v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = fmax(v, __shfl_xor(v, d));
    return v;
}

// vecnorm::compute_sft (scaling.hpp:3373-3383)
__device__ __forceinline__ int compute_sft(double amax, double vecnrm, float log2M) {
    const int e = ilogb(vecnrm);
    const float vf = __double2float_ru(scalbn(vecnrm, -e));
    const int kk = __float2int_rd(__fmaf_rd(-0.51F, __fadd_ru(__log2f(vf), (float)e), log2M));
    return min(__float2int_rd(log2M - 1.0f), kk) - ilogb(amax);
}
__device__ __forceinline__ int compute_sft(float amax, float vecnrm, float log2M) {
    const int kk = __float2int_rd(__fmaf_rd(-0.51F, __log2f(vecnrm), log2M));
    return min(__float2int_rd(log2M - 1.0f), kk) - ilogbf(amax);
}

// Accurate mode: the reference scales the 6-bit magnitudes with the int sft0 = 5 - ilogb(amax)
// (scaling.hpp:1909-1925) and keeps its int16 in sftA for the shift that follows.  The two differ
// only for amax = Inf: 5 - INT_MAX sends every finite magnitude to 0, its int16 (6) does not.  That
// case is stored as SFT0_INF, which neither finite amax (sft0 in [-1018, 1079]) nor amax = 0 can
// produce, and its two readers map it back: sft0_scale (the magnitude encode) to the int,
// sft0_stored (the final shift) to the int16.
constexpr int16_t SFT0_INF = INT16_MIN;
template <typename R> __device__ __forceinline__ int ilogb_r(R x) {
    return std::is_same<R, double>::value ? ilogb((double)x) : ilogbf((float)x);
}
template <typename R> __device__ __forceinline__ int16_t sft0_of(R amax) {
    return __builtin_isinf(amax) ? SFT0_INF : (int16_t)(5 - ilogb_r<R>(amax));
}
template <typename R> __device__ __forceinline__ int sft0_scale(int16_t s) {
    return s == SFT0_INF ? 5 - ilogb_r<R>(R(INFINITY)) : (int)s;
}
__device__ __forceinline__ int sft0_stored(int16_t s) {
    return s == SFT0_INF ? (int)(int16_t)(5 - ilogb((double)INFINITY)) : (int)s;
}

// NT: non-temporal loads for operands too large to stay in the Infinity Cache between the shift pass and the
// encode (they saved 6.5 % of the split at 8192^3 and cost 5-10 % below 4096^3, where the encode's re-read
// still hits the cache: tools/probes/nt_probe.py); the launchers pick it by operand size (use_nt).
template <typename R, bool CPLX, bool NT = false>
__device__ __forceinline__ void load_elem(const R *__restrict__ X, size_t idx, R &re, R &im) {
    if constexpr (CPLX) {
        typedef R R2v __attribute__((ext_vector_type(2)));
        const R2v *p = reinterpret_cast<const R2v *>(X) + idx;
        R2v z;
        if constexpr (NT) z = __builtin_nontemporal_load(p);
        else z = *p;
        re = z.x;
        im = z.y;
    } else {
        if constexpr (NT) re = __builtin_nontemporal_load(X + idx);
        else re = X[idx];
        im = 0;
    }
}

// s + x*x rounded upward (the reference's __fma_ru on the sum of squares, scaling.hpp:155-213) as
// inline code: the OCML helper behind __fma_ru is a call whose entry waits for every memory access
// in flight (s_waitcnt 0), which held each load of the stats passes behind the previous element's
// fma.  Same instruction, same rounding mode switch: FP64 round bits MODE[3:2], FP32 MODE[1:0],
// 1 = toward +inf, restored to 0 (nearest even, the kernels' mode) after one wait state.
template <typename R> __device__ __forceinline__ R sq_add_ru(R x, R s);
template <> __device__ __forceinline__ double sq_add_ru<double>(double x, double s) {
    asm("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 1\n\t"
        "v_fma_f64 %0, %1, %1, %0\n\t"
        "s_nop 0\n\t"
        "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 0"
        : "+v"(s)
        : "v"(x));
    return s;
}
template <> __device__ __forceinline__ float sq_add_ru<float>(float x, float s) {
    asm("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 2), 1\n\t"
        "v_fma_f32 %0, %1, %1, %0\n\t"
        "s_nop 0\n\t"
        "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 2), 0"
        : "+v"(s)
        : "v"(x));
    return s;
}

// Two chains of four round-up steps each (s0 += x[i]^2, s1 += y[i]^2 in order i, rounded upward) under ONE mode
// switch: the same instructions and roundings as eight sq_add_ru, for a wave that runs the chains alone (the
// fused split's vectors), where each switch's pipeline drain sat on the critical path.
__device__ __forceinline__ void sq_add4x2_ru(const double (&x)[4], const double (&y)[4], double &s0, double &s1) {
    asm("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 1\n\t"
        "v_fma_f64 %0, %2, %2, %0\n\t"
        "v_fma_f64 %1, %6, %6, %1\n\t"
        "v_fma_f64 %0, %3, %3, %0\n\t"
        "v_fma_f64 %1, %7, %7, %1\n\t"
        "v_fma_f64 %0, %4, %4, %0\n\t"
        "v_fma_f64 %1, %8, %8, %1\n\t"
        "v_fma_f64 %0, %5, %5, %0\n\t"
        "v_fma_f64 %1, %9, %9, %1\n\t"
        "s_nop 0\n\t"
        "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 0"
        : "+v"(s0), "+v"(s1)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]));
}

// SUM = false: the accurate-mode pass, which needs amax only
template <typename R, bool CPLX, bool SUM = true>
__device__ __forceinline__ void accum(R re, R im, R &amax, R &sum) {
    re = fabs(re);
    if constexpr (CPLX) {
        im = fabs(im);
        amax = fmax(amax, fmax(re, im));
        if (SUM) {
            sum = sq_add_ru<R>(re, sum);
            sum = sq_add_ru<R>(im, sum);
        }
    } else {
        amax = fmax(amax, re);
        if (SUM) sum = sq_add_ru<R>(re, sum);
    }
}

// ------------------------------------------------------------------
// pass 1a: contiguous vectors (B op N, A op T): one vector per VT-thread block
// ------------------------------------------------------------------
// vector v by the VT threads t = 0..VT-1 of a block (or of one half of a 2 VT block: every thread of
// the block must call it, it holds a barrier); v >= nvec computes nothing and stores nothing
template <typename R, bool CPLX, int VT, bool ACCU, bool NT = false>
__device__ __forceinline__ void stats_contig_body(const R *__restrict__ X, size_t ld, size_t len, size_t nvec,
                                                  float log2M, int16_t *__restrict__ sft_out, size_t v, int t,
                                                  R (&grp)[32], R (&gmax)[8]) {
    const int lane = t & 63, w = t >> 6;
    const R *__restrict__ x = X + (CPLX ? 2 : 1) * (v < nvec ? v : 0) * ld;
    if (v >= nvec) len = 0;
    R amax = 0, sum = 0;
    // loads are issued in unguarded batches of U ahead of the round-up chain (whose
    // mode-register writes would otherwise serialise each load behind the previous fma)
    constexpr int U = OZ2_CONTIG_LOADS;
    size_t e = t;
    for (; e + (U - 1) * VT < len; e += U * VT) {
        R re[U], im[U];
#pragma unroll
        for (int u = 0; u < U; ++u) load_elem<R, CPLX, NT>(x, e + u * VT, re[u], im[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) accum<R, CPLX, !ACCU>(re[u], im[u], amax, sum);
    }
    for (; e < len; e += VT) {
        R re, im;
        load_elem<R, CPLX, NT>(x, e, re, im);
        accum<R, CPLX, !ACCU>(re, im, amax, sum);
    }
    amax = wave_max<R>(amax);
    if (!ACCU) {
        sum = ref_wave_sum<R>(sum);
        if (lane == 1) grp[2 * w] = sum;
        if (lane == 33) grp[2 * w + 1] = sum;
    }
    if (lane == 0) gmax[w] = amax;
    __syncthreads();
    if (w == 0) {
        R mx = lane < VT / 64 ? gmax[lane] : R(0);
        mx = wave_max<R>(mx);
        if (ACCU) {
            if (lane == 0 && v < nvec) sft_out[v] = sft0_of<R>(mx);
        } else {
            R s2 = (lane >= 32 && lane - 32 < VT / 32) ? grp[lane - 32] : R(0);
            s2 = ref_wave_sum<R>(s2);
            const R nrm = __shfl(s2, 32);
            if (lane == 0 && v < nvec) sft_out[v] = (int16_t)(-compute_sft(mx, nrm, log2M));
        }
    }
}
template <typename R, bool CPLX, int VT, bool ACCU, bool NT>
__global__ __launch_bounds__(VT) void stats_contig_kernel(const R *__restrict__ X, size_t ld, size_t len, size_t nvec,
                                                         float log2M, int16_t *__restrict__ sft_out) {
    __shared__ R grp[32];
    __shared__ R gmax[8];
    stats_contig_body<R, CPLX, VT, ACCU, NT>(X, ld, len, nvec, log2M, sft_out, blockIdx.x, threadIdx.x, grp, gmax);
}

// ------------------------------------------------------------------
// pass 1b: strided vectors (A op N, B op T): ROWS vectors per 256-thread block, swept
// ROWS rows at a time so every wave load is a contiguous run of rows; thread (row, slot)
// carries the reference's virtual threads t = slot + SLOTS*c (c < NA).  The loads of U
// consecutive VT-chunks are issued before any of them is accumulated; each chain still
// consumes its elements in increasing order, so the round-up sums are unchanged.
// ROWS = 16 for m >= 4096; 8 / 4 below, where m/16 blocks leave CUs idle (1024: 15.2 -> 9.6 us,
// 2048: 23.2 -> 17.3 us; narrower rows cost HBM efficiency at 4096 and up: tools/probes/run_stats_rows.sh,
// in git history at ae0caaa).
// ------------------------------------------------------------------
template <typename R, int VT, int ROWS> struct StridedShared {
    R part[ROWS][VT + 1];
    R pmax[ROWS][256 / ROWS + 1];
};
template <typename R, bool CPLX, int VT, bool ACCU, int ROWS, bool NT = false>
__device__ __forceinline__ void stats_strided_body(const R *__restrict__ X, size_t ld, size_t len, size_t nvec,
                                                   float log2M, int16_t *__restrict__ sft_out, unsigned bx,
                                                   StridedShared<R, VT, ROWS> &sh) {
    constexpr int SLOTS = 256 / ROWS;
    constexpr int NA = VT / SLOTS;
    // loads in flight per thread: U * NA (OZ2_STRIDED_LOADS; probe builds vary it)
    constexpr int U = NA >= OZ2_STRIDED_LOADS ? 1 : OZ2_STRIDED_LOADS / NA;
    static_assert(SLOTS <= 64 && NA >= 1, "one reduction lane per slot");
    auto &part = sh.part;
    auto &pmax = sh.pmax;
    const int tid = threadIdx.x, row = tid % ROWS, slot = tid / ROWS;
    const size_t v = (size_t)bx * ROWS + row;
    R acc[NA];
#pragma unroll
    for (int c = 0; c < NA; ++c) acc[c] = 0;
    R amax = 0;
    if (v < nvec) {
        size_t b = 0;
        // full groups of U chunks: U*NA loads in flight, then the chains in element order
        for (; b + (size_t)U * VT <= len; b += (size_t)U * VT) {
            R re[U][NA], im[U][NA];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < NA; ++c) load_elem<R, CPLX, NT>(X, (b + u * VT + slot + SLOTS * c) * ld + v, re[u][c], im[u][c]);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < NA; ++c) accum<R, CPLX, !ACCU>(re[u][c], im[u][c], amax, acc[c]);
        }
        for (; b + VT <= len; b += VT) {
            R re[NA], im[NA];
#pragma unroll
            for (int c = 0; c < NA; ++c) load_elem<R, CPLX, NT>(X, (b + slot + SLOTS * c) * ld + v, re[c], im[c]);
#pragma unroll
            for (int c = 0; c < NA; ++c) accum<R, CPLX, !ACCU>(re[c], im[c], amax, acc[c]);
        }
        for (; b < len; b += VT) {
#pragma unroll
            for (int c = 0; c < NA; ++c) {
                const size_t e = b + slot + SLOTS * c;
                if (e < len) {
                    R re, im;
                    load_elem<R, CPLX, NT>(X, e * ld + v, re, im);
                    accum<R, CPLX, !ACCU>(re, im, amax, acc[c]);
                }
            }
        }
    }
    if (!ACCU) {
#pragma unroll
        for (int c = 0; c < NA; ++c) part[row][slot + SLOTS * c] = acc[c];
    }
    pmax[row][slot] = amax;
    __syncthreads();
    const int w = tid >> 6, lane = tid & 63;
#pragma unroll 1
    for (int r2 = w; r2 < ROWS; r2 += 4) {
        const size_t v2 = (size_t)bx * ROWS + r2;
        R mx = lane < SLOTS ? pmax[r2][lane] : R(0);
        mx = wave_max<R>(mx);
        if (ACCU) {
            if (lane == 0 && v2 < nvec) sft_out[v2] = sft0_of<R>(mx);
            continue;
        }
        R gv = 0;
#pragma unroll
        for (int vw = 0; vw < VT / 64; ++vw) {
            R s = ref_wave_sum<R>(part[r2][64 * vw + lane]);
            const R g0 = __shfl(s, 1), g1 = __shfl(s, 33);
            if (lane == 32 + 2 * vw) gv = g0;
            if (lane == 33 + 2 * vw) gv = g1;
        }
        gv = ref_wave_sum<R>(gv);
        const R nrm = __shfl(gv, 32);
        if (lane == 0 && v2 < nvec) sft_out[v2] = (int16_t)(-compute_sft(mx, nrm, log2M));
    }
}
// Blocks of fewer than 16 rows share the 128-byte lines of a strided sweep (16 f64 rows) with their neighbours: the
// blocks the dispatcher deals round-robin over the 8 XCDs are renumbered so that neighbours run on one XCD and its L2
// serves the line once (xcd_local_block: the GEMM's bijective XCD remap, over the first `nb` blocks)
__device__ __forceinline__ unsigned xcd_local_block(unsigned bid, unsigned nb) {
    const unsigned xcd = bid & 7, q8 = nb >> 3, r8 = nb & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}
template <typename R, bool CPLX, int VT, bool ACCU, int ROWS, bool NT>
__global__ __launch_bounds__(256) void stats_strided_kernel(const R *__restrict__ X, size_t ld, size_t len, size_t nvec,
                                                           float log2M, int16_t *__restrict__ sft_out) {
    __shared__ StridedShared<R, VT, ROWS> sh;
    const unsigned bx = ROWS < 16 && OZ2_STATS_XCD ? xcd_local_block(blockIdx.x, gridDim.x) : blockIdx.x;
    stats_strided_body<R, CPLX, VT, ACCU, ROWS, NT>(X, ld, len, nvec, log2M, sft_out, bx, sh);
}

// Both operands' fast-mode shifts in one launch (small problems, one stream; real f64, A rows strided,
// B columns contiguous, VT = 128): blocks [0, ga) sweep ROWS rows of A each, the others two columns of
// B each (one per 128-thread half, the contiguous pass's own block shape).
template <int ROWS, bool NT>
__global__ __launch_bounds__(256) void stats_pair_kernel(const double *__restrict__ A, size_t lda, size_t m,
                                                        const double *__restrict__ B, size_t ldb, size_t n, size_t len,
                                                        float log2M, int16_t *__restrict__ sftA,
                                                        int16_t *__restrict__ sftB, unsigned ga) {
    __shared__ StridedShared<double, 128, ROWS> sh;
    __shared__ double grp[2][32];
    __shared__ double gmax[2][8];
    if (blockIdx.x < ga) {
        // (the A blocks come first, so their block id modulo 8 is their XCD)
        const unsigned bx = ROWS < 16 && OZ2_STATS_XCD ? xcd_local_block(blockIdx.x, ga) : blockIdx.x;
        stats_strided_body<double, false, 128, false, ROWS, NT>(A, lda, len, m, log2M, sftA, bx, sh);
    } else {
        const int half = threadIdx.x >> 7;
        const size_t v = 2 * (size_t)(blockIdx.x - ga) + half;
        stats_contig_body<double, false, 128, false, NT>(B, ldb, len, n, log2M, sftB, v, threadIdx.x & 127, grp[half],
                                                     gmax[half]);
    }
}

// ------------------------------------------------------------------
// pass 2: encode.  Tile = 64 vectors x KT elements through LDS.
//   MODE 0: residues of trunc(x * 2^sft), N planes (fast & accurate modes)
//   MODE 1: 6-bit magnitudes ceil(|x| * 2^sft0), 1 plane (accurate-mode bound)
//   MODE 2: MODE 0 for f32 operands whose residues need mod_8i<float>'s four f32 steps (N > 10), in a
//           kernel without the f64 group form, whose registers (260 for complex f32) would otherwise set
//           its occupancy
// Complex A (IS_A): row v <- [re, -im], row v+m <- [im, re]  (scaling.hpp:753-838)
// Complex B:        col v <- [re; im]                           (scaling.hpp:1150-1230)
// flags: ENC_CONJ (op C: the imaginary part enters negated, scaling.hpp:840-1089,
// 1232-1498); ENC_BTAIL (accurate mode, big-matrix B: the reference's tail loop
// stores the last k mod 4 imaginary magnitudes outside the column, leaving them 0 in
// the bound product -- extract_B8i_kernel_bigmatrix, scaling.hpp:2313-2321).
// ------------------------------------------------------------------
// The N slices (MODE 0) or the magnitude plane (MODE 1) of 16 consecutive elements kk..kk+15 of
// vector v, already scaled (yr, yi = trunc(x * 2^sft) resp. |x| * 2^sft0), into the panel layout.
template <typename R, bool CPLX, bool IS_A, int MODE>
__device__ __forceinline__ void encode_vec16(const R (&yr)[16], const R (&yi)[16], size_t v, size_t kk, size_t nvec,
                                             size_t len, int8_t *__restrict__ out, size_t plane, size_t ksteps,
                                             size_t kblk, size_t vmax, int flags, const ModParams &MP,
                                             const ModGroups &G) {
    const bool top = v < nvec || !CPLX || !IS_A;  // complex A: rows >= m only emit their (zero) bottom copy
    const bool kara = CPLX && (flags & ENC_KARA) != 0;
    // one plane of slices: real -> (v, kk); complex A -> [wr, -wi] / [wi, wr]; complex B -> [wr; wi];
    // Karatsuba (either operand): vectors v, v + vmax, v + 2 vmax <- wr, wi, ws = (wr + wi) mod p
    auto emit = [&](int8_t *o, const uint32_t (&wr)[4], const uint32_t (&wi)[4], const uint32_t (&ws)[4]) {
        if (!CPLX) {
            if (OZ2_ENC_ABLATE == 3)  // probe builds only: vector-major slices (each vector's bytes contiguous)
                *reinterpret_cast<uint4 *>(o + v * ksteps * KSTEP + kk) = make_uint4(wr[0], wr[1], wr[2], wr[3]);
            else if (OZ2_ENC_ABLATE == 4)  // probe builds only: no slice stores
                asm volatile("" ::"v"(wr[0]), "v"(wr[1]), "v"(wr[2]), "v"(wr[3]));
            else if (OZ2_ENC_NTS) {
                typedef unsigned u4v __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(u4v{wr[0], wr[1], wr[2], wr[3]},
                                            reinterpret_cast<u4v *>(o + panel_offset(v, kk, ksteps)));
            } else
                *reinterpret_cast<uint4 *>(o + panel_offset(v, kk, ksteps)) = make_uint4(wr[0], wr[1], wr[2], wr[3]);
        } else if (kara) {
            *reinterpret_cast<uint4 *>(o + panel_offset(v, kk, ksteps)) = make_uint4(wr[0], wr[1], wr[2], wr[3]);
            *reinterpret_cast<uint4 *>(o + panel_offset(v + vmax, kk, ksteps)) = make_uint4(wi[0], wi[1], wi[2], wi[3]);
            *reinterpret_cast<uint4 *>(o + panel_offset(v + 2 * vmax, kk, ksteps)) = make_uint4(ws[0], ws[1], ws[2], ws[3]);
        } else if (IS_A) {
            // -im as bytes: per-byte two's complement negation
            uint32_t ni[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                uint32_t r = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) r |= ((0u - ((wi[d] >> (8 * b)) & 0xffu)) & 0xffu) << (8 * b);
                ni[d] = r;
            }
            const size_t vb = v + nvec;  // bottom row (v + m)
            if (top) {
                *reinterpret_cast<uint4 *>(o + panel_offset(v, kk, ksteps)) = make_uint4(wr[0], wr[1], wr[2], wr[3]);
                *reinterpret_cast<uint4 *>(o + panel_offset(v, kblk + kk, ksteps)) = make_uint4(ni[0], ni[1], ni[2], ni[3]);
            }
            if (vb < vmax) {
                *reinterpret_cast<uint4 *>(o + panel_offset(vb, kk, ksteps)) = make_uint4(wi[0], wi[1], wi[2], wi[3]);
                *reinterpret_cast<uint4 *>(o + panel_offset(vb, kblk + kk, ksteps)) = make_uint4(wr[0], wr[1], wr[2], wr[3]);
            }
        } else {
            *reinterpret_cast<uint4 *>(o + panel_offset(v, kk, ksteps)) = make_uint4(wr[0], wr[1], wr[2], wr[3]);
            *reinterpret_cast<uint4 *>(o + panel_offset(v, kblk + kk, ksteps)) = make_uint4(wi[0], wi[1], wi[2], wi[3]);
        }
    };

    if (MODE == 1) {
        const size_t tail = (flags & ENC_BTAIL) ? (len & ~(size_t)3) : len;
        uint32_t wr[4], wi[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t ar = 0, ai = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int q = 4 * d + b;
                const int vr = std::is_same<R, double>::value ? __double2int_ru((double)yr[q]) : __float2int_ru((float)yr[q]);
                ar |= ((uint32_t)vr & 0xffu) << (8 * b);
                if (CPLX) {
                    int vi = std::is_same<R, double>::value ? __double2int_ru((double)yi[q]) : __float2int_ru((float)yi[q]);
                    if (kk + q >= tail) vi = 0;
                    // op C: the reference's conjugate extractions carry the imaginary magnitude with the
                    // opposite sign (A rows [qr, qi] / [-qi, qr], B columns [qr; -qi]:
                    // scaling.hpp:2262-2329 with addCol, 1944-2016 without)
                    if (flags & ENC_CONJ) vi = -vi;
                    ai |= ((uint32_t)vi & 0xffu) << (8 * b);
                }
            }
            wr[d] = ar;
            wi[d] = ai;
        }
        emit(out, wr, wi, wi);
        return;
    }

    // Karatsuba sum plane from the two slices as stored (int8), whatever their representatives
    // (the f32 path's mod_8i<float> steps are not always the symmetric residue above N = 10)
    auto sum_words = [&](const int (&rr)[16], const int (&ri)[16], int p, uint32_t (&ws)[4]) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t a = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int s = ((int)(int8_t)rr[4 * d + b] + (int)(int8_t)ri[4 * d + b]) % p;  // (-p, p)
                a |= ((uint32_t)center_sum(s, 0, p) & 0xffu) << (8 * b);
            }
            ws[d] = a;
        }
    };

    // one plane: residues of the 16 elements from their f32 reductions t modulo P (one step of
    // the tail of mod_8i, scaling.hpp:218-222, on packed pairs) -> bytes -> emit
    auto plane_from = [&]<int STEPS>(unsigned j, const float (&tr)[16], const float (&tim)[16]) {
        const int p = MP.p[j];
        const float rf = MP.rinv_f[j];
        const float pf = -(float)p;
        int rr[16], ri[16];
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
            const f2v a = STEPS == 1 ? mod8_step_x2(f2v{tr[q], tr[q + 1]}, rf, pf) : mod8_tail_x2(f2v{tr[q], tr[q + 1]}, rf, pf);
            rr[q] = (int)a.x;
            rr[q + 1] = (int)a.y;
            if (CPLX) {
                const f2v b = STEPS == 1 ? mod8_step_x2(f2v{tim[q], tim[q + 1]}, rf, pf) : mod8_tail_x2(f2v{tim[q], tim[q + 1]}, rf, pf);
                ri[q] = (int)b.x;
                ri[q + 1] = (int)b.y;
            } else {
                ri[q] = ri[q + 1] = 0;
            }
        }
        if (OZ2_ENC_ABLATE == 1) {  // probe builds only: no residue arithmetic
#pragma unroll
            for (int q = 0; q < 16; ++q) rr[q] = (int)tr[q] + p;
        }
        uint32_t wr[4], wi[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t ar = 0, ai = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                ar |= ((uint32_t)rr[4 * d + b] & 0xffu) << (8 * b);
                ai |= ((uint32_t)ri[4 * d + b] & 0xffu) << (8 * b);
            }
            wr[d] = ar;
            wi[d] = ai;
        }
        uint32_t ws[4] = {0, 0, 0, 0};
        if (kara) sum_words(rr, ri, p, ws);
        emit(out + (size_t)j * plane, wr, wi, ws);
    };

    // Pair form (one f32 step per modulus) straight to bytes.  With C = 1.5*2^23 and tc = t + C
    // (exact, |t| < 2^22): y' = fma(t, fl(1/p), C) rounds t*fl(1/p) to an integer once (values in
    // [2^23, 2^24) have ulp 1), and fma(y' - C, -p, tc) = C + (t - rint(t/p)*p) exactly, whose bit
    // pattern carries the residue in its low byte (two's complement, as the int8 cast of mod_8i
    // stores it).  Three packed ops per pair and three byte permutes per four bytes replace the
    // multiply / round / fma, the f32 -> i32 conversion and the shift-or packing.
    // Karatsuba: the sum plane from ts = tr + ti (exact, |ts| <= P < 2^16, so the same one step is exact)
    auto plane_bytes = [&](unsigned j, const float (&tr)[16], const float (&trc)[16], const float (&ti)[16],
                           const float (&tic)[16], const float (&ts)[16], const float (&tsc)[16]) {
        const float rf = MP.rinv_f[j];
        const f2v C2 = {12582912.0f, 12582912.0f}, r2 = {rf, rf}, q2 = {-(float)MP.p[j], -(float)MP.p[j]};
        uint32_t ws[4] = {0, 0, 0, 0};
        if (kara) {
            uint32_t bs[16];
#pragma unroll
            for (int q = 0; q < 16; q += 2) {
                const f2v y = __builtin_elementwise_fma(f2v{ts[q], ts[q + 1]}, r2, C2) - C2;
                const f2v a = __builtin_elementwise_fma(y, q2, f2v{tsc[q], tsc[q + 1]});
                bs[q] = __float_as_uint(a.x);
                bs[q + 1] = __float_as_uint(a.y);
            }
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const uint32_t lo = __builtin_amdgcn_perm(bs[4 * d + 1], bs[4 * d], 0x0c0c0400u);
                const uint32_t hi = __builtin_amdgcn_perm(bs[4 * d + 3], bs[4 * d + 2], 0x0c0c0400u);
                ws[d] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
            }
        }
        uint32_t br[16], bi[16];
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
            f2v y = __builtin_elementwise_fma(f2v{tr[q], tr[q + 1]}, r2, C2) - C2;
            const f2v a = __builtin_elementwise_fma(y, q2, f2v{trc[q], trc[q + 1]});
            br[q] = __float_as_uint(a.x);
            br[q + 1] = __float_as_uint(a.y);
            if (CPLX) {
                y = __builtin_elementwise_fma(f2v{ti[q], ti[q + 1]}, r2, C2) - C2;
                const f2v b = __builtin_elementwise_fma(y, q2, f2v{tic[q], tic[q + 1]});
                bi[q] = __float_as_uint(b.x);
                bi[q + 1] = __float_as_uint(b.y);
            }
        }
        uint32_t wr[4], wi[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            // low bytes of four words -> one word (v_perm_b32: selectors 0-3 pick the second source)
            const uint32_t lo = __builtin_amdgcn_perm(br[4 * d + 1], br[4 * d], 0x0c0c0400u);
            const uint32_t hi = __builtin_amdgcn_perm(br[4 * d + 3], br[4 * d + 2], 0x0c0c0400u);
            wr[d] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
            if (CPLX) {
                const uint32_t l2 = __builtin_amdgcn_perm(bi[4 * d + 1], bi[4 * d], 0x0c0c0400u);
                const uint32_t h2 = __builtin_amdgcn_perm(bi[4 * d + 3], bi[4 * d + 2], 0x0c0c0400u);
                wi[d] = __builtin_amdgcn_perm(h2, l2, 0x05040100u);
            } else {
                wi[d] = 0;
            }
        }
        emit(out + (size_t)j * plane, wr, wi, ws);
    };

    // integer-valued f64 values -> group reductions -> planes
    auto residues_f64 = [&](const double (&dr)[16], const double (&di)[16]) {
        for (int gi = 0; gi < G.ng; ++gi) {
            const double P = G.P[gi], rP = G.rP[gi];
            float tr[16], tim[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                tr[q] = __double2float_rn(__builtin_fma(__builtin_rint(dr[q] * rP), -P, dr[q]));
                tim[q] = CPLX ? __double2float_rn(__builtin_fma(__builtin_rint(di[q] * rP), -P, di[q])) : 0.0f;
            }
            if (G.steps == 1 && G.bytes && OZ2_ENC_ABLATE == 0) {
                float trc[16], tic[16], ts[16], tsc[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    trc[q] = tr[q] + 12582912.0f;
                    tic[q] = tim[q] + 12582912.0f;
                    ts[q] = kara ? tr[q] + tim[q] : 0.0f;
                    tsc[q] = ts[q] + 12582912.0f;
                }
                for (int j = G.start[gi]; j < G.start[gi + 1]; ++j) plane_bytes((unsigned)j, tr, trc, tim, tic, ts, tsc);
            } else if (G.steps == 1) {
                for (int j = G.start[gi]; j < G.start[gi + 1]; ++j) plane_from.template operator()<1>((unsigned)j, tr, tim);
            } else {
                for (int j = G.start[gi]; j < G.start[gi + 1]; ++j) plane_from.template operator()<2>((unsigned)j, tr, tim);
            }
        }
    };

    // f32 operands, any N: mod_8i's four f32 steps per modulus (scaling.hpp:225-230)
    auto f32_steps = [&]() {
        for (unsigned j = 0; j < MP.N; ++j) {
            const int p = MP.p[j];
            const float rf = MP.rinv_f[j];
            int rr[16], ri[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                rr[q] = mod8_f32((float)yr[q], p, rf);
                ri[q] = CPLX ? mod8_f32((float)yi[q], p, rf) : 0;
            }
            uint32_t wr[4], wi[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                uint32_t ar = 0, ai = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    ar |= ((uint32_t)rr[4 * d + b] & 0xffu) << (8 * b);
                    ai |= ((uint32_t)ri[4 * d + b] & 0xffu) << (8 * b);
                }
                wr[d] = ar;
                wi[d] = ai;
            }
            uint32_t ws[4] = {0, 0, 0, 0};
            if (kara) sum_words(rr, ri, p, ws);
            emit(out + (size_t)j * plane, wr, wi, ws);
        }
    };

    if constexpr (std::is_same<R, double>::value) {
        residues_f64(yr, yi);
    } else if constexpr (MODE == 2) {
        f32_steps();
    } else if (G.f32_exact) {
        // f32 operands whose residues mod_8i<float> computes exactly (G.f32_exact): the same
        // residues through the f64 group form, a fraction of the f32 work
        double dr[16], di[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            dr[q] = (double)yr[q];
            di[q] = CPLX ? (double)yi[q] : 0.0;
        }
        residues_f64(dr, di);
    } else {
        f32_steps();
    }
}

// 64 k x 64 vectors (real) or 32 k x 64 vectors x re/im (complex), rows padded by one element.  OZ2_ENC_SWZ=1 (A/B
// builds): the real tile unpadded with the vector index XORed by the k index (32 KiB: five blocks per CU instead
// of four); same bits and the same time (cfg2 split 0.694 / 0.695 ms, profiles/r06/enc_swizzle_ab.txt)
#ifndef OZ2_ENC_SWZ
#define OZ2_ENC_SWZ 0
#endif
template <typename R, bool CPLX>
using EncTile = R[CPLX ? 32 : 64][CPLX || !OZ2_ENC_SWZ ? 65 : 64][CPLX ? 2 : 1];
template <bool CPLX> __device__ __forceinline__ int etx(int el, int vl) { return CPLX || !OZ2_ENC_SWZ ? vl : vl ^ el; }

// Accurate mode, real operands, one stream: the final shifts computed by the encode itself from sft0 and the bound
// maxima (finalize_accurate_sft_kernel's arithmetic), stored by the blocks of the first k-tile
struct AccShift {
    const int16_t *sft0;
    const int32_t *bound;
    int16_t *out;
    float log2M;
};
__device__ __forceinline__ int16_t accurate_sft(int16_t sft0, int32_t amax, float log2M) {
    const int s = sft0_stored(sft0) + __float2int_rd(__fmaf_rd(-0.51F, __log2f(__int2float_rn(amax)), log2M));
    return (int16_t)(-s);
}
template <typename R, bool CPLX, bool CONTIG, bool IS_A, int MODE, bool NTL = false, bool ACC = false>
__device__ __forceinline__ void encode_body(const R *__restrict__ X, size_t ld, size_t nvec, size_t len,
                                            const int16_t *__restrict__ sft, int8_t *__restrict__ out, size_t plane,
                                            size_t ksteps, size_t kblk, size_t vmax, int flags, const ModParams &MP,
                                            const ModGroups &G, unsigned bx, unsigned by, EncTile<R, CPLX> &tile,
                                            const AccShift *acc = nullptr) {
    constexpr int KT = CPLX ? 32 : 64;
    constexpr int NT = CPLX ? 128 : 256;
    constexpr int NC = CPLX ? 2 : 1;
    // contiguous vectors: blockIdx.x walks k so that co-running blocks read neighbouring 512-B
    // pieces of the same vectors (walking the vectors instead puts every co-running block at
    // the same offset modulo the vector stride, i.e. on the same HBM channels)
    const bool kfirst = CONTIG && (flags & ENC_KFIRST);
    const size_t v0 = (size_t)(kfirst ? by : bx) * 64;
    const size_t e0 = (size_t)(kfirst ? bx : by) * KT;
    const int tid = threadIdx.x;

    // this thread's vector's shift, loaded with the tile (after the barrier it cost one more memory round trip)
    const size_t vs = v0 + (tid & 63);
    int16_t sraw = 0;
    if constexpr (ACC) {
        if (vs < nvec) {
            sraw = accurate_sft(acc->sft0[vs], acc->bound[vs], acc->log2M);
            if (e0 == 0 && tid < 64) acc->out[vs] = sraw;
        }
    } else {
        sraw = vs < nvec ? sft[vs] : int16_t(0);
    }
    // stage the tile, coalesced along whichever index is contiguous in HBM; interior tiles
    // load without per-element guards so all loads are in flight at once
    constexpr int NL = (64 * KT) / NT;
    const bool interior = v0 + 64 <= nvec && e0 + KT <= len;
    R lre[NL], lim[NL];
    if (OZ2_ENC_ABLATE == 2) {  // probe builds only: no loads
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            lre[i] = (R)(tid * 37 + i * 1.25 + v0);
            lim[i] = 0;
        }
    } else if (interior) {  // block-uniform branch: one batch of unguarded loads
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            const int idx = tid + NT * i;
            int vl, el;
            if (CONTIG) { el = idx % KT; vl = idx / KT; } else { vl = idx & 63; el = idx >> 6; }
            const size_t v = v0 + vl, e = e0 + el;
            load_elem<R, CPLX, NTL>(X, CONTIG ? v * ld + e : e * ld + v, lre[i], lim[i]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            const int idx = tid + NT * i;
            int vl, el;
            if (CONTIG) { el = idx % KT; vl = idx / KT; } else { vl = idx & 63; el = idx >> 6; }
            const size_t v = v0 + vl, e = e0 + el;
            lre[i] = 0;
            lim[i] = 0;
            if (v < nvec && e < len) load_elem<R, CPLX, NTL>(X, CONTIG ? v * ld + e : e * ld + v, lre[i], lim[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const int idx = tid + NT * i;
        int vl, el;
        if (CONTIG) { el = idx % KT; vl = idx / KT; } else { vl = idx & 63; el = idx >> 6; }
        tile[el][etx<CPLX>(el, vl)][0] = lre[i];
        if (CPLX) tile[el][etx<CPLX>(el, vl)][NC - 1] = (flags & ENC_CONJ) ? -lim[i] : lim[i];
    }
    __syncthreads();

    const int vl = tid & 63, c = tid >> 6;  // c-th 16-element chunk of the tile
    const size_t v = v0 + vl;
    const size_t kk = e0 + 16 * c;
    int s = 0;
    if (v < nvec) s = MODE != 1 ? -(int)sraw : sft0_scale<R>(sraw);

    R yr[16], yi[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        R re = tile[16 * c + q][etx<CPLX>(16 * c + q, vl)][0];
        R im = CPLX ? tile[16 * c + q][etx<CPLX>(16 * c + q, vl)][NC - 1] : R(0);
        if (MODE != 1) {
            yr[q] = trunc(scalbn(re, s));
            yi[q] = trunc(scalbn(im, s));
        } else {
            yr[q] = scalbn(fabs(re), s);
            yi[q] = scalbn(fabs(im), s);
        }
    }

    encode_vec16<R, CPLX, IS_A, MODE>(yr, yi, v, kk, nvec, len, out, plane, ksteps, kblk, vmax, flags, MP, G);
}

template <typename R, bool CPLX, bool CONTIG, bool IS_A, int MODE, bool NTL>
__global__ __launch_bounds__(CPLX ? 128 : 256) void encode_kernel(const R *__restrict__ X, size_t ld, size_t nvec,
                                                                   size_t len, const int16_t *__restrict__ sft,
                                                                   int8_t *__restrict__ out, size_t plane,
                                                                   size_t ksteps, size_t kblk, size_t vmax,
                                                                   int flags, ModParams MP, ModGroups G) {
    __shared__ EncTile<R, CPLX> tile;
    if (MP.zero_queue && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 8) MP.zero_queue[threadIdx.x] = 0;
    encode_body<R, CPLX, CONTIG, IS_A, MODE, NTL>(X, ld, nvec, len, sft, out, plane, ksteps, kblk, vmax, flags, MP, G,
                                             blockIdx.x, blockIdx.y, tile);
}

// ------------------------------------------------------------------
// Accurate mode, real operands: sft0 and the 6-bit magnitudes in ONE read of the operand.
// The reference (scaling.hpp:1897-1941, 2215-2260) scales every element of a vector by 2^sft0,
// sft0 = 5 - ilogb(amax of the vector), so it needs the amax before the first magnitude and reads the
// vector twice.  Pass 1 (mag_tile_kernel) stages the encode's 64-vector x 64-element tiles and scales each
// vector's 64 elements of a tile by the TILE's amax instead: m_t = ceil(|x| 2^(5 - e_t)), e_t = ilogb(tile
// amax) <= e_v = ilogb(vector amax), recording e_t and the least exponent e_min of the tile's nonzero
// elements per (tile, vector).  For real x > 0 and an integer d >= 0, ceil(ceil(x) / 2^d) = ceil(x / 2^d), so
// pass 2 (mag_fixup_kernel) turns m_t into the reference's byte with integer arithmetic,
// (m_t + 2^d - 1) >> d with d = e_v - e_t (d >= 7: m_t > 0, as m_t <= 64), provided the reference's scaled
// values are exact: no element of the tile is subnormal under the final scale (e_min + 5 - e_v >= the least
// normal exponent).  Tiles where that fails (a dynamic range beyond ~2^1000 (f64) / 2^120 (f32) inside one
// vector, an infinite vector amax) and tiles holding a NaN are recomputed by pass 2 from the operand with the
// final shift, exactly as encode_vec16's MODE 1.  Pass 2 reads and writes the magnitude plane (1 byte per
// element) instead of re-reading the operand (8 or 4 bytes per element) and writes sft0 -- the same sft0 and
// bytes as split_stats(accurate) + split_encode(MODE 1) (tests/test_gpu_parity.py, accurate cases).
// tinfo codes: e_t = INT_MIN for a tile whose amax is 0; e_min = INT_MAX without a nonzero finite element,
// INT_MIN with a NaN.
constexpr int TI_ZERO = INT_MIN, TI_NAN = INT_MIN, TI_NONE = INT_MAX;

// sft0_of(vector amax) from e_v = ilogb(amax) = max over the tiles of ilogb(tile amax)
template <typename R> __device__ __forceinline__ int16_t sft0_of_exp(int ev) {
    return ev == TI_ZERO ? sft0_of<R>(R(0)) : ev == INT_MAX ? SFT0_INF : (int16_t)(5 - ev);
}

template <typename R> __device__ __forceinline__ int mag_byte(R y) {
    return std::is_same<R, double>::value ? __double2int_ru((double)y) : __float2int_ru((float)y);
}

template <typename R, bool CONTIG, bool NTL>
__device__ __forceinline__ void mag_tile_body(const R *__restrict__ X, size_t ld, size_t nvec, size_t len,
                                              int8_t *__restrict__ out, size_t ksteps, int2 *__restrict__ tinfo,
                                              size_t tstride, int flags, unsigned bx, unsigned by,
                                              EncTile<R, false> &tile) {
    const bool kfirst = CONTIG && (flags & ENC_KFIRST);
    const size_t kt = kfirst ? bx : by;
    const size_t v0 = (size_t)(kfirst ? by : bx) * 64, e0 = kt * 64;
    const int tid = threadIdx.x;
    constexpr int NL = 16;  // 64 x 64 / 256
    const bool interior = v0 + 64 <= nvec && e0 + 64 <= len;
    R lre[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const int idx = tid + 256 * i;
        const int el = CONTIG ? idx % 64 : idx >> 6, vl = CONTIG ? idx / 64 : idx & 63;
        const size_t v = v0 + vl, e = e0 + el;
        R im;
        lre[i] = 0;
        if (interior || (v < nvec && e < len)) load_elem<R, false, NTL>(X, CONTIG ? v * ld + e : e * ld + v, lre[i], im);
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const int idx = tid + 256 * i;
        const int el = CONTIG ? idx % 64 : idx >> 6, vl = CONTIG ? idx / 64 : idx & 63;
        tile[el][etx<false>(el, vl)][0] = lre[i];
    }
    __syncthreads();
    // the 4 lanes of a vector's tile row are neighbours in one wave (c-th 16-element chunk): its tile
    // amax / least nonzero / NaN flag by two lane exchanges, no second block barrier
    const int vl = tid >> 2, c = tid & 3;
    R x[16], mx = 0, mn = R(INFINITY);
    int nan = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        x[q] = fabs(tile[16 * c + q][etx<false>(16 * c + q, vl)][0]);
        mx = fmax(mx, x[q]);  // NaN ignored, as the stats pass's amax
        if (x[q] != R(0) && x[q] < mn) mn = x[q];
        nan |= __builtin_isnan(x[q]) ? 1 : 0;
    }
#pragma unroll
    for (int sh = 1; sh <= 2; sh <<= 1) {
        mx = fmax(mx, __shfl_xor(mx, sh));
        mn = fmin(mn, __shfl_xor(mn, sh));
        nan |= __shfl_xor(nan, sh);
    }
    const R amax = mx, amin = mn;
    const bool anan = nan != 0;
    // the tile's scale: sft0_scale of sft0_of(tile amax) (for an Inf amax 5 - ilogb(Inf), the reference's int)
    const int s = amax == R(0) ? 0 : 5 - ilogb_r<R>(amax);
    uint32_t w[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t a = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) a |= ((uint32_t)mag_byte<R>(scalbn(x[4 * d + b], s)) & 0xffu) << (8 * b);
        w[d] = a;
    }
    const size_t v = v0 + vl;
    *reinterpret_cast<uint4 *>(out + panel_offset(v, e0 + 16 * c, ksteps)) = make_uint4(w[0], w[1], w[2], w[3]);
    if (c == 0 && v < tstride) {
        const int et = amax == R(0) ? TI_ZERO : __builtin_isinf(amax) ? INT_MAX : ilogb_r<R>(amax);
        const int em = anan ? TI_NAN : amin == R(INFINITY) ? TI_NONE : ilogb_r<R>(amin);
        tinfo[kt * tstride + v] = make_int2(et, em);
    }
}
template <typename R, bool CONTIG, bool NTL>
__global__ __launch_bounds__(256) void mag_tile_kernel(const R *__restrict__ X, size_t ld, size_t nvec, size_t len,
                                                        int8_t *__restrict__ out, size_t ksteps,
                                                        int2 *__restrict__ tinfo, size_t tstride, int flags) {
    __shared__ EncTile<R, false> tile;
    mag_tile_body<R, CONTIG, NTL>(X, ld, nvec, len, out, ksteps, tinfo, tstride, flags, blockIdx.x, blockIdx.y, tile);
}

// the vector exponent e_v = max over its tiles of e_t (= ilogb of the vector amax) and sft0 = sft0_of(amax):
// 64 vectors x 4 tile slices per block
template <typename R>
__global__ __launch_bounds__(256) void mag_vexp_kernel(size_t nvec, size_t ktiles, const int2 *__restrict__ tinfo,
                                                        size_t tstride, int *__restrict__ vexp,
                                                        int16_t *__restrict__ sft0_out) {
    __shared__ int part[4][64];
    const int vl = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const size_t v = (size_t)blockIdx.x * 64 + vl;
    int ev = INT_MIN;
    if (v < nvec) {
        constexpr int U = 8;  // loads in flight per thread
        size_t t = sl;
        for (; t + 4 * (U - 1) < ktiles; t += 4 * U) {
            int e[U];
#pragma unroll
            for (int u = 0; u < U; ++u) e[u] = tinfo[(t + 4 * u) * tstride + v].x;
#pragma unroll
            for (int u = 0; u < U; ++u) ev = max(ev, e[u]);
        }
        for (; t < ktiles; t += 4) ev = max(ev, tinfo[t * tstride + v].x);
    }
    part[sl][vl] = ev;
    __syncthreads();
    if (sl == 0 && v < nvec) {
        ev = max(max(part[0][vl], part[1][vl]), max(part[2][vl], part[3][vl]));
        vexp[v] = ev;
        sft0_out[v] = sft0_of_exp<R>(ev);
    }
}

// one wave per (32 vectors, FIX_T consecutive k-tiles): lane (r, h) handles vector v0 + r and the 16-byte chunk h
// of each 32-element half of a tile, so a wave's chunk accesses are 1 KiB contiguous in the panel layout.  The
// bytes of all FIX_T tiles are loaded before any is rewritten (one wave-tile alone left too few bytes in flight:
// 3.7-3.9 TB/s, profiles/r05/cfg4_single_stream/)
constexpr int FIX_T = 4;
// VEXP: the block finds its vectors' e_v itself (the 8 threads of a vector over every 8th tile, an LDS max;
// blocks of k-tile group 0 store sft0) instead of reading mag_vexp_kernel's: the small-problem pair launch
template <typename R, bool CONTIG, bool VEXP = false>
__device__ __forceinline__ void mag_fixup_body(const R *__restrict__ X, size_t ld, size_t nvec, size_t len,
                                               int8_t *__restrict__ out, size_t ksteps, size_t ktiles,
                                               const int2 *__restrict__ tinfo, size_t tstride,
                                               const int *__restrict__ vexp, int16_t *__restrict__ sft0_out,
                                               unsigned bx, unsigned by, int (*part)[32]) {
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const size_t v = (size_t)bx * 32 + r;
    const size_t t0 = ((size_t)by * 4 + (threadIdx.x >> 6)) * FIX_T;
    int ev;
    if constexpr (VEXP) {
        const int q = (threadIdx.x >> 6) * 2 + h;
        int e = INT_MIN;
        if (v < nvec)
            for (size_t t = q; t < ktiles; t += 8) e = max(e, tinfo[t * tstride + v].x);
        part[q][r] = e;
        __syncthreads();
        ev = part[0][r];
#pragma unroll
        for (int i = 1; i < 8; ++i) ev = max(ev, part[i][r]);
        if (by == 0 && threadIdx.x < 32 && v < nvec) sft0_out[v] = sft0_of_exp<R>(ev);
    }
    if (v >= nvec || t0 >= ktiles) return;  // padding vectors: pass 1 wrote their zeros
    if constexpr (!VEXP) ev = vexp[v];
    uint4 *p0[FIX_T], *p1[FIX_T];
    uint4 b0[FIX_T], b1[FIX_T];
    int2 ti[FIX_T];
    // the bytes are loaded before they are known to be needed: one memory round trip instead of two (the
    // test on b0.x & b1.x, never all ones as every byte is <= 64, keeps the compiler from sinking the loads
    // below the branches)
#pragma unroll
    for (int i = 0; i < FIX_T; ++i) {
        const size_t t = t0 + i < ktiles ? t0 + i : t0;  // (a tile past the end repeats t0: loaded, never written)
        p0[i] = reinterpret_cast<uint4 *>(out + panel_offset(v, t * 64 + h * 16, ksteps));
        p1[i] = reinterpret_cast<uint4 *>(out + panel_offset(v, t * 64 + 32 + h * 16, ksteps));
        b0[i] = *p0[i];
        b1[i] = *p1[i];
        ti[i] = tinfo[t * tstride + v];
    }
    const int srow = sft0_scale<R>(sft0_of_exp<R>(ev));  // (as mag_vexp_kernel stored it: no third load)
    constexpr long long EMIN = std::is_same<R, double>::value ? -1022 : -126;
#pragma unroll
    for (int i = 0; i < FIX_T; ++i) {
        if (t0 + i >= ktiles) break;
        const bool final_bytes = (ti[i].x == ev && ti[i].y != TI_NAN)          // d = 0 (the vector's own amax tile)
                                 || (ti[i].x == TI_ZERO && ti[i].y == TI_NONE);  // zeros only
        if (final_bytes && (b0[i].x & b1[i].x) != ~0u) continue;
        const bool exact = ti[i].y != TI_NAN && ev != INT_MAX && (ti[i].y == TI_NONE || (long long)ti[i].y + srow >= EMIN);
        if (exact) {
            const int d = min(ev - ti[i].x, 7);  // (m_t <= 64: from d = 7 on every nonzero byte becomes 1)
            const uint32_t add = ((1u << d) - 1u) * 0x01010101u, mask = (0xffu >> d) * 0x01010101u;
            // bytes <= 64: the byte-wise add cannot carry
            *p0[i] = make_uint4(((b0[i].x + add) >> d) & mask, ((b0[i].y + add) >> d) & mask,
                                ((b0[i].z + add) >> d) & mask, ((b0[i].w + add) >> d) & mask);
            *p1[i] = make_uint4(((b1[i].x + add) >> d) & mask, ((b1[i].y + add) >> d) & mask,
                                ((b1[i].z + add) >> d) & mask, ((b1[i].w + add) >> d) & mask);
            continue;
        }
        // the reference's own arithmetic with the final shift (encode_vec16, MODE 1)
        for (int half = 0; half < 2; ++half) {
            const size_t kk = (t0 + i) * 64 + half * 32 + h * 16;
            uint32_t w[4];
#pragma unroll
            for (int dd = 0; dd < 4; ++dd) {
                uint32_t a = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const size_t e = kk + 4 * dd + b;
                    R re = 0, im;
                    if (e < len) load_elem<R, false, false>(X, CONTIG ? v * ld + e : e * ld + v, re, im);
                    a |= ((uint32_t)mag_byte<R>(scalbn(fabs(re), srow)) & 0xffu) << (8 * b);
                }
                w[dd] = a;
            }
            *(half ? p1[i] : p0[i]) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}
template <typename R, bool CONTIG>
__global__ __launch_bounds__(256) void mag_fixup_kernel(const R *__restrict__ X, size_t ld, size_t nvec, size_t len,
                                                         int8_t *__restrict__ out, size_t ksteps, size_t ktiles,
                                                         const int2 *__restrict__ tinfo, size_t tstride,
                                                         const int *__restrict__ vexp) {
    mag_fixup_body<R, CONTIG>(X, ld, nvec, len, out, ksteps, ktiles, tinfo, tstride, vexp, nullptr, blockIdx.x,
                              blockIdx.y, nullptr);
}

// Accurate mode, small problems (one stream): both operands' magnitude passes in two launches instead of six,
// and both finalizations in one instead of two.  MagOperand: one operand's pass-1 / fix-up geometry.
struct MagOperand {
    const void *X;
    size_t ld, nvec, len, tstride, ktiles;
    int8_t *out;
    int2 *tinfo;
    int16_t *sft0;
    int flags;
    unsigned g1x, g1y, g3x, g3y;
};
template <typename R, bool CA, bool CB>
__global__ __launch_bounds__(256) void mag_tile_pair_kernel(MagOperand a, MagOperand b, size_t ksteps) {
    __shared__ EncTile<R, false> tile;
    const unsigned na = a.g1x * a.g1y;
    if (blockIdx.x < na)
        mag_tile_body<R, CA, false>(static_cast<const R *>(a.X), a.ld, a.nvec, a.len, a.out, ksteps, a.tinfo,
                                    a.tstride, a.flags, blockIdx.x % a.g1x, blockIdx.x / a.g1x, tile);
    else {
        const unsigned t = blockIdx.x - na;
        mag_tile_body<R, CB, false>(static_cast<const R *>(b.X), b.ld, b.nvec, b.len, b.out, ksteps, b.tinfo,
                                    b.tstride, b.flags, t % b.g1x, t / b.g1x, tile);
    }
}
// (zeroes the bound maxima too: the bound product that follows accumulates into them with atomicMax)
template <typename R, bool CA, bool CB>
__global__ __launch_bounds__(256) void mag_fixup_pair_kernel(MagOperand a, MagOperand b, size_t ksteps,
                                                              int32_t *__restrict__ bound, size_t nbound) {
    __shared__ int part[8][32];
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nbound; i += (size_t)gridDim.x * 256) bound[i] = 0;
    const unsigned na = a.g3x * a.g3y;
    if (blockIdx.x < na)
        mag_fixup_body<R, CA, true>(static_cast<const R *>(a.X), a.ld, a.nvec, a.len, a.out, ksteps, a.ktiles,
                                    a.tinfo, a.tstride, nullptr, a.sft0, blockIdx.x % a.g3x, blockIdx.x / a.g3x, part);
    else {
        const unsigned t = blockIdx.x - na;
        mag_fixup_body<R, CB, true>(static_cast<const R *>(b.X), b.ld, b.nvec, b.len, b.out, ksteps, b.ktiles,
                                    b.tinfo, b.tstride, nullptr, b.sft0, t % b.g3x, t / b.g3x, part);
    }
}

// Both operands' slices in one launch (small problems, one stream): blocks [0, gx*gy of A) encode A,
// the rest B.  Saves a launch boundary and lets A's and B's tiles share the chip.
struct EncOperand {
    const void *X;
    size_t ld, nvec, len;
    const int16_t *sft;
    int8_t *out;
    size_t plane, vmax;
    int flags;
    unsigned gx, gy;
    AccShift acc;  // ACC launches: where the shifts come from (sft is then unused)
};
template <typename R, bool CPLX, bool CONTIG_A, bool CONTIG_B, bool NTL, bool ACC = false>
__global__ __launch_bounds__(CPLX ? 128 : 256) void encode_pair_kernel(EncOperand a, EncOperand b, size_t ksteps,
                                                                        size_t kblk, ModParams MP, ModGroups G) {
    __shared__ EncTile<R, CPLX> tile;
    const unsigned na = a.gx * a.gy;
    if (MP.zero_queue && blockIdx.x == 0 && threadIdx.x < 8) MP.zero_queue[threadIdx.x] = 0;
    if (blockIdx.x < na) {
        encode_body<R, CPLX, CONTIG_A, true, 0, NTL, ACC>(static_cast<const R *>(a.X), a.ld, a.nvec, a.len, a.sft, a.out,
                                                          a.plane, ksteps, kblk, a.vmax, a.flags, MP, G,
                                                          blockIdx.x % a.gx, blockIdx.x / a.gx, tile, &a.acc);
    } else {
        const unsigned t = blockIdx.x - na;
        encode_body<R, CPLX, CONTIG_B, false, 0, NTL, ACC>(static_cast<const R *>(b.X), b.ld, b.nvec, b.len, b.sft, b.out,
                                                           b.plane, ksteps, kblk, b.vmax, b.flags, MP, G, t % b.gx,
                                                           t / b.gx, tile, &b.acc);
    }
}

// ------------------------------------------------------------------
// Fast mode, small k, one stream: shifts and slices of both operands in ONE launch that reads each operand once.
// A block holds FZ_V = 4 (GEMMUL8_FUSED_V=8: 8) whole vectors (k <= KMAX elements each, f64) in LDS: it loads them
// (coalesced along whichever index is contiguous), sums them in the reference's order -- wave w takes vector w,
// lane l the reference's virtual threads l and l + 64 of VT = 128 (their round-up chains in element order), then
// the tail of stats_strided_body -- and encodes its vectors from the same LDS copy (encode_vec16, MODE 0).  Same
// shifts and bytes as split_stats_pair + split_encode_pair (tests/test_gpu_parity.py), one launch and one
// operand read instead of two each.  Blocks [0, na) take A's vectors, the rest B's.  MAG: accurate mode's first
// pass in the same form (sft0 from the vector amax, the 6-bit magnitudes, MODE 1).
// ------------------------------------------------------------------
// A/B builds (profiles/r06/fused_split/): OZ2_FZ_PAD=1 pads 16 bytes after every 16 elements of the LDS panel
// (the encode's chunks 144 bytes apart), OZ2_FZ_XCD_CONTIG=1 renumbers a contiguous operand's blocks onto one
// XCD as the strided operand's are; both measured slower (1536^3 split 33.5 -> 40.5 us with both)
#ifndef OZ2_FZ_PAD
#define OZ2_FZ_PAD 0
#endif
#ifndef OZ2_FZ_XCD_CONTIG
#define OZ2_FZ_XCD_CONTIG 0
#endif
__device__ __forceinline__ int fz_idx(int e) { return OZ2_FZ_PAD ? e + 2 * (e >> 4) : e; }
template <int KMAX> constexpr int FZ_ROW = KMAX + (OZ2_FZ_PAD ? KMAX / 8 : 0) + 2;
struct FusedOperand {
    const double *X;
    size_t ld, nvec, vpad, plane, vmax;
    int16_t *sft;
    int8_t *out;
};
// MAG: accurate mode's first pass instead -- sft0 = 5 - ilogb(vector amax) and the 6-bit magnitude plane (MODE 1)
// the loads of vectors [v0, v0 + FZ_V) into registers (zeros past len and past nvec): KMAX / 64 per thread
template <int KMAX, int FZ_V, int FZ_NT, bool CONTIG, bool NTL>
__device__ __forceinline__ void fz_load(const FusedOperand &o, size_t len, size_t v0, double (&x)[KMAX / 64]) {
    static_assert(KMAX % 128 == 0 && KMAX % FZ_NT == 0 && FZ_NT == 64 * FZ_V, "whole chains and load rounds");
    const int tid = threadIdx.x;
    if (CONTIG) {
        // vector j's elements e = tid + FZ_NT i: each wave load is 512 contiguous bytes
        constexpr int PER = KMAX / FZ_NT;
#pragma unroll
        for (int j = 0; j < FZ_V; ++j)
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const size_t v = v0 + j, e = tid + (size_t)FZ_NT * i;
                double im;
                x[j * PER + i] = 0.0;
                if (v < o.nvec && e < len) load_elem<double, false, NTL>(o.X, v * o.ld + e, x[j * PER + i], im);
            }
    } else {
        // row r = tid mod FZ_V of column e = tid / FZ_V + 64 i: 8 FZ_V contiguous bytes per column
        constexpr int PER = KMAX / (FZ_NT / FZ_V);
        const int r = tid & (FZ_V - 1), c = tid / FZ_V;
        const size_t v = v0 + r;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const size_t e = c + (size_t)(FZ_NT / FZ_V) * i;
            double im;
            x[i] = 0.0;
            if (v < o.nvec && e < len) load_elem<double, false, NTL>(o.X, e * o.ld + v, x[i], im);
        }
    }
}
template <int KMAX, int FZ_V, int FZ_NT, bool CONTIG>
__device__ __forceinline__ void fz_stage(const double (&x)[KMAX / 64], double (&panel)[FZ_V][FZ_ROW<KMAX>]) {
    const int tid = threadIdx.x;
    if (CONTIG) {
        constexpr int PER = KMAX / FZ_NT;
#pragma unroll
        for (int j = 0; j < FZ_V; ++j)
#pragma unroll
            for (int i = 0; i < PER; ++i) panel[j][fz_idx(tid + FZ_NT * i)] = x[j * PER + i];
    } else {
        constexpr int PER = KMAX / (FZ_NT / FZ_V);
        const int r = tid & (FZ_V - 1), c = tid / FZ_V;
#pragma unroll
        for (int i = 0; i < PER; ++i) panel[r][fz_idx(c + (FZ_NT / FZ_V) * i)] = x[i];
    }
}
// shifts and slices of the staged vectors [v0, v0 + FZ_V) (the panel filled and synchronised); ends with the panel
// still being read (the caller synchronises before restaging it)
template <int KMAX, int FZ_V, int FZ_NT, bool MAG = false>
__device__ __forceinline__ void fz_compute(const FusedOperand &o, bool is_a, size_t len, size_t ksteps, size_t kblk,
                                           float log2M, const ModParams &MP, const ModGroups &G, size_t v0,
                                           double (&panel)[FZ_V][FZ_ROW<KMAX>], int (&shl)[FZ_V]) {
    const int tid = threadIdx.x;
    {
        // wave w < FZ_V: vector v0 + w; lane l: the chains of virtual threads l and l + 64 (elements vt + 128 i, in
        // order)
        const int w = tid >> 6, lane = tid & 63;
        if (MAG && w < FZ_V) {
            double amax = 0;
            for (int i = 0; i < KMAX / 64; ++i) amax = fmax(amax, fabs(panel[w][fz_idx(lane + 64 * i)]));
            const double mx = wave_max<double>(amax);
            const size_t v = v0 + w;
            if (lane == 0) {
                int sh = 0;
                if (v < o.nvec) {
                    const int16_t s0 = sft0_of<double>(mx);
                    o.sft[v] = s0;
                    sh = sft0_scale<double>(s0);
                }
                shl[w] = sh;
            }
        } else if (w < FZ_V) {
            double a0 = 0, a1 = 0, amax = 0;
            static_assert(KMAX % 512 == 0, "chains in groups of four");
            for (int i = 0; i < KMAX / 128; i += 4) {
                double x0[4], x1[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    x0[u] = fabs(panel[w][fz_idx(lane + 128 * (i + u))]);
                    x1[u] = fabs(panel[w][fz_idx(lane + 64 + 128 * (i + u))]);
                    amax = fmax(amax, fmax(x0[u], x1[u]));
                }
                sq_add4x2_ru(x0, x1, a0, a1);
            }
            const double mx = wave_max<double>(amax);
            const double s0 = ref_wave_sum<double>(a0), s1 = ref_wave_sum<double>(a1);
            const double g00 = __shfl(s0, 1), g01 = __shfl(s0, 33), g10 = __shfl(s1, 1), g11 = __shfl(s1, 33);
            double gv = lane == 32 ? g00 : lane == 33 ? g01 : lane == 34 ? g10 : lane == 35 ? g11 : 0.0;
            gv = ref_wave_sum<double>(gv);
            const double nrm = __shfl(gv, 32);
            const size_t v = v0 + w;
            if (lane == 0) {
                int sh = 0;
                if (v < o.nvec) {
                    const int16_t st = (int16_t)(-compute_sft(mx, nrm, log2M));
                    o.sft[v] = st;
                    sh = -(int)st;
                }
                shl[w] = sh;
            }
        }
    }
    __syncthreads();
    // encode: thread (vector tid mod FZ_V, 16-element chunk tid / FZ_V): FZ_V x 16 contiguous panel bytes
    const int r = tid & (FZ_V - 1), c = tid / FZ_V;
    const size_t v = v0 + r;
    const int sh = shl[r];
    for (size_t kk = 16 * (size_t)c; kk < kblk; kk += 16 * (FZ_NT / FZ_V)) {
        double yr[16], yi[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const double x = panel[r][fz_idx((int)kk) + q];
            yr[q] = MAG ? scalbn(fabs(x), sh) : trunc(scalbn(x, sh));
            yi[q] = 0;
        }
        constexpr int MODE = MAG ? 1 : 0;
        if (is_a) encode_vec16<double, false, true, MODE>(yr, yi, v, kk, o.nvec, len, o.out, o.plane, ksteps, kblk, o.vmax, 0, MP, G);
        else encode_vec16<double, false, false, MODE>(yr, yi, v, kk, o.nvec, len, o.out, o.plane, ksteps, kblk, o.vmax, 0, MP, G);
    }
}
// GRP groups of FZ_V vectors per block, software-pipelined: the next group's loads are in flight (registers) while
// the current group is summed and encoded from LDS
template <int KMAX, int FZ_V, int FZ_NT, bool CONTIG, bool NTL, bool MAG, int GRP>
__device__ __forceinline__ void fused_body(const FusedOperand &o, bool is_a, size_t len, size_t ksteps, size_t kblk,
                                           float log2M, const ModParams &MP, const ModGroups &G, unsigned bx,
                                           double (&panel)[FZ_V][FZ_ROW<KMAX>], int (&shl)[FZ_V]) {
    double x[KMAX / 64];
    const size_t vb = (size_t)bx * FZ_V * GRP;
    fz_load<KMAX, FZ_V, FZ_NT, CONTIG, NTL>(o, len, vb, x);
    fz_stage<KMAX, FZ_V, FZ_NT, CONTIG>(x, panel);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < GRP; ++t) {
        if (t + 1 < GRP) fz_load<KMAX, FZ_V, FZ_NT, CONTIG, NTL>(o, len, vb + (size_t)(t + 1) * FZ_V, x);
        fz_compute<KMAX, FZ_V, FZ_NT, MAG>(o, is_a, len, ksteps, kblk, log2M, MP, G, vb + (size_t)t * FZ_V, panel, shl);
        if (t + 1 < GRP) {
            __syncthreads();
            fz_stage<KMAX, FZ_V, FZ_NT, CONTIG>(x, panel);
            __syncthreads();
        }
    }
}
template <int KMAX, int FZ_V, int FZ_NT, bool CA, bool CB, bool NTL = false, bool MAG = false, int GRP = 1>
__global__ __launch_bounds__(FZ_NT) void split_fused_kernel(FusedOperand a, FusedOperand b, size_t len,
                                                            size_t ksteps, size_t kblk, float log2M, ModParams MP,
                                                            ModGroups G, int32_t *zero, size_t nzero) {
    __shared__ double panel[FZ_V][FZ_ROW<KMAX>];
    __shared__ int shl[FZ_V];
    if (MP.zero_queue && blockIdx.x == 0 && threadIdx.x < 8) MP.zero_queue[threadIdx.x] = 0;
    // (MAG: the bound maxima the bound product accumulates into with atomicMax)
    for (size_t i = (size_t)blockIdx.x * FZ_NT + threadIdx.x; i < nzero; i += (size_t)gridDim.x * FZ_NT) zero[i] = 0;
    const unsigned na = (unsigned)(a.vpad / (FZ_V * GRP)), nb = (unsigned)(b.vpad / (FZ_V * GRP));
    // (a strided operand's neighbouring blocks, which share its 128-byte input lines, are renumbered onto one XCD)
    if (blockIdx.x < na) {
        const unsigned bx = CA && !OZ2_FZ_XCD_CONTIG ? blockIdx.x : xcd_local_block(blockIdx.x, na);
        fused_body<KMAX, FZ_V, FZ_NT, CA, NTL, MAG, GRP>(a, true, len, ksteps, kblk, log2M, MP, G, bx, panel, shl);
    } else {
        const unsigned t = blockIdx.x - na;
        const unsigned bx = CB && !OZ2_FZ_XCD_CONTIG ? t : xcd_local_block(t, nb);
        fused_body<KMAX, FZ_V, FZ_NT, CB, NTL, MAG, GRP>(b, false, len, ksteps, kblk, log2M, MP, G, bx, panel, shl);
    }
}

// accurate mode: sft = sft0 + floor_rd(-0.51*log2(amax) + log2M)  (int8tc::compute_sft, scaling.hpp:1504-1506)
__global__ void finalize_accurate_sft_kernel(const int16_t *__restrict__ sft0, const int32_t *__restrict__ bound,
                                             size_t nvec, float log2M, int16_t *__restrict__ sft_out, int cplx_rows) {
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nvec) return;
    const int amax = cplx_rows ? max(bound[v], bound[v + nvec]) : bound[v];
    sft_out[v] = accurate_sft(sft0[v], amax, log2M);
}

// both operands: vectors [0, nA) of A (sft0A, boundA), then [0, nB) of B
__global__ void finalize_accurate_pair_kernel(const int16_t *__restrict__ sft0A, const int32_t *__restrict__ boundA,
                                              size_t nA, const int16_t *__restrict__ sft0B,
                                              const int32_t *__restrict__ boundB, size_t nB, float log2M,
                                              int16_t *__restrict__ outA, int16_t *__restrict__ outB) {
    size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool isA = v < nA;
    if (!isA) v -= nA;
    if (!isA && v >= nB) return;
    (isA ? outA : outB)[v] = accurate_sft((isA ? sft0A : sft0B)[v], (isA ? boundA : boundB)[v], log2M);
}

// zeroes the accurate-mode bound maxima before the bound product (a kernel rather than
// hipMemsetAsync: a memset captured into a HIP graph did not run on replay -- the replayed
// atomicMax then kept the previous call's maxima, tests/test_gpu_streams.py)
__global__ void zero_i32_kernel(int32_t *__restrict__ p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 0;
}
void zero_i32(int32_t *p, size_t n, hipStream_t st) {
    if (n == 0) return;
    const size_t blocks = (n + 255) / 256;
    launch(zero_i32_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), st, p, n);
}

// ------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------
// rows per block of the strided pass: enough blocks to give every CU several (m/16 < 2 per CU leaves
// the chip latency-bound); GEMMUL8_STATS_ROWS overrides (probe / A-B runs)
static int stats_rows(size_t nvec) {
    static const int forced = [] {
        const char *e = getenv("GEMMUL8_STATS_ROWS");
        const int r = e ? atoi(e) : 0;
        return (r == 4 || r == 8 || r == 16) ? r : 0;
    }();
    return forced ? forced : nvec >= 4096 ? 16 : nvec >= 2048 ? 8 : 4;
}

// non-temporal operand loads from this many operand bytes (see load_elem)
constexpr size_t NT_OPERAND_BYTES = size_t(1) << 27;

template <typename R, bool CPLX>
static void launch_stats(const void *X, size_t ld, bool contig, size_t len, size_t nvec, int VT, bool accurate,
                         float log2M, int16_t *out, hipStream_t st) {
    const R *x = static_cast<const R *>(X);
    const bool nt = nvec * len * sizeof(R) * (CPLX ? 2 : 1) >= NT_OPERAND_BYTES;
    if (contig) {
#define OZ2_SC(vt, ac) do { if (nt) launch(stats_contig_kernel<R, CPLX, vt, ac, true>, dim3((unsigned)nvec), dim3(vt), st, x, ld, len, nvec, log2M, out); \
                            else launch(stats_contig_kernel<R, CPLX, vt, ac, false>, dim3((unsigned)nvec), dim3(vt), st, x, ld, len, nvec, log2M, out); } while (0)
        if (VT == 512) { if (accurate) OZ2_SC(512, true); else OZ2_SC(512, false); }
        else { if (accurate) OZ2_SC(128, true); else OZ2_SC(128, false); }
#undef OZ2_SC
    } else {
        const int rows = stats_rows(nvec);
        const unsigned g = (unsigned)((nvec + rows - 1) / rows);
#define OZ2_SS(vt, ac, rw, n) launch(stats_strided_kernel<R, CPLX, vt, ac, rw, n>, dim3(g), dim3(256), st, x, ld, len, nvec, log2M, out)
        // (operands of NT size always take 16-row blocks: stats_rows gives 16 from 4096 vectors)
#define OZ2_SSR(vt, ac) do { if (rows == 16) { if (nt) OZ2_SS(vt, ac, 16, true); else OZ2_SS(vt, ac, 16, false); } \
                             else if (rows == 8) OZ2_SS(vt, ac, 8, false); else OZ2_SS(vt, ac, 4, false); } while (0)
        if (VT == 512) { if (accurate) OZ2_SSR(512, true); else OZ2_SSR(512, false); }
        else { if (accurate) OZ2_SSR(128, true); else OZ2_SSR(128, false); }
#undef OZ2_SSR
#undef OZ2_SS
    }
}

template <typename R, bool CPLX, bool IS_A>
static void launch_encode(const void *X, size_t ld, bool contig, size_t nvec, size_t len, const int16_t *sft,
                          int8_t *out, size_t plane, const Layout &L, size_t vpad_grid, size_t vmax, int mode,
                          int flags, const ModParams &MP, hipStream_t st) {
    constexpr int KT = CPLX ? 32 : 64;
    constexpr int NT = CPLX ? 128 : 256;
    if (L.kblk == 0 || vpad_grid == 0) return;  // k = 0: the slice planes are empty
    const R *x = static_cast<const R *>(X);
    // k-first block order for contiguous vectors (-4.5 % on B, see encode_body), unless the vector tiles
    // would exceed the grid's reported y limit (hipDeviceAttributeMaxGridDimY = 65536: more than 4 Mi
    // vectors; a 65540-tile launch still ran on MI355X, but nothing documents more); the k-tiles never do
    // (k <= 2^22)
    const bool kf = contig && vpad_grid / 64 <= 65536;
    if (kf) flags |= ENC_KFIRST;
    const dim3 grid = kf ? dim3((unsigned)(L.kblk / KT), (unsigned)(vpad_grid / 64))
                         : dim3((unsigned)(vpad_grid / 64), (unsigned)(L.kblk / KT));
    const ModGroups G = make_groups(MP, L.N);  // grouping by the call's N (magnitude bound), not the sub-range
    const bool nt = nvec * len * sizeof(R) * (CPLX ? 2 : 1) >= NT_OPERAND_BYTES;
// MODE 2 exists for f32 operands only
#define OZ2_EN_F32(cg) do { if constexpr (std::is_same<R, float>::value) OZ2_EN(cg, 2); } while (0)
#define OZ2_EN(cg, md) do { if (nt) launch(encode_kernel<R, CPLX, cg, IS_A, md, true>, grid, dim3(NT), st, x, ld, nvec, len, sft, out, plane, L.ksteps, L.kblk, vmax, flags, MP, G); \
                            else launch(encode_kernel<R, CPLX, cg, IS_A, md, false>, grid, dim3(NT), st, x, ld, nvec, len, sft, out, plane, L.ksteps, L.kblk, vmax, flags, MP, G); } while (0)
    if constexpr (std::is_same<R, float>::value) {
        if (mode == 0 && !G.f32_exact) mode = 2;
    }
    if (contig) { if (mode == 0) OZ2_EN(true, 0); else if (mode == 1) OZ2_EN(true, 1); else OZ2_EN_F32(true); }
    else { if (mode == 0) OZ2_EN(false, 0); else if (mode == 1) OZ2_EN(false, 1); else OZ2_EN_F32(false); }
#undef OZ2_EN_F32
#undef OZ2_EN
}

void split_stats(const OperandDesc &d, size_t len, size_t nvec, int VT, bool accurate, float log2M, int16_t *out,
                 hipStream_t st) {
    if (d.dbl) {
        if (d.cplx) launch_stats<double, true>(d.ptr, d.ld, d.contig, len, nvec, VT, accurate, log2M, out, st);
        else launch_stats<double, false>(d.ptr, d.ld, d.contig, len, nvec, VT, accurate, log2M, out, st);
    } else {
        if (d.cplx) launch_stats<float, true>(d.ptr, d.ld, d.contig, len, nvec, VT, accurate, log2M, out, st);
        else launch_stats<float, false>(d.ptr, d.ld, d.contig, len, nvec, VT, accurate, log2M, out, st);
    }
}

void split_encode(const OperandDesc &d, bool is_A, size_t nvec, size_t len, const int16_t *sft, int8_t *out,
                  size_t plane, const Layout &L, int mode, const ModParams &MP, hipStream_t st, bool btail_quirk) {
    const bool kara = L.kara && mode == 0;  // (the accurate-mode bound is encoded as the big matrix)
    const int flags = (d.conj ? ENC_CONJ : 0) | (btail_quirk && mode == 1 && !is_A ? ENC_BTAIL : 0) |
                      (kara ? ENC_KARA : 0);
    // grid extent over vectors: padded rows/cols get zero slices; complex A covers
    // [0, m_pad - m) so that rows [2m, m_pad) are zeroed through their bottom copy; Karatsuba
    // covers one sub-block, each vector emitting its three copies (vmax = the sub-block stride)
    size_t vpad = kara ? (is_A ? L.vsA : L.vsB) : is_A ? (d.cplx ? L.m_pad - L.m : L.m_pad) : L.n_pad;
    vpad = round_up(vpad, 64);
    const size_t vmax = kara ? (is_A ? L.vsA : L.vsB) : is_A ? L.m_pad : L.n_pad;
#define OZ2_LE(R, C, A) launch_encode<R, C, A>(d.ptr, d.ld, d.contig, nvec, len, sft, out, plane, L, vpad, vmax, mode, flags, MP, st)
    if (d.dbl) {
        if (d.cplx) { if (is_A) OZ2_LE(double, true, true); else OZ2_LE(double, true, false); }
        else OZ2_LE(double, false, false);
    } else {
        if (d.cplx) { if (is_A) OZ2_LE(float, true, true); else OZ2_LE(float, true, false); }
        else OZ2_LE(float, false, false);
    }
#undef OZ2_LE
}

bool split_magnitudes(const OperandDesc &d, bool is_A, size_t nvec, size_t len, int16_t *sft0, int8_t *out,
                      const Layout &L, void *scratch, size_t scratch_bytes, hipStream_t st) {
    if (d.cplx || L.kblk == 0) return false;
    const size_t vpad = round_up(is_A ? L.m_pad : L.n_pad, 64), ktiles = L.kblk / 64;
    if (scratch_bytes < ktiles * vpad * sizeof(int2) + vpad * sizeof(int)) return false;
    if (d.contig && vpad / 64 > 65536) return false;
    int2 *ti = static_cast<int2 *>(scratch);
    int *vexp = reinterpret_cast<int *>(ti + ktiles * vpad);
    const int flags = d.contig ? ENC_KFIRST : 0;
    const dim3 g1 = d.contig ? dim3((unsigned)ktiles, (unsigned)(vpad / 64)) : dim3((unsigned)(vpad / 64), (unsigned)ktiles);
    const dim3 g2((unsigned)((nvec + 63) / 64)),
        g3((unsigned)((nvec + 31) / 32), (unsigned)((ktiles + 4 * FIX_T - 1) / (4 * FIX_T)));
    if (g3.y > 65535) return false;
    const bool nt = nvec * len * (d.dbl ? 8 : 4) >= NT_OPERAND_BYTES;
#define OZ2_MG(R, C) do { \
        const R *x = static_cast<const R *>(d.ptr); \
        if (nt) launch(mag_tile_kernel<R, C, true>, g1, dim3(256), st, x, d.ld, nvec, len, out, L.ksteps, ti, vpad, flags); \
        else launch(mag_tile_kernel<R, C, false>, g1, dim3(256), st, x, d.ld, nvec, len, out, L.ksteps, ti, vpad, flags); \
        if (nvec) { \
            launch(mag_vexp_kernel<R>, g2, dim3(256), st, nvec, ktiles, (const int2 *)ti, vpad, vexp, sft0); \
            launch(mag_fixup_kernel<R, C>, g3, dim3(256), st, x, d.ld, nvec, len, out, L.ksteps, ktiles, \
                   (const int2 *)ti, vpad, (const int *)vexp); \
        } } while (0)
    if (d.dbl) { if (d.contig) OZ2_MG(double, true); else OZ2_MG(double, false); }
    else { if (d.contig) OZ2_MG(float, true); else OZ2_MG(float, false); }
#undef OZ2_MG
    return true;
}

bool split_magnitudes_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len,
                           int16_t *sft0A, int16_t *sft0B, int8_t *outA, int8_t *outB, const Layout &L,
                           void *scratchA, size_t bytesA, void *scratchB, size_t bytesB, int32_t *bound,
                           size_t nbound, hipStream_t st) {
    if (dA.cplx || dB.cplx || dA.dbl != dB.dbl || L.kblk == 0 || m == 0 || n == 0) return false;
    const size_t ktiles = L.kblk / 64;
    auto operand = [&](const OperandDesc &d, size_t nvec, size_t vpad_rows, int16_t *sft0, int8_t *out,
                       void *scratch, size_t bytes, MagOperand &o) {
        const size_t vpad = round_up(vpad_rows, 64);
        if (bytes < ktiles * vpad * sizeof(int2) || (d.contig && vpad / 64 > 65536)) return false;
        o.X = d.ptr;
        o.ld = d.ld;
        o.nvec = nvec;
        o.len = len;
        o.tstride = vpad;
        o.ktiles = ktiles;
        o.out = out;
        o.tinfo = static_cast<int2 *>(scratch);
        o.sft0 = sft0;
        o.flags = d.contig ? ENC_KFIRST : 0;
        o.g1x = d.contig ? (unsigned)ktiles : (unsigned)(vpad / 64);
        o.g1y = d.contig ? (unsigned)(vpad / 64) : (unsigned)ktiles;
        o.g3x = (unsigned)((nvec + 31) / 32);
        o.g3y = (unsigned)((ktiles + 4 * FIX_T - 1) / (4 * FIX_T));
        return true;
    };
    MagOperand a{}, b{};
    if (!operand(dA, m, L.m_pad, sft0A, outA, scratchA, bytesA, a) ||
        !operand(dB, n, L.n_pad, sft0B, outB, scratchB, bytesB, b))
        return false;
    const size_t g1 = (size_t)a.g1x * a.g1y + (size_t)b.g1x * b.g1y, g3 = (size_t)a.g3x * a.g3y + (size_t)b.g3x * b.g3y;
    if (g1 > 0x7fffffff || g3 > 0x7fffffff) return false;
#define OZ2_MP(R, CA, CB) do { \
        launch(mag_tile_pair_kernel<R, CA, CB>, dim3((unsigned)g1), dim3(256), st, a, b, L.ksteps); \
        launch(mag_fixup_pair_kernel<R, CA, CB>, dim3((unsigned)g3), dim3(256), st, a, b, L.ksteps, bound, nbound); \
    } while (0)
#define OZ2_MPR(R) do { if (dA.contig) { if (dB.contig) OZ2_MP(R, true, true); else OZ2_MP(R, true, false); } \
                        else { if (dB.contig) OZ2_MP(R, false, true); else OZ2_MP(R, false, false); } } while (0)
    if (dA.dbl) OZ2_MPR(double);
    else OZ2_MPR(float);
#undef OZ2_MPR
#undef OZ2_MP
    return true;
}

static int fused_split_mode() {  // GEMMUL8_FUSED_SPLIT=0: the two-launch split (A/B runs)
    static const int v = [] {
        const char *e = getenv("GEMMUL8_FUSED_SPLIT");
        return e ? atoi(e) : 1;
    }();
    return v;
}
template <bool MAG>
static bool fused_pair_launch(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len,
                              float log2M, int16_t *sftA, int16_t *sftB, int8_t *outA, int8_t *outB, const Layout &L,
                              const ModParams &MP, int32_t *zero, size_t nzero, hipStream_t st) {
    if (!fused_split_mode() || dA.cplx || dB.cplx || !dA.dbl || !dB.dbl || L.kara || L.kblk == 0 || L.kblk > 2048 ||
        m == 0 || n == 0)
        return false;
    FusedOperand a{}, b{};
    a.X = static_cast<const double *>(dA.ptr);
    a.ld = dA.ld;
    a.nvec = m;
    a.vpad = round_up(L.m_pad, 64);
    a.plane = L.planeA;
    a.vmax = L.m_pad;
    a.sft = sftA;
    a.out = outA;
    b.X = static_cast<const double *>(dB.ptr);
    b.ld = dB.ld;
    b.nvec = n;
    b.vpad = round_up(L.n_pad, 64);
    b.plane = L.planeB;
    b.vmax = L.n_pad;
    b.sft = sftB;
    b.out = outB;
    // vectors per block: GEMMUL8_FUSED_V = 4 / 8 (read once), by default 4.  (Two or four pipelined groups of 4 per
    // block, GRP in fused_body, measured 1.3-1.9x slower: fewer blocks, fewer waves; fused_split/grp_ab.txt.)
    static const int fv = [] {
        const char *e = getenv("GEMMUL8_FUSED_V");
        return e && atoi(e) == 8 ? 8 : 4;
    }();
    const size_t blocks = (a.vpad + b.vpad) / fv;
    if (blocks > 0x7fffffff) return false;
    const ModGroups G = make_groups(MP, L.N);
    const dim3 grid((unsigned)blocks), block(64 * fv);
#define OZ2_FZ1(K, V, CA, CB) launch(split_fused_kernel<K, V, 64 * V, CA, CB, false, MAG>, grid, block, st, a, b, len, L.ksteps, L.kblk, log2M, MP, G, zero, nzero)
#define OZ2_FZ(K, V) do { if (dA.contig) { if (dB.contig) OZ2_FZ1(K, V, true, true); else OZ2_FZ1(K, V, true, false); } \
                          else { if (dB.contig) OZ2_FZ1(K, V, false, true); else OZ2_FZ1(K, V, false, false); } } while (0)
    if (L.kblk <= 1024) { if (fv == 8) OZ2_FZ(1024, 8); else OZ2_FZ(1024, 4); }
    else if (L.kblk <= 1536) { if (fv == 8) OZ2_FZ(1536, 8); else OZ2_FZ(1536, 4); }
    else { if (fv == 8) OZ2_FZ(2048, 8); else OZ2_FZ(2048, 4); }
#undef OZ2_FZ
#undef OZ2_FZ1
    return true;
}
bool split_fused_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len, int VT,
                      float log2M, int16_t *sftA, int16_t *sftB, int8_t *outA, int8_t *outB, const Layout &L,
                      const ModParams &MP, hipStream_t st) {
    if (VT != 128) return false;  // (the reference's VT = 128 summation order)
    return fused_pair_launch<false>(dA, m, dB, n, len, log2M, sftA, sftB, outA, outB, L, MP, nullptr, 0, st);
}
bool split_fused_magnitudes_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len,
                                 int16_t *sft0A, int16_t *sft0B, int8_t *outA, int8_t *outB, const Layout &L,
                                 const ModParams &MP, int32_t *bound, size_t nbound, hipStream_t st) {
    return fused_pair_launch<true>(dA, m, dB, n, len, 0.f, sft0A, sft0B, outA, outB, L, MP, bound, nbound, st);
}

void split_finalize_accurate_pair(const int16_t *sft0A, const int32_t *boundA, size_t m, const int16_t *sft0B,
                                  const int32_t *boundB, size_t n, float log2M, int16_t *outA, int16_t *outB,
                                  hipStream_t st) {
    if (m + n == 0) return;
    launch(finalize_accurate_pair_kernel, dim3((unsigned)((m + n + 255) / 256)), dim3(256), st, sft0A, boundA, m,
           sft0B, boundB, n, log2M, outA, outB);
}

bool split_stats_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len, int VT,
                      float log2M, int16_t *sftA, int16_t *sftB, hipStream_t st) {
    if (dA.cplx || dB.cplx || !dA.dbl || !dB.dbl || dA.contig || !dB.contig || VT != 128) return false;
    const int rows = stats_rows(m);
    const unsigned ga = (unsigned)((m + rows - 1) / rows), gb = (unsigned)((n + 1) / 2);
    const double *a = static_cast<const double *>(dA.ptr), *b = static_cast<const double *>(dB.ptr);
    const bool nt = (m + n) * len * sizeof(double) >= 2 * NT_OPERAND_BYTES;
#define OZ2_SP(r, t) launch(stats_pair_kernel<r, t>, dim3(ga + gb), dim3(256), st, a, dA.ld, m, b, dB.ld, n, len, log2M, sftA, sftB, ga)
    if (rows == 16) { if (nt) OZ2_SP(16, true); else OZ2_SP(16, false); }
    else if (rows == 8) OZ2_SP(8, false);
    else OZ2_SP(4, false);
#undef OZ2_SP
    return true;
}

template <typename R, bool CPLX, bool CA, bool CB>
static void launch_encode_pair(const EncOperand &a, const EncOperand &b, const Layout &L, const ModParams &MP,
                               hipStream_t st) {
    const ModGroups G = make_groups(MP, L.N);
    const dim3 grid(a.gx * a.gy + b.gx * b.gy), block(CPLX ? 128 : 256);
    if constexpr (!CPLX) {
        if (a.acc.sft0) {  // accurate shifts in the encode (small problems: plain loads)
            launch(encode_pair_kernel<R, CPLX, CA, CB, false, true>, grid, block, st, a, b, L.ksteps, L.kblk, MP, G);
            return;
        }
    }
    // non-temporal loads only for the real f64 form, the one large calls take (the others fork per operand)
    if (!CPLX && sizeof(R) == 8 && (a.nvec + b.nvec) * a.len * sizeof(R) >= 2 * NT_OPERAND_BYTES)
        launch(encode_pair_kernel<R, CPLX, CA, CB, !CPLX && sizeof(R) == 8>, grid, block, st, a, b, L.ksteps, L.kblk, MP, G);
    else
        launch(encode_pair_kernel<R, CPLX, CA, CB, false>, grid, block, st, a, b, L.ksteps, L.kblk, MP, G);
}
template <typename R, bool CPLX>
static void launch_encode_pair_ops(bool ca, bool cb, const EncOperand &a, const EncOperand &b, const Layout &L,
                                   const ModParams &MP, hipStream_t st) {
    if (ca) { if (cb) launch_encode_pair<R, CPLX, true, true>(a, b, L, MP, st); else launch_encode_pair<R, CPLX, true, false>(a, b, L, MP, st); }
    else { if (cb) launch_encode_pair<R, CPLX, false, true>(a, b, L, MP, st); else launch_encode_pair<R, CPLX, false, false>(a, b, L, MP, st); }
}

bool split_encode_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len,
                       const int16_t *sftA, const int16_t *sftB, int8_t *outA, int8_t *outB, const Layout &L,
                       const ModParams &MP, hipStream_t st, const AccurateShifts *accs) {
    // operands of one element type (the same ModGroups and tile type); anything else: two launches
    if (dA.cplx != dB.cplx || dA.dbl != dB.dbl || L.kblk == 0) return false;
    if (accs && (dA.cplx || L.kara)) return false;  // (real operands only: complex A rows take two bound maxima)
    const bool cplx = dA.cplx;
    const int KT = cplx ? 32 : 64;
    // per operand exactly what split_encode sets up for mode 0
    auto operand = [&](const OperandDesc &d, bool is_A, size_t nvec, const int16_t *sft, int8_t *out, size_t plane) {
        EncOperand e{};
        e.X = d.ptr;
        e.ld = d.ld;
        e.nvec = nvec;
        e.len = len;
        e.sft = sft;
        e.out = out;
        e.plane = plane;
        const bool kara = L.kara;
        size_t vpad = kara ? (is_A ? L.vsA : L.vsB) : is_A ? (cplx ? L.m_pad - L.m : L.m_pad) : L.n_pad;
        vpad = round_up(vpad, 64);
        e.vmax = kara ? (is_A ? L.vsA : L.vsB) : is_A ? L.m_pad : L.n_pad;
        e.flags = (d.contig ? ENC_KFIRST : 0) | (d.conj ? ENC_CONJ : 0) | (kara ? ENC_KARA : 0);
        e.gx = d.contig ? (unsigned)(L.kblk / KT) : (unsigned)(vpad / 64);
        e.gy = d.contig ? (unsigned)(vpad / 64) : (unsigned)(L.kblk / KT);
        return e;
    };
    EncOperand a = operand(dA, true, m, sftA, outA, L.planeA);
    EncOperand b = operand(dB, false, n, sftB, outB, L.planeB);
    if (accs) {
        a.acc = AccShift{accs->sft0A, accs->boundA, const_cast<int16_t *>(sftA), accs->log2M};
        b.acc = AccShift{accs->sft0B, accs->boundB, const_cast<int16_t *>(sftB), accs->log2M};
    }
    if (a.gx * a.gy == 0 || b.gx * b.gy == 0) return false;
    if (dA.dbl) {
        if (cplx) launch_encode_pair_ops<double, true>(dA.contig, dB.contig, a, b, L, MP, st);
        else launch_encode_pair_ops<double, false>(dA.contig, dB.contig, a, b, L, MP, st);
    } else {
        if (cplx) launch_encode_pair_ops<float, true>(dA.contig, dB.contig, a, b, L, MP, st);
        else launch_encode_pair_ops<float, false>(dA.contig, dB.contig, a, b, L, MP, st);
    }
    return true;
}

void split_finalize_accurate(const int16_t *sft0, const int32_t *bound, size_t nvec, float log2M, int16_t *out,
                             hipStream_t st, bool cplx_rows) {
    launch(finalize_accurate_sft_kernel, dim3((unsigned)((nvec + 255) / 256)), dim3(256), st, sft0, bound, nvec, log2M,
           out, cplx_rows ? 1 : 0);
}

}  // namespace oz2
