// oz2_common.hpp -- shared definitions of the MI355X (gfx950) Ozaki-II GEMM emulator.
//
// Data layout in HBM (one workspace, caller-owned, see oz2_layout below):
//
//   slice planes   int8  [N][vtile][kstep][16 KiB]   for A (rows of op(A)) and B (cols of op(B))
//                  A 16 KiB panel holds 256 vectors x 64 k-bytes, pre-arranged in MFMA
//                  fragment order: [s:2][blk:8][h:2][r:32][16 B] with
//                  vector = 32*blk + r, k = 32*s + 16*h + byte.  A wave's operand read of
//                  one 32x32 fragment is therefore one contiguous 1 KiB ds_read_b128 sweep,
//                  and the panel is staged HBM->LDS by linear global_load_lds (no swizzle
//                  math, no bank conflicts, no power-of-two row strides in HBM).
//   residue planes uint8 [N][n_pad][m_pad]          column-major, value in [0, p_i)
//   sftA, sftB     int16                            exponents (reference convention: -shift)
//   bound          int32 [m_pad + n_pad]            accurate mode: row/col max |A6 B6^T|
//   sft0           int16 [m_pad + n_pad]            accurate mode: 5 - ilogb(amax)
//
// The reference keeps K-contiguous slices with ld = k rounded to 16 (+64 when a
// multiple of 1024) and a separate int32 product buffer (GEMMul8/src/gemmul8.cu:182-234);
// the tiled layout above replaces both.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#ifndef OCML_BASIC_ROUNDED_OPERATIONS
#error "build with -DOCML_BASIC_ROUNDED_OPERATIONS (directed-rounding intrinsics)"
#endif

#include "oz2_tables.inc"

namespace oz2 {

constexpr int TILE = 256;          // vectors per panel (GEMM block tile edge)
constexpr int KSTEP = 64;          // k-bytes per panel
constexpr int PANEL = TILE * KSTEP;  // 16 KiB
constexpr int QUEUE_HEADS = 8;       // tile-queue heads per products launch (one per XCD)

enum class Scal : int { F64 = 0, F32 = 1 };

struct Layout {
    // logical problem
    size_t m, n, k;  // complex: logical complex sizes
    unsigned N;
    bool cplx;
    // int8 product shape
    size_t mr, kr;       // rows of the int8 A (m, 2m big matrix, 3 m_s Karatsuba), k-extent incl. complex blocks
    size_t kblk;         // k padded to KSTEP (offset of the imaginary block of the big-matrix encode)
    size_t m_pad, n_pad, k_pad;
    size_t ksteps, mtiles, ntiles;  // tiles of ONE sub-product
    size_t planeA, planeB, planeR;  // bytes per modulus
    size_t ldr;                     // leading dimension of a residue (sub-)plane
    // Karatsuba complex products (kara): per modulus three sub-products of the sub-blocks
    // [re | im | re + im] of A's rows and of B's columns, P1 = Ar Br, P2 = Ai Bi, P3 = (Ar+Ai)(Br+Bi):
    // 3 m n k MACs instead of the big matrix's 4 m n k.  The CRT combines their residues into
    // Re = P1 - P2 and Im = P3 - P1 - P2 (mod p).  Otherwise nsub = 1 and the sub strides are 0.
    bool kara;
    unsigned nsub;
    size_t subA, subB, subR;  // byte stride between the sub-blocks of a slice plane / residue plane
    size_t vsA, vsB;          // vectors per sub-block (m and n rounded up to TILE)
    // accurate-mode bound product: always the big-matrix geometry (the reference's bound, quirks
    // included); its row / column maxima and sft0 are indexed with these extents
    size_t bm_pad, bn_pad;
    unsigned S;                    // slice planes held at once (= N unless low-memory mode)
    // workspace offsets (bytes)
    size_t offA, offB, offR, offSftA, offSftB, offBound, offSft0, offQueue, total;
};

static inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Complex products as Karatsuba sub-products or as the reference's big matrix.  The residues of
// Re(AB) and Im(AB) mod p, hence C, are the same bits either way.  Karatsuba saves a quarter of
// the MACs but reads a third residue plane per modulus in the CRT, writes a third B sub-block,
// and halves the k-steps per product block (whose fixed cost then weighs twice as much); measured
// on MI355X (tools/probes/kara_sweep.py, N = 12, Karatsuba / big-matrix time): 4096^3 0.87,
// 3072^3 0.92, 4096 x 256 x 4096 0.89; 2048^3 0.97-1.00, 1536^3 1.00-1.04, 1024^3 1.07,
// 8192^2 x 1024 1.07, 256 x 4096 x 4096 1.13.  Hence the rule below.
// GEMMUL8_CPLX_PRODUCTS=karatsuba / bigmatrix forces either (tests, A/B runs).
static inline bool kara_default(size_t m, size_t n, size_t k) {
    static const int forced = [] {
        const char *e = getenv("GEMMUL8_CPLX_PRODUCTS");
        if (!e) return 0;
        if (e[0] == 'k') return 1;
        if (e[0] == 'b') return 2;
        return 0;
    }();
    if (forced) return forced == 1;
    (void)n;
    return k >= 3072 && m >= 1024;
}

// slice_planes: planes of A / B slices held at once (N: all resident; fewer: the low-memory
// mode encodes the moduli in groups of that size into the same planes, gemmul8.hip run())
// kara: -1 = kara_default(m, n, k) for complex, 0 = the big-matrix geometry (the accurate-mode bound)
static inline Layout make_layout(size_t m, size_t n, size_t k, unsigned N, bool cplx, unsigned slice_planes = 0,
                                 int kara = -1) {
    Layout L{};
    const unsigned S = (slice_planes == 0 || slice_planes > N) ? N : slice_planes;
    L.S = S;
    L.m = m; L.n = n; L.k = k; L.N = N; L.cplx = cplx;
    L.kblk = round_up(k, KSTEP);
    // big-matrix geometry (real operands: the only one)
    L.mr = cplx ? 2 * m : m;
    L.kr = cplx ? 2 * L.kblk : L.kblk;
    L.m_pad = round_up(L.mr, TILE);
    L.n_pad = round_up(n, TILE);
    L.k_pad = L.kr;
    L.bm_pad = L.m_pad;
    L.bn_pad = L.n_pad;
    const size_t big_planeA = L.m_pad * L.k_pad, big_planeB = L.n_pad * L.k_pad;
    L.kara = cplx && (kara < 0 ? kara_default(m, n, k) : kara != 0);
    L.nsub = 1;
    if (L.kara) {
        L.vsA = round_up(m, TILE);
        L.vsB = round_up(n, TILE);
        L.nsub = 3;
        L.mr = 3 * L.vsA;
        L.kr = L.kblk;
        L.m_pad = L.mr;
        L.n_pad = 3 * L.vsB;
        L.k_pad = L.kblk;
        L.subA = L.vsA * L.k_pad;
        L.subB = L.vsB * L.k_pad;
        L.subR = L.vsA * L.vsB;
    }
    L.ksteps = L.k_pad / KSTEP;
    L.mtiles = (L.kara ? L.vsA : L.m_pad) / TILE;
    L.ntiles = (L.kara ? L.vsB : L.n_pad) / TILE;
    L.planeA = L.m_pad * L.k_pad;
    L.planeB = L.n_pad * L.k_pad;
    L.ldr = L.kara ? L.vsA : L.m_pad;
    L.planeR = L.kara ? 3 * L.subR : L.m_pad * L.n_pad;
    // the slice regions also hold the bound product's big-matrix magnitude plane (accurate mode)
    const size_t regA = L.planeA * S > big_planeA ? L.planeA * S : big_planeA;
    const size_t regB = L.planeB * S > big_planeB ? L.planeB * S : big_planeB;
    size_t off = 0;
    L.offA = off; off += round_up(regA, 256);
    L.offB = off; off += round_up(regB, 256);
    L.offR = off; off += round_up(L.planeR * N, 256);
    L.offSftA = off; off += round_up(L.bm_pad * 2, 256);
    L.offSftB = off; off += round_up(L.bn_pad * 2, 256);
    L.offBound = off; off += round_up((L.bm_pad + L.bn_pad) * 4, 256);
    L.offSft0 = off; off += round_up((L.bm_pad + L.bn_pad) * 2, 256);
    // 8 per-XCD tile-queue heads of the persistent product kernel, one set per first modulus of a
    // products launch: launches of disjoint moduli ranges may share the workspace on different streams
    L.offQueue = off; off += round_up(QUEUE_HEADS * OZ2_MAX_MODULI * 4, 256);
    L.total = off;
    return L;
}

// the products of one column range [t0, t1) of B's vector tiles (the residue planes' column
// tiles): the same planes and strides, fewer column tiles.  gemm_i8's tile indices are relative,
// so the caller offsets the B slice pointer by t0 * ksteps panels and the output by t0 * 256 * ldr.
static inline Layout col_tiles(const Layout &L, size_t t0, size_t t1) {
    Layout S = L;
    S.ntiles = t1 - t0;
    return S;
}

// byte offset of the 16-B chunk holding (vector v, k-bytes kk..kk+15), kk % 16 == 0
__host__ __device__ inline size_t panel_offset(size_t v, size_t kk, size_t ksteps) {
    return ((v >> 8) * ksteps + (kk >> 6)) * (size_t)PANEL + ((kk >> 5) & 1) * 8192 + ((v >> 5) & 7) * 1024 +
           (((kk >> 4) & 1) * 32 + (v & 31)) * 16;
}

// ------------------------------------------------------------------
// CRT variant of a call: num_moduli and whether the single-double form (numM = 1) applies.  The
// weights, M and 1/M are compile-time constants of that pair in crt.hip (from oz2_tables.inc); the
// reference uploads them to __constant__ on every call (gemmul8.cu:236-241).
// ------------------------------------------------------------------
struct CrtParams {
    int numM1;
    unsigned N;
};

struct ModParams {
    int p[OZ2_MAX_MODULI];
    int barrett[OZ2_MAX_MODULI];
    double rinv_d[OZ2_MAX_MODULI];
    float rinv_f[OZ2_MAX_MODULI];
    unsigned N;
    // slice encodes only: the persistent product kernel's 8 tile-queue heads, zeroed by the encode's
    // first block (the products follow the encode on the stream; saves a zeroing launch per call)
    uint32_t *zero_queue;
};

static inline ModParams make_mod_params(unsigned N) {
    ModParams P{};
    for (int i = 0; i < OZ2_MAX_MODULI; ++i) {
        P.p[i] = oz2_p[i];
        P.barrett[i] = oz2_barrett[i];
        P.rinv_d[i] = oz2_rinv_d[i];
        P.rinv_f[i] = oz2_rinv_f[i];
    }
    P.N = N;
    return P;
}

static inline CrtParams make_crt_params(unsigned N, bool force_numM1) {
    CrtParams C{};
    C.numM1 = (oz2_numM[N - 2] == 1) || force_numM1;  // float outputs: the no-numM overload (inverse_scaling.hpp:823-856)
    C.N = N;
    return C;
}

// ------------------------------------------------------------------
// device arithmetic shared by the split kernels
// ------------------------------------------------------------------
// residue of an integer-valued x in [-p/2, p/2] as int8 (v_cvt_i32_f32 + byte pack,
// i.e. +128 wraps to -128), restating mod_8i (scaling.hpp:215-230)
__device__ __forceinline__ int mod8_f64(double x, int p, double rinv, float rinvf) {
    float t = __double2float_rn(__builtin_fma(__builtin_rint(x * rinv), -(double)p, x));
    const float pf = -(float)p;
    t = __builtin_fmaf(__builtin_rintf(t * rinvf), pf, t);
    t = __builtin_fmaf(__builtin_rintf(t * rinvf), pf, t);
    return (int)t;
}
// Steps 2-3 of mod8_f64 on two values at once: packed f32 multiply / add / fma, with
// round-to-nearest-even by the 1.5*2^23 shift ((y + c) - c == rintf(y) for |y| <= 2^22; here
// |y| < 2^15), so the result is bit-identical to the scalar form above.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v mod8_tail_x2(f2v t, float rinvf, float pf) {
    const f2v c = {12582912.0f, 12582912.0f};
    const f2v r = {rinvf, rinvf}, q = {pf, pf};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        f2v y = t * r;
        y = (y + c) - c;
        t = __builtin_elementwise_fma(y, q, t);
    }
    return t;
}
// One such step: the residue of t modulo p when |t/p| < 2^10 (t reduced modulo a two-moduli
// product first, split.hip ModGroups)
__device__ __forceinline__ f2v mod8_step_x2(f2v t, float rinvf, float pf) {
    const f2v c = {12582912.0f, 12582912.0f};
    const f2v r = {rinvf, rinvf}, q = {pf, pf};
    f2v y = t * r;
    y = (y + c) - c;
    return __builtin_elementwise_fma(y, q, t);
}
__device__ __forceinline__ float mod8_head_f64(double x, int p, double rinv) {
    return __double2float_rn(__builtin_fma(__builtin_rint(x * rinv), -(double)p, x));
}

__device__ __forceinline__ int mod8_f32(float x, int p, float rinvf) {
    const float pf = -(float)p;
    float t = __builtin_fmaf(__builtin_rintf(x * rinvf), pf, x);
    t = __builtin_fmaf(__builtin_rintf(t * rinvf), pf, t);
    t = __builtin_fmaf(__builtin_rintf(t * rinvf), pf, t);
    t = __builtin_fmaf(__builtin_rintf(t * rinvf), pf, t);
    return (int)t;
}

}  // namespace oz2
