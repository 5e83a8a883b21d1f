// gemm_i8.hip -- exact int8 x int8 -> int32 slice products on CDNA4 MFMA with fused epilogues.
//
// Replaces the reference's per-modulus hipblasGemmEx + conv_32i_2_8u pair
// (GEMMul8/src/gemmul8.cu:259-275, conv_32i_2_8u.hpp:7-71): one launch covers all
// N moduli (grid.y = modulus; 3 j + s for the Karatsuba complex sub-products s = 0..2 of
// modulus j, an instantiation of its own), each 256x256 output tile accumulates with
// v_mfma_i32_16x16x64_i8 and is reduced mod p_i in the epilogue, so the int32
// product never reaches HBM (the reference writes and re-reads 4*m*n bytes per
// modulus).  The accurate-mode bound product (scaling.hpp:3113-3121) runs the same
// main loop with a row/column-max epilogue instead of an m x n int32 buffer.
//
// Block: 512 threads = 8 waves, two per SIMD, as 2 (M) x 4 (N); each wave owns a
// 128 x 64 sub-tile = 8 x 4 tiles of 16x16 (128 accumulator registers; the
// 32x32x32 form, 4 x 2 tiles, remains behind OZ2_MFMA16=0 for A/B probes).
// The two waves of a SIMD PING-PONG: waves 0-3 (group 0) and 4-7 (group 1) run the
// same per-k-step sequence
//     load interval:  12 fragment reads (ds_read_b128, 1 KiB conflict-free sweeps)
//                     + 4 LDS-DMA pieces of the step D ahead; wait for them
//     barrier
//     MFMA interval:  32 MFMAs (16x16x64; 16 of 32x32x32)
//     barrier
// with group 1 one barrier behind, so on every SIMD one wave's MFMAs run while the
// other wave issues its LDS reads and LDS-DMA (whose issue costs 60-185 cycles each
// and, with one wave per SIMD, stalled the matrix core).
// Operand panels (16 KiB, pre-arranged in fragment order by split.hip) stream
// HBM -> LDS through a 4-slot ring (128 KiB) with LDS-DMA issued three k-steps
// ahead; waits are counted by hand (vmcnt), barriers are raw s_barrier.
#include <atomic>
#include <type_traits>

#include "oz2_split.hpp"

namespace oz2 {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// MFMA shape of the products: 1 = v_mfma_i32_16x16x64_i8 (8 x 4 tiles of 16 x 16 per wave), 0 =
// v_mfma_i32_32x32x32_i8 (4 x 2 tiles of 32 x 32).  Same operand bytes, LDS reads and accumulator
// registers per k-step; the 16x16 form moves a quarter of the accumulator data per instruction.
#ifndef OZ2_MFMA16
#define OZ2_MFMA16 1
#endif
#if OZ2_MFMA16
typedef v4i AccTile;
constexpr int ACC_I = 8, ACC_J = 4;  // 16-row x 16-col tiles of a wave's 128 x 64
#else
typedef v16i AccTile;
constexpr int ACC_I = 4, ACC_J = 2;  // 32 x 32 tiles
#endif

constexpr int NTHREADS = 512;
#ifndef OZ2_RES_NTS
// the persistent kernel's residue stores are non-temporal: they no longer allocate in the L2, where they evicted
// operand panels (same bits; tools/probes/lib_ab.py, 4 interleaved rounds, profiles/r05/nt_store_ab/: 8192^2 x
// 1024 -2.4 %, cfg5 -0.3 %, cfg2 -0.2 %).  0 = plain stores (A/B builds)
#define OZ2_RES_NTS 1
#endif
#ifndef OZ2_STAGES
#define OZ2_STAGES 4
#endif
constexpr int STAGES = OZ2_STAGES;  // ring slots; DMA runs STAGES-1 k-steps ahead
constexpr int SLOT = 2 * PANEL;     // A panel + B panel
constexpr int LDS_BYTES = STAGES * SLOT;  // the epilogue reuses 64 KiB of it
constexpr int GLDS_PER_STEP = 4;
// internal epilogue: RESIDUE whose residues are added mod p into the planes (k-chunks after the
// first); a separate instantiation so the one-pass kernel's code stays as it is
constexpr int EPI_RESIDUE_ADD = 3;          // 1 KiB LDS-DMA pieces per wave per k-step (2 A + 2 B)

struct GemmArgs {
    const int8_t *A;
    const int8_t *B;
    size_t planeA, planeB;
    unsigned ksteps, mtiles, ntiles;
    unsigned kstride, k0;            // panels per tile in the planes, first k-step of this launch
    void *out;
    size_t planeOut, ldo;
    int32_t *rowmax, *colmax;
    int p[OZ2_MAX_MODULI];
    int barrett[OZ2_MAX_MODULI];     // floor(2^32/p) - 1 (signed path, reference conv_32i_2_8u)
    uint32_t minv[OZ2_MAX_MODULI];   // floor(2^32/p)     (biased unsigned path)
    int bias[OZ2_MAX_MODULI];        // ceil(2^30/p) * p  (accumulator start value, biased path)
    double invp[OZ2_MAX_MODULI];     // fl(1/p)           (f64 form of the biased path)
    int biased;                      // |product| <= 2^30 (k_pad <= 2^16): biased path
    // sub-products per modulus (Karatsuba complex: 3, blockIdx.y = 3 j + s), each offset by s times
    // these strides in the A, B and output planes
    unsigned nsub;
    size_t subA, subB, subOut;
    // persistent kernel: planes of the launch (sub-products counted)
    unsigned nplanes;
    uint32_t *queue;  // 8 per-XCD tile-queue heads, zeroed before the launch
    unsigned long long *stamps;  // probe builds (OZ2_STAMPS): per-wave phase cycle sums
};

// One 16-byte-per-lane LDS-DMA: LDS[m0 + lane*16] <- gsrc (per lane).  Issued from inline asm
// so the compiler neither waits for it nor reorders it; completion is counted with vmcnt by hand.
// M0 is compiler-reserved: saved and restored inside the statement.
#ifndef OZ2_ABLATE
#define OZ2_ABLATE 0  // probe builds only: 1 = no LDS-DMA, 2 = no MFMA, 3 = no LDS reads, 5 = LDS reads of the first
                     // step only, 6 = LDS-DMA of the prologue only (real operands, no data movement in the loop),
                     // 7 = residue epilogue reduced to the low byte, 8 = every LDS-DMA re-reads k-steps 0/1
                     // (L2 hits: the fabric / Infinity-Cache share of the DMA), 9 = residues parked in LDS but
                     // not stored, 10 = no epilogue (accumulators kept live)
#endif
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_addr) {
    if (OZ2_ABLATE == 1) return;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
    __builtin_amdgcn_sched_barrier(0);
}
// The same LDS-DMA through a buffer descriptor (SGPR base + 32-bit per-lane offset).  Measured on
// the product kernel: the texture units spend 20 % fewer cycles per byte on it than on the 64-bit
// flat form (TD_TD_BUSY 1.91e9 vs 2.38e9 per cfg2 launch), MFMA busy 68 % -> 85 % of the cycles.
typedef int v4si __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4si make_rsrc(const void *base, uint32_t bytes) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    v4si r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32) & 0xffff);  // stride 0
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);                         // num_records
    r[3] = 0x00020000;                                                         // raw buffer, dword data
    return r;
}
__device__ __forceinline__ void bglds16(v4si rsrc, uint32_t voff, uint32_t lds_addr) {
    if (OZ2_ABLATE == 1) return;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rsrc), "s"(lds_addr)
                 : "memory");
    __builtin_amdgcn_sched_barrier(0);
}
// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]);
// the builtin form is visible to the compiler's own waitcnt tracking of its ds_reads.
template <int N> __device__ __forceinline__ void wait_vm_lgkm0() {
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (0 << 8) | ((N >> 4) << 14));
    __builtin_amdgcn_sched_barrier(0);
}
// drain: wait until at most `younger` k-steps of this wave's LDS-DMA remain in flight
template <int PER_STEP> __device__ __forceinline__ void wait_steps_lgkm0(int younger) {
    switch (younger) {
    case 0: wait_vm_lgkm0<0>(); break;
    case 1: wait_vm_lgkm0<PER_STEP>(); break;
    case 2: wait_vm_lgkm0<2 * PER_STEP>(); break;
    default: wait_vm_lgkm0<3 * PER_STEP>(); break;
    }
}
__device__ __forceinline__ void barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// r = x mod p in [0, p), the value of conv_32i_2_8u.hpp:7-56 (modulus 256 = low byte, others
// Barrett).  Signed path, any |x| <= 2^31:
__device__ __forceinline__ uint32_t residue(int x, int p, int barrett, bool p256) {
    if (p256) return (uint32_t)x & 0xffu;
    x -= __mulhi(x, barrett) * p;
    x -= (x >= p) * p;
    x += (x < 0) * p;
    return (uint32_t)x;
}
// Biased path: the accumulator started at bias = ceil(2^30/p)*p (a multiple of p), so for
// |x| <= 2^30 it holds u = x + bias in [0, 2^31 + p).  With m = floor(2^32/p),
// q = floor(u*m / 2^32) is floor(u/p) or one less, so u - q*p lies in [0, 2p) and one
// unsigned min folds it into [0, p).  q < 2^24, so q*p is a full-rate 24-bit multiply.
// Five VALU ops, no branches, one formula for every modulus including 256.
__device__ __forceinline__ uint32_t residue_biased(uint32_t u, uint32_t p, uint32_t m) {
    const uint32_t q = __umulhi(u, m);
    const uint32_t r = u - __umul24(q, p);
    return min(r, r - p);
}

// The same residue in f64 (p < 256; the product epilogues' form): zc = 2^52 + u exactly (the bit
// pattern 0x43300000:u), so fma(zc, fl(1/p), -2^52 fl(1/p) + 2^-8) = u fl(1/p) + 2^-8 (the constant
// is exact: 2^52 fl(1/p) is a multiple of 2^-8; the fma's rounding and fl(1/p)'s error stay below
// 2^-28 for u < 2^32), whose floor is floor(u/p) because 0 < r/p + 2^-8 < 1 for every r <= p - 1 < 255;
// then fma(q, -p, zc) = 2^52 + r exactly and the low dword of that double is r.  Three f64 ops, no
// 32-bit integer multiply.  For p = 256 the epilogues take the low byte of u (the bias is a multiple
// of 256).  gemmul8_residue_selftest path 3 checks it for every u of the biased range.
__device__ __forceinline__ uint32_t residue_biased_f64(uint32_t u, double invp, double cneg, double pneg) {
    const double zc = __hiloint2double(0x43300000, (int)u);
    const double q = __builtin_floor(__builtin_fma(zc, invp, cneg));
    return (uint32_t)__double2loint(__builtin_fma(q, pneg, zc));
}

// Two forms without v_floor_f64 (A/B probes, EPIM 3 / 4).  y = fma(zc, fl(1/p), c - 1/2) is u/p + 2^-8 - 1/2
// within 2^-28 (c - 1/2 stays exact: a multiple of 2^-8 below 2^45), i.e. q + f with |f| < 1/2 strictly
// (r/p + 2^-8 <= 254/255 + 2^-8 < 1 for p <= 255), so t = y + 1.5 * 2^52 rounds to 1.5 * 2^52 + q exactly and
// the low dword of t is q = floor(u/p).  EPIM 3 finishes in f64 (q = t - 1.5 * 2^52, fma back), EPIM 4 in
// 32-bit integers (r = u - q p, q < 2^24).
__device__ __forceinline__ uint32_t residue_biased_f64r(uint32_t u, double invp, double chalf, double pneg) {
    const double zc = __hiloint2double(0x43300000, (int)u);
    const double t = __builtin_fma(zc, invp, chalf) + 0x1.8p52;
    return (uint32_t)__double2loint(__builtin_fma(t - 0x1.8p52, pneg, zc));
}
__device__ __forceinline__ uint32_t residue_biased_f64i(uint32_t u, double invp, double chalf, uint32_t p) {
    const double zc = __hiloint2double(0x43300000, (int)u);
    const double t = __builtin_fma(zc, invp, chalf) + 0x1.8p52;
    return u - __umul24((uint32_t)__double2loint(t), p);
}

// four residues in [0, p) per word: (a + b) mod p bytewise
__device__ __forceinline__ uint32_t add_mod_bytes(uint32_t a, uint32_t b, uint32_t p) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = ((a >> (8 * i)) & 0xffu) + ((b >> (8 * i)) & 0xffu);
        r |= min(s, s - p) << (8 * i);
    }
    return r;
}

#if OZ2_MFMA16
// One k-step (64 deep) of fragments for a wave: 8 row blocks of 16 of A, 4 column blocks of 16 of B.
// The panel layout [s:2][blk:8][h:2][r:32][16 B] (vector 32 blk + r, k 32 s + 16 h + byte) is read
// with per-lane addresses: lane l = r16 + 16 q takes the 16 k-bytes 16q.. of vector r16 of the block,
// i.e. (s, h) = (q >> 1, q & 1); A and B lanes pair the same k-bytes, which is all the dot product
// needs.  Each group of 16 lanes reads 256 contiguous bytes (conflict-free).
struct Frags {
    v4i a[8];
    v4i b[4];
};
__device__ __forceinline__ int frag_lane_offset(int lane) {
    const int q = lane >> 4;
    return (q >> 1) * 8192 + ((q & 1) * 32 + (lane & 15)) * 16;
}
__device__ __forceinline__ void read_frags(Frags &f, const int8_t *slot, int wr, int wc, int lane) {
    const int8_t *base = slot + frag_lane_offset(lane);
    if (OZ2_ABLATE == 3 || OZ2_ABLATE == 4) {  // probe: no LDS reads (operands = slot address bits)
#pragma unroll
        for (int i = 0; i < 8; ++i) f.a[i] = v4i{} + (int)(uintptr_t)slot + i;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) f.b[jj] = v4i{} + (int)(uintptr_t)slot + jj;
        return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)  // rows 16 i.. of the wave's 128: block wr*4 + i/2, half i&1
        f.a[i] = *reinterpret_cast<const v4i *>(base + (wr * 4 + (i >> 1)) * 1024 + (i & 1) * 256);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)  // columns 16 jj.. of the wave's 64: block wc*2 + jj/2, half jj&1
        f.b[jj] = *reinterpret_cast<const v4i *>(base + PANEL + (wc * 2 + (jj >> 1)) * 1024 + (jj & 1) * 256);
}
#ifndef OZ2_MFMA_ORDER
#define OZ2_MFMA_ORDER 0  // probe builds: 0 = A-major (4 consecutive MFMAs share an A fragment), 1 = B-major
#endif
// PRIO 0: the MFMA interval runs at priority 1 (raised and dropped around every interval); other
// values leave the wave's priority alone (the persistent kernel's static-priority variants)
template <int PRIO = 0>
__device__ __forceinline__ void mfma_step(AccTile (&acc)[ACC_I][ACC_J], const Frags &f) {
    if (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int x = 0; x < 32; ++x) {
        const int i = OZ2_MFMA_ORDER ? (x & 7) : (x >> 2), jj = OZ2_MFMA_ORDER ? (x >> 3) : (x & 3);
        if (OZ2_ABLATE == 2 || OZ2_ABLATE == 4) {
            acc[i][jj][0] += f.a[i][0] ^ f.b[jj][1];
        } else {
            acc[i][jj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[i], f.b[jj], acc[i][jj], 0, 0, 0);
        }
    }
    if (PRIO == 0) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
}
// accumulator map (16x16 tiles): col = lane & 15, row = 4 (lane >> 4) + e, e = 0..3
__device__ __forceinline__ int acc_row(int i, int e, int lane) { return i * 16 + 4 * (lane >> 4) + e; }
__device__ __forceinline__ int acc_col(int jj, int lane) { return jj * 16 + (lane & 15); }
constexpr int ACC_E = 4;
#else
// One k-step of fragments for a wave: 4 row blocks of A, 2 column blocks of B, both 32-deep halves.
struct Frags {
    v4i a[2][4];
    v4i b[2][2];
};

// panel layout [s:2][blk:8][h:2][r:32][16 B]: fragment (s, blk) is the 1 KiB at s*8192 + blk*1024
__device__ __forceinline__ void read_frags(Frags &f, const int8_t *slot, int wr, int wc, int lane) {
    if (OZ2_ABLATE == 3 || OZ2_ABLATE == 4) {  // probe: no LDS reads (operands = slot address bits)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int i = 0; i < 4; ++i) f.a[s][i] = v4i{} + (int)(uintptr_t)slot + i;
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) f.b[s][jj] = v4i{} + (int)(uintptr_t)slot + jj;
        }
        return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            f.a[s][i] = *reinterpret_cast<const v4i *>(slot + s * 8192 + (wr * 4 + i) * 1024 + lane * 16);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
            f.b[s][jj] = *reinterpret_cast<const v4i *>(slot + PANEL + s * 8192 + (wc * 2 + jj) * 1024 + lane * 16);
    }
}

template <int PRIO = 0>
__device__ __forceinline__ void mfma_step(AccTile (&acc)[ACC_I][ACC_J], const Frags &f) {
    if (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int x = 0; x < 8; ++x) {
            const int i = x >> 1, jj = x & 1;  // (serpentine orders that share an operand between
                                               // consecutive MFMAs measured the same clock)
            if (OZ2_ABLATE == 2 || OZ2_ABLATE == 4) {
                acc[i][jj][0] += f.a[s][i][0] ^ f.b[s][jj][1];
            } else {
                acc[i][jj] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f.a[s][i], f.b[s][jj], acc[i][jj], 0, 0, 0);
            }
        }
    if (PRIO == 0) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
}

// accumulator map (32x32 tiles): col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
__device__ __forceinline__ int acc_row(int i, int e, int lane) { return i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5); }
__device__ __forceinline__ int acc_col(int jj, int lane) { return jj * 32 + (lane & 31); }
constexpr int ACC_E = 16;
#endif

// Epilogues over the 8 compute waves' accumulators (active = this wave holds a 128 x 64 block;
// every thread of the block must call it: it contains block barriers).
template <int EPI>
__device__ __forceinline__ void epilogue(const GemmArgs &g, AccTile (&acc)[ACC_I][ACC_J], int8_t *smem, int tid, int lane, int wr,
                                         int wc, unsigned tm, unsigned tn, unsigned j, unsigned sb, bool active) {
    if constexpr (EPI == (int)Epi::RESIDUE || EPI == EPI_RESIDUE_ADD) {
        const int p = g.p[j];
        // residues -> LDS as [256 cols][PARK_CS dwords], dword d = rows 4d..4d+3 of the column.  The column stride of
        // 68 dwords (272 B) keeps the 16-byte chunks aligned and spreads a 16 x 16 accumulator tile's dword writes
        // over the banks (two lanes per bank), and every write of a lane is ONE base address plus an immediate
        // offset (the XOR-swizzled layout before it cost ~5 address instructions per write and a runtime dword
        // permutation per 16-byte read; tools/probes/onetile_ablate.hip)
        constexpr int PARK_CS = 68;
        static_assert(256 * PARK_CS * 4 <= LDS_BYTES, "park area");
        uint32_t *lo = reinterpret_cast<uint32_t *>(smem);
        uint32_t *pbase = lo + (wc * 64 + (lane & 15)) * PARK_CS + wr * 32 + (lane >> 4);
        auto park = [&](auto &&res) {
            if (!active) return;
#pragma unroll
            for (int i = 0; i < ACC_I; ++i)
#pragma unroll
                for (int jj = 0; jj < ACC_J; ++jj) {
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w |= res(acc[i][jj][e]) << (8 * e);
                    pbase[jj * 16 * PARK_CS + 4 * i] = w;
                }
        };
        static_assert(OZ2_MFMA16, "park map: 16x16 accumulator tiles");
        if (OZ2_ABLATE == 7 || (g.biased && p == 256)) {  // (7: probe) p = 256: bias is a multiple of 256
            park([&](int x) { return (uint32_t)x & 0xffu; });
        } else if (g.biased) {
            const double invp = g.invp[j], pneg = -(double)p;
            const double cneg = __builtin_fma(-0x1p52, invp, 0x1p-8);
            park([&](int x) { return residue_biased_f64((uint32_t)x, invp, cneg, pneg); });
        } else {
            const int bar = g.barrett[j];
            const bool p256 = (p == 256);  // modulus 256: the low byte (conv_32i_2_8u.hpp:7-20)
            park([&](int x) { return residue(x, p, bar, p256); });
        }
        __syncthreads();
        uint8_t *out = static_cast<uint8_t *>(g.out) + j * g.planeOut + sb * g.subOut + (size_t)tn * 256 * g.ldo +
                       (size_t)tm * 256;
#pragma unroll
        for (int it = 0; it < 4096 / 512; ++it) {
            if (tid >= 512) break;
            const int chunk = tid + 512 * it;
            const int col = chunk >> 4, qd = chunk & 15;
            uint4 res = *reinterpret_cast<const uint4 *>(lo + col * PARK_CS + 4 * qd);
            uint4 *dst = reinterpret_cast<uint4 *>(out + (size_t)col * g.ldo + 16 * qd);
            if (OZ2_ABLATE == 9) {  // probe: no residue store
                asm volatile("" ::"v"(res.x), "v"(res.y), "v"(res.z), "v"(res.w));
                continue;
            }
            if constexpr (EPI == EPI_RESIDUE_ADD) {  // k-chunked product: (earlier chunks + this chunk) mod p
                const uint4 prev = *dst;
                res = make_uint4(add_mod_bytes(res.x, prev.x, (uint32_t)p), add_mod_bytes(res.y, prev.y, (uint32_t)p),
                                 add_mod_bytes(res.z, prev.z, (uint32_t)p), add_mod_bytes(res.w, prev.w, (uint32_t)p));
            }
            *dst = res;
        }
    } else if constexpr (EPI == (int)Epi::BOUND) {
        int32_t *rmax = reinterpret_cast<int32_t *>(smem);
        int32_t *cmax = rmax + 256;
        if (tid < 256) {
            rmax[tid] = 0;
            cmax[tid] = 0;
        }
        __syncthreads();
        // rows: lanes sharing a row are those with the same row part of the lane index; columns: the same
        // column part (32x32: lane & 31 / lane >> 5; 16x16: lane >> 4 / lane & 15)
        constexpr int COLS_PER_TILE = OZ2_MFMA16 ? 16 : 32;
#pragma unroll
        for (int i = 0; i < ACC_I && active; ++i)
#pragma unroll
            for (int rr = 0; rr < ACC_E; ++rr) {
                int v = 0;
#pragma unroll
                for (int jj = 0; jj < ACC_J; ++jj) v = max(v, abs(acc[i][jj][rr]));
#pragma unroll
                for (int d = COLS_PER_TILE / 2; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, COLS_PER_TILE));
                if ((lane & (COLS_PER_TILE - 1)) == 0) atomicMax(&rmax[wr * 128 + acc_row(i, rr, lane)], v);
            }
#pragma unroll
        for (int jj = 0; jj < ACC_J && active; ++jj) {
            int v = 0;
#pragma unroll
            for (int i = 0; i < ACC_I; ++i)
#pragma unroll
                for (int rr = 0; rr < ACC_E; ++rr) v = max(v, abs(acc[i][jj][rr]));
#pragma unroll
            for (int d = COLS_PER_TILE; d < 64; d <<= 1) v = max(v, __shfl_xor(v, d));
            if (lane < COLS_PER_TILE) atomicMax(&cmax[wc * 64 + acc_col(jj, lane)], v);
        }
        __syncthreads();
        if (tid < 256) {
            atomicMax(&g.rowmax[tm * 256 + tid], rmax[tid]);
            atomicMax(&g.colmax[tn * 256 + tid], cmax[tid]);
        }
    } else if (active) {  // RAW int32 (plane 0): validation path
        int32_t *out = static_cast<int32_t *>(g.out);
#pragma unroll
        for (int i = 0; i < ACC_I; ++i)
#pragma unroll
            for (int jj = 0; jj < ACC_J; ++jj)
#pragma unroll
                for (int rr = 0; rr < ACC_E; ++rr) {
                    const size_t row = (size_t)tm * 256 + wr * 128 + acc_row(i, rr, lane);
                    const size_t col = (size_t)tn * 256 + wc * 64 + acc_col(jj, lane);
                    out[col * g.ldo + row] = acc[i][jj][rr];
                }
    }
}

// BUF: operand planes below 4 GiB are staged through buffer descriptors (bglds16), larger ones
// through 64-bit flat addresses (glds16).  SUB: Karatsuba complex, 3 sub-products per modulus
// (an instantiation of its own, so the real-operand kernel's code is unchanged).
template <int EPI, int BUF, bool SUB = false>
__global__ __launch_bounds__(NTHREADS, 1) void gemm_i8_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(1024))) int8_t smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;  // wr doubles as the ping-pong group
    const unsigned j = SUB ? blockIdx.y / 3 : blockIdx.y;  // modulus
    const unsigned sb = SUB ? blockIdx.y - 3 * j : 0;      // Karatsuba sub-product

    // XCD-aware, bijective remap: blocks dealt round-robin over the 8 XCDs get
    // contiguous logical ids per XCD, then a grouped (4 row tiles) raster so the
    // ~32 co-resident tiles of one XCD share 4 A panels and 8 B panels in its L2.
    const unsigned nwg = gridDim.x, bid = blockIdx.x;
    const unsigned xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    constexpr unsigned GM = 4;
    const unsigned grp = wgid / (GM * g.ntiles);
    const unsigned gm = min(GM, g.mtiles - grp * GM);
    const unsigned idx = wgid - grp * GM * g.ntiles;
    const unsigned tm = grp * GM + idx % gm, tn = idx / gm;

    // LDS-DMA pieces of this wave: 1 KiB blocks {wave, wave + 8} of the A and of the B panel
    const int8_t *Ag = g.A + j * g.planeA + sb * g.subA + ((size_t)tm * g.kstride + g.k0) * PANEL + wave * 1024 + lane * 16;
    const int8_t *Bg = g.B + j * g.planeB + sb * g.subB + ((size_t)tn * g.kstride + g.k0) * PANEL + wave * 1024 + lane * 16;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int8_t *)smem;
    const uint32_t lds_wave = lds_base + wave * 1024;
    const v4si rA = make_rsrc(g.A + j * g.planeA, (uint32_t)g.planeA);
    const v4si rB = make_rsrc(g.B + j * g.planeB, (uint32_t)g.planeB);
    const uint32_t oA = (uint32_t)(sb * g.subA + ((size_t)tm * g.kstride + g.k0) * PANEL) + wave * 1024 + lane * 16;
    const uint32_t oB = (uint32_t)(sb * g.subB + ((size_t)tn * g.kstride + g.k0) * PANEL) + wave * 1024 + lane * 16;
    auto stage = [&](unsigned ks, unsigned slot) {
        const size_t go = (size_t)(OZ2_ABLATE == 8 ? (ks & 1) : ks) * PANEL;  // 8: two k-steps only (all L2 hits)
        const uint32_t lo = lds_wave + slot * SLOT;
        if constexpr (BUF) {
            const uint32_t g32 = (uint32_t)go;
            bglds16(rA, oA + g32, lo);
            bglds16(rA, oA + g32 + 8192, lo + 8192);
            bglds16(rB, oB + g32, lo + PANEL);
            bglds16(rB, oB + g32 + 8192, lo + PANEL + 8192);
        } else {
            glds16(Ag + go, lo);
            glds16(Ag + go + 8192, lo + 8192);
            glds16(Bg + go, lo + PANEL);
            glds16(Bg + go + 8192, lo + PANEL + 8192);
        }
    };

    AccTile acc[ACC_I][ACC_J];
    const int acc0 = ((EPI == (int)Epi::RESIDUE || EPI == EPI_RESIDUE_ADD) && g.biased) ? g.bias[j] : 0;
#pragma unroll
    for (int i = 0; i < ACC_I; ++i)
#pragma unroll
        for (int jj = 0; jj < ACC_J; ++jj) acc[i][jj] = AccTile{} + acc0;  // splat

    const unsigned K = g.ksteps;
    constexpr unsigned D = STAGES - 1;  // prefetch distance in k-steps
    static_assert(D >= 2 && D <= 5, "drain-loop vmcnt cases cover prefetch distances 2..5");
    if (K > 0) {
        // prologue: steps 0..D-1 in flight, step 0 landed for every wave, then group 1 falls one
        // barrier behind.  Barrier accounting (the same for both groups): 1 + 2K + 1 before the epilogue.
        for (unsigned s0 = 0; s0 < D; ++s0)
            if (s0 < K) stage(s0, s0);
        if (K >= D) wait_vm_lgkm0<GLDS_PER_STEP *(D - 1)>();
        else wait_steps_lgkm0<GLDS_PER_STEP>((int)K - 1);
        barrier();
        if (wr == 1) barrier();

        // Step t, per wave: load interval (reads of slot t%S, DMA of step t+D into the slot of
        // step t-1, wait until step t+1 landed and the reads returned), barrier, MFMA interval,
        // barrier.  RAW: every wave retires its part of step t+1 before the barrier that ends its
        // load interval of step t; the first read of step t+1 (group 0) follows group 1's next
        // barrier.  WAR: the slot of step t-1 was last read by group 1 in its previous load
        // interval, which waited lgkmcnt(0) before its barrier.
        Frags f;
        unsigned slot_cur = 0, slot_issue = D % STAGES;
        unsigned t = 0;
        if (OZ2_ABLATE == 6 && K > D) {  // probe: every ring slot filled once, no DMA in the loop
            stage(D, D % STAGES);
            wait_vm_lgkm0<0>();
            barrier();
        }
        for (; t + D < K; ++t) {  // steady state
            if (OZ2_ABLATE != 5 || t == 0) read_frags(f, smem + slot_cur * SLOT, wr, wc, lane);  // 5: reads once
            __builtin_amdgcn_sched_barrier(0);
            if (OZ2_ABLATE != 6) stage(t + D, slot_issue);
            wait_vm_lgkm0<GLDS_PER_STEP *(D - 1)>();
            barrier();
            mfma_step(acc, f);
            barrier();
            slot_cur = slot_cur == STAGES - 1 ? 0 : slot_cur + 1;
            slot_issue = slot_issue == STAGES - 1 ? 0 : slot_issue + 1;
        }
        for (; t < K; ++t) {  // drain: nothing left to stage
            read_frags(f, smem + slot_cur * SLOT, wr, wc, lane);
            __builtin_amdgcn_sched_barrier(0);
            wait_steps_lgkm0<GLDS_PER_STEP>(t + 2 < K ? (int)(K - t - 2) : 0);  // steps t+2..K-1 may fly
            barrier();
            mfma_step(acc, f);
            barrier();
            slot_cur = slot_cur == STAGES - 1 ? 0 : slot_cur + 1;
        }
        if (wr == 0) barrier();
    }
    barrier();  // all waves done with the ring before the epilogue reuses it

    if (OZ2_ABLATE == 10) {  // probe: no epilogue
#pragma unroll
        for (int i = 0; i < ACC_I; ++i)
#pragma unroll
            for (int jj = 0; jj < ACC_J; ++jj) asm volatile("" ::"v"(acc[i][jj]));
        return;
    }
    epilogue<EPI>(g, acc, smem, tid, lane, wr, wc, tm, tn, j, sb, true);
}

// ---------------------------------------------------------------------------------------------
// Small-launch form (round 6): 128 x 128 output tiles, 256 threads = 4 waves (2 x 2, one per SIMD, each 64 x 64 =
// 4 x 4 tiles of 16 x 16), a 4-slot ring of 16 KiB k-steps (64 KiB: two blocks per CU).  For launches with few
// 256 x 256 tiles per CU (1024^3: 224 tiles on 256 CUs, the accurate-mode bound product of a 1024^2 or 2048^2
// problem: 16 or 64 tiles) the 256-tile kernels leave CUs idle and expose each block's first-data latency and
// epilogue; four times the blocks, two co-resident per CU, hide one block's epilogue and DMA waits under the
// other's MFMAs.  The operand panels are the same 256-vector panels: a 128-row half is blocks 4h..4h+3 of both
// 32-deep halves (two 4 KiB runs per panel), staged by LDS-DMA as 16 pieces of 1 KiB per k-step (4 per wave).
// Per k-step and wave: wait (step t+1 landed, fragments of t in registers), barrier, fragment reads of t+1,
// LDS-DMA of t+4 into the slot of t, 16 MFMAs of t -- the reads of the next step run under this step's MFMAs.
constexpr int SM_THREADS = 256;
constexpr int SM_SLOT = PANEL;           // 8 KiB A half-panel + 8 KiB B half-panel
constexpr int SM_STAGES = 4;
constexpr int SM_LDS = SM_STAGES * SM_SLOT;  // 64 KiB
struct SmFrags {
    v4i a[4];
    v4i b[4];
};
// the half-panel in LDS: [s:2][blk:4][h:2][r:32][16 B] (4 KiB per s); lane l = r16 + 16 q reads the 16 k-bytes
// 16 q.. of vector r16 of a 16-row group, as read_frags
__device__ __forceinline__ void sm_read_frags(SmFrags &f, const int8_t *slot, int wr, int wc, int lane) {
    const int q = lane >> 4;
    const int8_t *base = slot + (q >> 1) * 4096 + ((q & 1) * 32 + (lane & 15)) * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i)  // rows 16 i.. of the wave's 64: block wr*2 + i/2, half i&1
        f.a[i] = *reinterpret_cast<const v4i *>(base + (wr * 2 + (i >> 1)) * 1024 + (i & 1) * 256);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
        f.b[jj] = *reinterpret_cast<const v4i *>(base + 8192 + (wc * 2 + (jj >> 1)) * 1024 + (jj & 1) * 256);
}
__device__ __forceinline__ void sm_mfma(v4i (&acc)[4][4], const SmFrags &f) {
#pragma unroll
    for (int x = 0; x < 16; ++x) {
        const int i = x >> 2, jj = x & 3;
        acc[i][jj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[i], f.b[jj], acc[i][jj], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int EPI, bool SUB = false>
__global__ __launch_bounds__(SM_THREADS, 2) void gemm_i8_small_kernel(GemmArgs g) {
    static_assert(OZ2_MFMA16, "small tiles: 16x16x64 accumulator map");
    __shared__ __attribute__((aligned(1024))) int8_t smem[SM_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const unsigned j = SUB ? blockIdx.y / 3 : blockIdx.y;
    const unsigned sb = SUB ? blockIdx.y - 3 * j : 0;

    // XCD-aware bijective remap (as gemm_i8_kernel), grouped raster of 8 row tiles: the ~64 co-resident tiles
    // of an XCD (two per CU) share 8 A and 8 B half-panels
    const unsigned mt2 = 2 * g.mtiles, nt2 = 2 * g.ntiles;
    const unsigned nwg = gridDim.x, bid = blockIdx.x;
    const unsigned xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    constexpr unsigned GM = 8;
    const unsigned grp = wgid / (GM * nt2);
    const unsigned gm = min(GM, mt2 - grp * GM);
    const unsigned idx = wgid - grp * GM * nt2;
    const unsigned tm2 = grp * GM + idx % gm, tn2 = idx / gm;
    const unsigned tm = tm2 >> 1, hm = tm2 & 1, tn = tn2 >> 1, hn = tn2 & 1;

    // this wave's LDS-DMA pieces: A and B pieces w (s = 0) and w + 4 (s = 1) of the half-panels
    const v4si rA = make_rsrc(g.A + j * g.planeA, (uint32_t)g.planeA);
    const v4si rB = make_rsrc(g.B + j * g.planeB, (uint32_t)g.planeB);
    const uint32_t oA = (uint32_t)(sb * g.subA + ((size_t)tm * g.kstride + g.k0) * PANEL) + (4 * hm + wave) * 1024 + lane * 16;
    const uint32_t oB = (uint32_t)(sb * g.subB + ((size_t)tn * g.kstride + g.k0) * PANEL) + (4 * hn + wave) * 1024 + lane * 16;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int8_t *)smem;
    const uint32_t lds_wave = lds_base + wave * 1024;
    auto stage = [&](unsigned ks) {
        const uint32_t go = ks * (uint32_t)PANEL, lo = lds_wave + (ks & (SM_STAGES - 1)) * SM_SLOT;
        bglds16(rA, oA + go, lo);
        bglds16(rA, oA + go + 8192, lo + 4096);
        bglds16(rB, oB + go, lo + 8192);
        bglds16(rB, oB + go + 8192, lo + 8192 + 4096);
    };

    v4i acc[4][4];
    const int acc0 = ((EPI == (int)Epi::RESIDUE) && g.biased) ? g.bias[j] : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = v4i{} + acc0;

    const unsigned K = g.ksteps;
    SmFrags fa, fb;
    if (K > 0) {
        // prologue: steps 0..3 in flight (the ring's four slots), step 0 landed, its fragments read
        for (unsigned s0 = 0; s0 < SM_STAGES; ++s0)
            if (s0 < K) stage(s0);
        wait_steps_lgkm0<GLDS_PER_STEP>((int)min(K, (unsigned)SM_STAGES) - 1);
        barrier();
        sm_read_frags(fa, smem, wr, wc, lane);
        for (unsigned t = 0; t < K; t += 2) {
            // step t (fragments in fa): wait for step t+1 (steps t+2, t+3 may fly) and fa, barrier, read t+1,
            // stage t+4 into the slot of t, MFMAs of t; then the same for t+1 with fa / fb swapped
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const unsigned tt = t + u;
                if (tt >= K) break;
                SmFrags &cur = u == 0 ? fa : fb, &nxt = u == 0 ? fb : fa;
                const int fly = (int)min(K - 1 - min(tt + 1, K - 1), 2u);  // steps younger than tt+1 in flight
                wait_steps_lgkm0<GLDS_PER_STEP>(fly);
                barrier();
                if (tt + 1 < K) sm_read_frags(nxt, smem + ((tt + 1) & (SM_STAGES - 1)) * SM_SLOT, wr, wc, lane);
                __builtin_amdgcn_sched_barrier(0);
                if (tt + SM_STAGES < K) stage(tt + SM_STAGES);
                sm_mfma(acc, cur);
            }
        }
    }
    barrier();  // every wave's MFMAs issued and its reads of the ring done: the epilogue reuses slot 0

    if constexpr (EPI == (int)Epi::RESIDUE) {
        const int p = g.p[j];
        uint32_t *park = reinterpret_cast<uint32_t *>(smem);  // [128 cols][32 dwords], swizzled as the pg kernel
        auto park_all = [&](auto &&res) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int col = wc * 64 + acc_col(jj, lane), q = lane >> 4, c = wr * 4 + i;
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w |= res(acc[i][jj][e]) << (8 * e);
                    park[col * 32 + ((c ^ ((col >> 1) & 7)) << 2) + (q ^ ((col & 1) << 1))] = w;
                }
        };
        if (g.biased && p == 256) {
            park_all([&](int x) { return (uint32_t)x & 0xffu; });
        } else if (g.biased) {
            const double invp = g.invp[j], pneg = -(double)p;
            const double cneg = __builtin_fma(-0x1p52, invp, 0x1p-8);
            park_all([&](int x) { return residue_biased_f64((uint32_t)x, invp, cneg, pneg); });
        } else {
            const int bar = g.barrett[j];
            const bool p256 = (p == 256);
            park_all([&](int x) { return residue(x, p, bar, p256); });
        }
        __syncthreads();
        uint8_t *out = static_cast<uint8_t *>(g.out) + j * g.planeOut + sb * g.subOut + (size_t)tn2 * 128 * g.ldo +
                       (size_t)tm2 * 128;
#pragma unroll
        for (int it = 0; it < 4; ++it) {  // 128 columns x 8 chunks of 16 B
            const int chunk = tid + SM_THREADS * it;
            const int col = chunk >> 3, c = chunk & 7;
            const uint4 v = *reinterpret_cast<const uint4 *>(park + col * 32 + ((c ^ ((col >> 1) & 7)) << 2));
            const int pm = (col & 1) << 1;
            const uint32_t e[4] = {v.x, v.y, v.z, v.w};
            *reinterpret_cast<uint4 *>(out + (size_t)col * g.ldo + 16 * c) = make_uint4(e[0 ^ pm], e[1 ^ pm], e[2 ^ pm], e[3 ^ pm]);
        }
    } else if constexpr (EPI == (int)Epi::BOUND) {
        int32_t *rmax = reinterpret_cast<int32_t *>(smem);
        int32_t *cmax = rmax + 128;
        rmax[tid & 127] = 0;  // (threads 0-127 and 128-255 write the same zeros)
        cmax[tid & 127] = 0;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                int v = 0;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) v = max(v, abs(acc[i][jj][rr]));
#pragma unroll
                for (int d = 8; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 16));
                if ((lane & 15) == 0) atomicMax(&rmax[wr * 64 + acc_row(i, rr, lane)], v);
            }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            int v = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) v = max(v, abs(acc[i][jj][rr]));
#pragma unroll
            for (int d = 16; d < 64; d <<= 1) v = max(v, __shfl_xor(v, d));
            if (lane < 16) atomicMax(&cmax[wc * 64 + acc_col(jj, lane)], v);
        }
        __syncthreads();
        if (tid < 128) atomicMax(&g.rowmax[tm2 * 128 + tid], rmax[tid]);
        else atomicMax(&g.colmax[tn2 * 128 + tid - 128], cmax[tid - 128]);
    }
}

// ---------------------------------------------------------------------------------------------
// Persistent form of the residue product (buffer DMA; real operands and Karatsuba sub-products).
// One block per CU.  The k-steps of a block's consecutive tiles form ONE pipeline: the LDS-DMA
// runs D steps ahead across tile boundaries, so the next tile's first panels land while the
// current tile finishes and its epilogue runs (the one-tile kernel pays that first-data latency,
// the block teardown and the next block's launch once per tile).  The epilogue parks the residues
// in the ring slot of the tile's last step plus a spare 32 KiB and issues the 8 residue stores per
// wave without waiting for them: they stay in flight under the next tile's first two k-steps (the
// vmcnt waits there count them as younger than the awaited DMA; from the third step on they are
// older and complete first).
// Tiles come from one queue per XCD (head counters zeroed before the launch), in the order the
// hardware dispatcher hands the one-tile kernel's blocks to that XCD: plane by plane, the XCD's
// contiguous share of each plane's grouped raster.  So the ~32 tiles in flight on an XCD are always
// neighbours and share 4 A and 8 B panels in its L2.  (A static tile list per block was measured:
// the blocks drift apart over the launch and the L2 hit rate fell from 79 % to 69 %.)  The first
// tile of a block is its slot on the XCD, the second is dequeued at the start, every later one in
// the epilogue two tiles ahead, so the DMA cursor always knows the tile it runs into.
constexpr int PSTAGES = 4;                   // the persistent kernel's ring (its vmcnt bookkeeping assumes 4)
constexpr int PLDS_BYTES = PSTAGES * SLOT;
constexpr int PARK_SPARE = 32768;
constexpr int PARK_STORES = 4096 / NTHREADS;  // 16-byte residue stores per thread (and per wave) per tile
constexpr unsigned NO_TILE = 0xffffffffu;

struct TileRef {
    unsigned j, sb, tm, tn;
    uint32_t offA, offB;  // byte offsets of the tile's first staged k-step panel in its modulus's A and B planes
    uint32_t step;        // byte step of the DMA cursor from one k-step to the next (PANEL, or -PANEL mod 2^32)
};

template <bool SUB> __device__ __forceinline__ TileRef decode_tile(const GemmArgs &g, unsigned u) {
    constexpr unsigned GM = 4;
    const unsigned P = g.mtiles * g.ntiles;
    const unsigned y = u / P, v = u - y * P;
    TileRef t;
    t.j = SUB ? y / 3 : y;
    t.sb = SUB ? y - 3 * t.j : 0;
    const unsigned grp = v / (GM * g.ntiles);
    const unsigned gm = min(GM, g.mtiles - grp * GM);
    const unsigned idx = v - grp * GM * g.ntiles;
    t.tm = grp * GM + idx % gm;
    t.tn = idx / gm;
    t.offA = (uint32_t)(t.sb * g.subA + (size_t)t.tm * g.kstride * PANEL);
    t.offB = (uint32_t)(t.sb * g.subB + (size_t)t.tn * g.kstride * PANEL);
    // block-uniform: keep them in SGPRs (the compiler's divergence analysis does not see it)
    t.j = __builtin_amdgcn_readfirstlane(t.j);
    t.sb = __builtin_amdgcn_readfirstlane(t.sb);
    t.tm = __builtin_amdgcn_readfirstlane(t.tm);
    t.tn = __builtin_amdgcn_readfirstlane(t.tn);
    t.offA = __builtin_amdgcn_readfirstlane(t.offA);
    t.offB = __builtin_amdgcn_readfirstlane(t.offB);
    return t;
}

// PRIO: 1 (default) = static priority 1 for waves 4-7, the younger half (one barrier behind), which
// otherwise loses every issue arbitration to its older partner (MI355X_MICROARCH.md, two waves per
// SIMD, item 4); 0 = priority 1 around every MFMA interval (as the one-tile kernel); 2 = no priority
// changes.  Measured in one process (tools/probes/persist_prio.hip, random bytes): 1 and 2 are
// 0.3-0.8 % faster than 0 at 8192^3, 4096^3 and 8192^2 x 1024, with identical residues.
// EPIM (A/B probes): 0 = the f64 form of the biased residue (default; residue_biased_f64, the low byte
// for p = 256), 1 = the low byte only (wrong residues: the cost of the reduction), 2 = the integer form
// (residue_biased).  Measured in one process (tools/probes/persist_epim.hip): the reduction costs 2 % of
// the cfg2 products and 6-10 % at k = 1024-2048; the f64 form is 0.5-1 % faster than the integer one.
#ifndef OZ2_STAMPS
#define OZ2_STAMPS 0  // probe builds only (tools/probes/persist_stamps.hip): s_memtime phase sums per wave
#endif
// ORD (A/B probes): 0 = every tile walks k ascending (default); 1 = serpentine: the tiles of every other round of
// a queue (queue position / blocks per queue odd) walk k descending, so a round's first k-steps read the A panels
// its predecessor round (same row tiles, the next column tiles) read last, while they may still sit in the XCD's
// L2.  Integer sums in any order: identical residues.
template <bool SUB, int PRIO = 1, int EPIM = 0, int ORD = 0>
__global__ __launch_bounds__(NTHREADS, 1) void gemm_i8_persistent_kernel(GemmArgs g) {
#if OZ2_STAMPS
    // [0] realign, [1] residues -> LDS, [2] park barrier, [3] stores + barrier, [4] accumulator reset +
    // stagger, [5] step 0, [6] step 1, [7] the other k-steps, [8] tiles
    unsigned long long st_acc[9] = {};
    unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#define OZ2_STAMP(slot)                                                  \
    do {                                                                 \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();      \
        st_acc[slot] += _t - t_prev;                                     \
        t_prev = _t;                                                     \
    } while (0)
#else
#define OZ2_STAMP(slot) \
    do {                \
    } while (0)
#endif
    __shared__ __attribute__((aligned(1024))) int8_t smem[PLDS_BYTES + PARK_SPARE];
    static_assert(PLDS_BYTES + PARK_SPARE <= 160 * 1024, "LDS");
    static_assert(PSTAGES == 4 && GLDS_PER_STEP == 4 && PARK_STORES == 8, "vmcnt bookkeeping below assumes these");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    uint32_t *const spare = reinterpret_cast<uint32_t *>(smem + PLDS_BYTES);
    if (PRIO == 1 && wr == 1) __builtin_amdgcn_s_setprio(1);

    // this block's XCD queue: the XCD's share of every plane (the one-tile kernel's remap)
    const unsigned G = gridDim.x, bid = blockIdx.x, xcd = bid & 7;
    const unsigned nblk = (G >> 3) + (xcd < (G & 7) ? 1u : 0u);  // blocks serving this queue
    const unsigned P = g.mtiles * g.ntiles, q8 = P >> 3, r8 = P & 7;
    const unsigned tx = q8 + (xcd < r8 ? 1u : 0u);
    const unsigned basex = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
    const unsigned total = g.nplanes * tx;
    auto tile_u = [&](unsigned i) {
        const unsigned y = __builtin_amdgcn_readfirstlane(i / tx);
        return y * P + basex + (i - y * tx);
    };
    auto claim = [&]() {  // raw queue position; the tile is (position + nblk) if below total
        return __hip_atomic_fetch_add(g.queue + xcd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto to_tile = [&](unsigned pos) { return pos + nblk < total ? pos + nblk : NO_TILE; };
    unsigned ccur = (bid >> 3) < total ? (bid >> 3) : NO_TILE;
    if (ccur == NO_TILE) return;  // block-uniform, before any barrier
    if (tid == 0) spare[0] = to_tile(claim());

    // K >= 6 (host): the DMA cursor jumps to the next tile after staging this tile's last step, at
    // k = K - 4, which must come after steps 0 and 1, where a block's later tiles learn their successor
    // (with K = 5 the jump read the successor's offsets before they were decoded)
    const unsigned K = g.ksteps;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int8_t *)smem;
    const uint32_t lds_wave = lds_base + wave * 1024;
    const uint32_t lane_off = wave * 1024 + lane * 16;
    // buffer descriptors of one modulus's A and B planes (each < 4 GiB; the launch's planes together
    // may exceed it): the DMA switches to the successor tile's descriptors with its cursor
    auto rsrcA = [&](const TileRef &t) { return make_rsrc(g.A + (size_t)t.j * g.planeA, (uint32_t)g.planeA); };
    auto rsrcB = [&](const TileRef &t) { return make_rsrc(g.B + (size_t)t.j * g.planeB, (uint32_t)g.planeB); };
    auto lo_of = [&](unsigned step) { return lds_wave + (step & (PSTAGES - 1)) * SLOT; };
    auto rd_of = [&](unsigned step) { return smem + (step & (PSTAGES - 1)) * SLOT; };

    auto ref_of = [&](unsigned pos) {  // the tile at queue position pos, with its k direction
        TileRef t = decode_tile<SUB>(g, tile_u(pos));
        t.step = PANEL;
        if (ORD == 1 && ((pos / nblk) & 1u)) {
            t.offA += (K - 1) * PANEL;
            t.offB += (K - 1) * PANEL;
            t.step = 0u - (uint32_t)PANEL;
        }
        return t;
    };
    TileRef ct = ref_of(ccur);
    v4si rA = rsrcA(ct), rB = rsrcB(ct);  // descriptors of the DMA cursor
    uint32_t cstep = ct.step;             // and its step
    constexpr unsigned D = PSTAGES - 1;
    for (unsigned s0 = 0; s0 < D; ++s0) {  // steps 0..2 of the first tile
        const uint32_t lo = lo_of(s0);
        bglds16(rA, ct.offA + s0 * cstep + lane_off, lo);
        bglds16(rA, ct.offA + s0 * cstep + lane_off + 8192, lo + 8192);
        bglds16(rB, ct.offB + s0 * cstep + lane_off, lo + PANEL);
        bglds16(rB, ct.offB + s0 * cstep + lane_off + 8192, lo + PANEL + 8192);
    }
    wait_vm_lgkm0<GLDS_PER_STEP *(D - 1)>();  // step 0 landed (and the claim's LDS write)
    barrier();

    unsigned s = 0;                                             // global k-step of this block (slot s mod 4)
    unsigned cnext = __builtin_amdgcn_readfirstlane(spare[0]);  // the tile after the current one
    uint32_t da = ct.offA + D * cstep, db = ct.offB + D * cstep;  // DMA cursor: panels of the next step staged
    Frags f;
    AccTile acc[ACC_I][ACC_J];
    for (unsigned r = 0;; ++r) {
        const int acc0 = g.biased ? g.bias[ct.j] : 0;
#pragma unroll
        for (int i = 0; i < ACC_I; ++i)
#pragma unroll
            for (int jj = 0; jj < ACC_J; ++jj) acc[i][jj] = AccTile{} + acc0;
        if (wr == 1) barrier();  // group 1 falls one barrier behind (ping-pong, as in the one-tile kernel)
        OZ2_STAMP(4);
        unsigned k = 0;
        uint32_t na = 0, nb = 0, nstep = PANEL;  // the next tile's first panels and its step
        v4si nrA = rA, nrB = rB;  // and its descriptors
        // one k-step: reads of slot s, DMA of step s+3 (this tile's step k+3, or the next tile's step
        // k+3-K once k+3 >= K: the cursor jumps there after staging this tile's last step), wait, MFMAs
        auto step = [&](auto wait) {
            read_frags(f, rd_of(s), wr, wc, lane);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t lo = lo_of(s + D);
            bglds16(rA, da + lane_off, lo);
            bglds16(rA, da + lane_off + 8192, lo + 8192);
            bglds16(rB, db + lane_off, lo + PANEL);
            bglds16(rB, db + lane_off + 8192, lo + PANEL + 8192);
            const bool jump = k + D + 1 == K;
            da = jump ? na : da + cstep;
            db = jump ? nb : db + cstep;
            if (jump) {  // block-uniform
                rA = nrA;
                rB = nrB;
                cstep = nstep;
            }
            wait();
            barrier();
            mfma_step<PRIO>(acc, f);
            barrier();
        };
        if (r > 0) {
            // steps 0 and 1: the previous tile's 8 residue stores are younger than the awaited DMA
            step([] { wait_vm_lgkm0<GLDS_PER_STEP *(D - 1) + PARK_STORES>(); });
            ++k, ++s;
            OZ2_STAMP(5);
            step([] { wait_vm_lgkm0<GLDS_PER_STEP *(D - 1) + PARK_STORES>(); });
            ++k, ++s;
            OZ2_STAMP(6);
            cnext = __builtin_amdgcn_readfirstlane(spare[0]);  // written by wave 0 two barriers ago
        }
        TileRef nt = ct;
        if (cnext != NO_TILE) {
            nt = ref_of(cnext);
            na = nt.offA;
            nb = nt.offB;
            nstep = nt.step;
            nrA = rsrcA(nt);
            nrB = rsrcB(nt);
        }
        // steady steps; the block's last tile stops staging three steps before its end
        const unsigned kend = cnext != NO_TILE ? K : K - D;
        for (; k < kend; ++k, ++s) step([] { wait_vm_lgkm0<GLDS_PER_STEP *(D - 1)>(); });
        for (; k < K; ++k, ++s) {  // drain of the block's last tile
            read_frags(f, rd_of(s), wr, wc, lane);
            __builtin_amdgcn_sched_barrier(0);
            wait_steps_lgkm0<GLDS_PER_STEP>(k + 2 < K ? (int)(K - k - 2) : 0);  // steps k+2..K-1 may fly
            barrier();
            mfma_step<PRIO>(acc, f);
            barrier();
        }
        OZ2_STAMP(7);
        if (wr == 0) barrier();  // realign the groups
        barrier();
        OZ2_STAMP(0);

        // epilogue: the tile after next is claimed first (its latency hides under the residue
        // arithmetic), residues -> LDS (columns 0..127 in the slot of the tile's last step, 128..255
        // in the spare), then 16-byte column stores; the ring slot is reused by the DMA of step
        // s+3, issued after the closing barrier
        unsigned pos = 0;
        const bool claiming = tid == 0 && cnext != NO_TILE;
        if (claiming) pos = claim();
        // per-thread epilogue addresses derive from this copy of the thread index, opaque to the
        // compiler, so they are recomputed per tile instead of hoisted out of the tile loop (held
        // across the main loop they spilled, and the spill reloads' vmcnt waits then serialised the
        // residue stores)
        int etid = tid;
        asm volatile("" : "+v"(etid));
        const int elane = etid & 63;
        const int p = g.p[ct.j];
        uint32_t *parkA = reinterpret_cast<uint32_t *>(rd_of(s - 1));
        uint32_t *parkB = spare;
        uint32_t *lo = wc < 2 ? parkA : parkB;  // this wave's 64 columns lie in one half
        auto park = [&](auto &&res) {
#pragma unroll
            for (int i = 0; i < ACC_I; ++i)
#pragma unroll
                for (int jj = 0; jj < ACC_J; ++jj) {
                    const int col = wc * 64 + acc_col(jj, elane);
#pragma unroll
                    for (int gq = 0; gq < ACC_E / 4; ++gq) {
                        uint32_t w = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e) w |= res(acc[i][jj][4 * gq + e]) << (8 * e);
                        const int rdw = (wr * 128 + acc_row(i, 4 * gq, elane)) >> 2;
                        lo[(col & 127) * 64 + (rdw ^ (col & 31))] = w;
                    }
                }
        };
        if (EPIM == 1 || (g.biased && p == 256)) {  // (EPIM 1: probe ablation) p = 256: bias is a multiple of 256
            park([&](int x) { return (uint32_t)x & 0xffu; });
        } else if (EPIM == 0 && g.biased) {
            const double invp = g.invp[ct.j], pneg = -(double)p;
            const double cneg = __builtin_fma(-0x1p52, invp, 0x1p-8);
            park([&](int x) { return residue_biased_f64((uint32_t)x, invp, cneg, pneg); });
        } else if (EPIM == 3 && g.biased) {
            const double invp = g.invp[ct.j], pneg = -(double)p;
            const double chalf = __builtin_fma(-0x1p52, invp, 0x1p-8) - 0.5;
            park([&](int x) { return residue_biased_f64r((uint32_t)x, invp, chalf, pneg); });
        } else if (EPIM == 4 && g.biased) {
            const double invp = g.invp[ct.j];
            const double chalf = __builtin_fma(-0x1p52, invp, 0x1p-8) - 0.5;
            park([&](int x) { return residue_biased_f64i((uint32_t)x, invp, chalf, (uint32_t)p); });
        } else if (g.biased) {
            const uint32_t m = g.minv[ct.j];
            park([&](int x) { return residue_biased((uint32_t)x, (uint32_t)p, m); });
        } else {
            const int bar = g.barrett[ct.j];
            const bool p256 = (p == 256);
            park([&](int x) { return residue(x, p, bar, p256); });
        }
        OZ2_STAMP(1);
        __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0), vmcnt untouched
        barrier();
        OZ2_STAMP(2);
        uint8_t *out = static_cast<uint8_t *>(g.out) + ct.j * g.planeOut + ct.sb * g.subOut +
                       (size_t)ct.tn * 256 * g.ldo + (size_t)ct.tm * 256;
#pragma unroll
        for (int it = 0; it < PARK_STORES; ++it) {
            const int chunk = etid + NTHREADS * it;
            const int col = chunk >> 4, qd = chunk & 15;
            const int x = col & 31;
            const uint32_t *src = it < PARK_STORES / 2 ? parkA : parkB;
            const uint4 v = *reinterpret_cast<const uint4 *>(src + (col & 127) * 64 + ((4 * qd) ^ (x & ~3)));
            const uint32_t e[4] = {v.x, v.y, v.z, v.w};
            const int pm = x & 3;
            if (OZ2_RES_NTS) {
                typedef unsigned u4v __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(u4v{e[0 ^ pm], e[1 ^ pm], e[2 ^ pm], e[3 ^ pm]},
                                            reinterpret_cast<u4v *>(out + (size_t)col * g.ldo + 16 * qd));
            } else {
                *reinterpret_cast<uint4 *>(out + (size_t)col * g.ldo + 16 * qd) =
                    make_uint4(e[0 ^ pm], e[1 ^ pm], e[2 ^ pm], e[3 ^ pm]);
            }
        }
        __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));  // park reads done
        barrier();
        OZ2_STAMP(3);
#if OZ2_STAMPS
        st_acc[8] += 1;
#endif
        if (tid == 0) spare[0] = claiming ? to_tile(pos) : NO_TILE;  // read at the next tile's k = 1
        if (cnext == NO_TILE) break;
        ct = nt;
    }
#if OZ2_STAMPS
    if (lane == 0 && g.stamps)
        for (int i = 0; i < 9; ++i) g.stamps[((size_t)blockIdx.x * 8 + wave) * 9 + i] = st_acc[i];
#endif
#undef OZ2_STAMP
}

// ---------------------------------------------------------------------------------------------
// Persistent residue product with PER-GROUP epilogues (round 6; the default, GEMMUL8_PG_EPILOGUE=0 selects
// gemm_i8_persistent_kernel above).  The same DMA pipeline, tile queues and
// main loop as gemm_i8_persistent_kernel, but the two wave groups (rows 0-127 / 128-255 of the tile) stay one
// barrier apart for the whole launch: no realignment around the epilogue.  Each group parks and stores its
// own 128 rows right after its own last MFMA interval, so per SIMD the intervals pair as
//     group 0:  ... M(K-1) | park | store | L'(0) | M'(0) ...
//     group 1:  ... L(K-1) | M(K-1) | park | store | L'(0) ...
// (L = fragment reads + DMA issue, M = MFMAs; ' = the next tile): group 0's park runs beside group 1's last
// MFMAs, and the two epilogues overlap each other instead of following each other with the whole block
// waiting at four barriers.  Per tile each group passes 2K + 2 barriers.
// Measured in one process against the block-epilogue kernel (tools/probes/persist_pg_ab.hip, profiles/r06/epilogue_ab/):
// with the park layout below, 0.5-1.2 % shorter at cfg2's shape and 2-5 % at k = 1024 (per-tile overhead 6.2-6.3
// against 6.7-7.7 k-step equivalents, three runs on two boxes; the first layout, with XOR addresses per write and
// a dword permutation per read-back, was neutral); identical residues.
// Group 0 parks in the ring slot of the tile's last step (its next writer is group 0's own DMA of the next
// tile's step 3, issued in L'(0) after its store sweep has read the slot back), group 1 in the spare 32 KiB.
// The accumulators are not reset: the first MFMA of each tile reads its C operand from a splat of the
// tile's bias (or 0) and writes the accumulator, i.e. no 128 v_mov per wave and tile.
// The tile after next is claimed by thread 0 at the start of group 0's park; it is published in the spare's
// first dword during group 0's MFMA interval of the next tile's step 0 (group 1 has read its parked
// residues back by then) and read by every wave after step 1, as before.
// Park layout of a group's 128 x 256 residue block: [256 cols][32 dwords], dword d = 4 consecutive rows
// 4d..4d+3; the 16-byte chunk c = d >> 2 of column col sits at chunk position c ^ ((col >> 1) & 7) and its
// dword q at (q ^ 2 (col & 1)): conflict-free ds_write_b32 of a 16 x 16 accumulator tile (32 lanes, 32 banks)
// and ds_read_b128 of 8 columns x 128 B per wave.
__device__ __forceinline__ void mfma_step_first(AccTile (&acc)[ACC_I][ACC_J], const Frags &f, const v4i c) {
#pragma unroll
    for (int x = 0; x < 32; ++x) {
        const int i = x >> 2, jj = x & 3;
        acc[i][jj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[i], f.b[jj], c, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// ABL (probe builds, tools/probes/persist_pg_ab.hip): 1 = residues reduced to the low byte (wrong residues), 2 = no
// residue stores, 3 = neither park nor stores (the epilogue's barriers only)
#ifndef OZ2_PG_CLAIM_EARLY
#define OZ2_PG_CLAIM_EARLY 0
#endif
#ifndef OZ2_PG_STATIC2
#define OZ2_PG_STATIC2 1
#endif
template <bool SUB, int PRIO = 1, int ABL = 0>
__global__ __launch_bounds__(NTHREADS, 1) void gemm_i8_persistent_pg_kernel(GemmArgs g) {
    static_assert(OZ2_MFMA16, "per-group epilogue: 16x16x64 accumulator map");
    __shared__ __attribute__((aligned(1024))) int8_t smem[PLDS_BYTES + PARK_SPARE];
    static_assert(PLDS_BYTES + PARK_SPARE <= 160 * 1024, "LDS");
    static_assert(PSTAGES == 4 && GLDS_PER_STEP == 4 && PARK_STORES == 8, "vmcnt bookkeeping below assumes these");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    uint32_t *const spare = reinterpret_cast<uint32_t *>(smem + PLDS_BYTES);
    if (PRIO == 1 && wr == 1) __builtin_amdgcn_s_setprio(1);

    const unsigned G = gridDim.x, bid = blockIdx.x, xcd = bid & 7;
    const unsigned nblk = (G >> 3) + (xcd < (G & 7) ? 1u : 0u);
    const unsigned P = g.mtiles * g.ntiles, q8 = P >> 3, r8 = P & 7;
    const unsigned tx = q8 + (xcd < r8 ? 1u : 0u);
    const unsigned basex = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
    const unsigned total = g.nplanes * tx;
    auto tile_u = [&](unsigned i) {
        const unsigned y = __builtin_amdgcn_readfirstlane(i / tx);
        return y * P + basex + (i - y * tx);
    };
    auto claim = [&]() { return __hip_atomic_fetch_add(g.queue + xcd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    // queue positions count from the block's third tile when the second is static (OZ2_PG_STATIC2)
    constexpr unsigned STATIC_TILES = OZ2_PG_STATIC2 ? 2 : 1;
    auto to_tile = [&](unsigned pos) { return pos + STATIC_TILES * nblk < total ? pos + STATIC_TILES * nblk : NO_TILE; };
    unsigned ccur = (bid >> 3) < total ? (bid >> 3) : NO_TILE;
    if (ccur == NO_TILE) return;  // block-uniform, before any barrier
    // the second tile: static, the block's position plus the XCD's block count (OZ2_PG_STATIC2, the default: no
    // atomic round trip before the first DMA), or claimed before the prologue DMA and waited for at once.
    // OZ2_PG_CLAIM_EARLY=1 (A/B builds) issued that claim after the DMA: same time, but the blocks' second tiles
    // then left dispatch order and the launch fetched 5 % more (profiles/r06/epilogue_ab/claim_ab.txt)
    if (OZ2_PG_STATIC2 && tid == 0) {
        const unsigned second = nblk + (bid >> 3);
        spare[0] = second < total ? second : NO_TILE;
    }
    if (!OZ2_PG_STATIC2 && !OZ2_PG_CLAIM_EARLY && tid == 0) spare[0] = to_tile(claim());

    const unsigned K = g.ksteps;  // >= 6 (host)
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int8_t *)smem;
    const uint32_t lds_wave = lds_base + wave * 1024;
    const uint32_t lane_off = wave * 1024 + lane * 16;
    auto rsrcA = [&](const TileRef &t) { return make_rsrc(g.A + (size_t)t.j * g.planeA, (uint32_t)g.planeA); };
    auto rsrcB = [&](const TileRef &t) { return make_rsrc(g.B + (size_t)t.j * g.planeB, (uint32_t)g.planeB); };
    auto lo_of = [&](unsigned step) { return lds_wave + (step & (PSTAGES - 1)) * SLOT; };
    auto rd_of = [&](unsigned step) { return smem + (step & (PSTAGES - 1)) * SLOT; };

    TileRef ct = decode_tile<SUB>(g, tile_u(ccur));
    v4si rA = rsrcA(ct), rB = rsrcB(ct);
    constexpr unsigned D = PSTAGES - 1;
    for (unsigned s0 = 0; s0 < D; ++s0) {
        const uint32_t lo = lo_of(s0);
        bglds16(rA, ct.offA + s0 * PANEL + lane_off, lo);
        bglds16(rA, ct.offA + s0 * PANEL + lane_off + 8192, lo + 8192);
        bglds16(rB, ct.offB + s0 * PANEL + lane_off, lo + PANEL);
        bglds16(rB, ct.offB + s0 * PANEL + lane_off + 8192, lo + PANEL + 8192);
    }
    if (!OZ2_PG_STATIC2 && OZ2_PG_CLAIM_EARLY && tid == 0) spare[0] = to_tile(claim());
    wait_vm_lgkm0<GLDS_PER_STEP *(D - 1)>();  // step 0 landed (and the claim's LDS write)
    barrier();

    unsigned s = 0;
    unsigned cnext = __builtin_amdgcn_readfirstlane(spare[0]);
    uint32_t da = ct.offA + D * PANEL, db = ct.offB + D * PANEL;
    Frags f;
    AccTile acc[ACC_I][ACC_J];
    unsigned pos = 0;  // thread 0: the queue position claimed for the tile after next
    bool claimed = false;
    if (wr == 1) barrier();  // group 1 falls one barrier behind, for the whole launch
    for (unsigned r = 0;; ++r) {
        const v4i bias = v4i{} + (g.biased ? g.bias[ct.j] : 0);
        unsigned k = 0;
        uint32_t na = 0, nb = 0;
        v4si nrA = rA, nrB = rB;
        // one k-step: reads of slot s, DMA of step s+3 (the cursor jumps to the next tile after staging this
        // tile's last step), wait, MFMAs (the first of a tile from the bias splat), then `mid` (wave 0's publish)
        auto step = [&](auto wait, auto first, auto mid) {
            read_frags(f, rd_of(s), wr, wc, lane);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t lo = lo_of(s + D);
            bglds16(rA, da + lane_off, lo);
            bglds16(rA, da + lane_off + 8192, lo + 8192);
            bglds16(rB, db + lane_off, lo + PANEL);
            bglds16(rB, db + lane_off + 8192, lo + PANEL + 8192);
            const bool jump = k + D + 1 == K;
            da = jump ? na : da + PANEL;
            db = jump ? nb : db + PANEL;
            if (jump) {  // block-uniform
                rA = nrA;
                rB = nrB;
            }
            wait();
            barrier();
            if constexpr (decltype(first)::value) mfma_step_first(acc, f, bias);
            else mfma_step<PRIO>(acc, f);
            mid();
            barrier();
        };
        auto none = [] {};
        // steps 0 and 1 (one code path for every tile: the accumulators get ONE defining MFMA): from the second
        // tile on, the previous tile's 8 residue stores are younger than the awaited DMA
        auto wait01 = [&] {
            if (r > 0) wait_vm_lgkm0<GLDS_PER_STEP *(D - 1) + PARK_STORES>();
            else wait_vm_lgkm0<GLDS_PER_STEP *(D - 1)>();
        };
        step(wait01, std::true_type{}, [&] {
            if (claimed) {  // group 0's MFMA interval: group 1 has read its parked residues back
                // (the opaque copy keeps the compiler from using the claim's result -- and waiting for it, with
                // every older memory operation -- right after the atomic in the epilogue)
                unsigned p2 = pos;
                asm volatile("" : "+v"(p2));
                spare[0] = to_tile(p2);
                __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0)
            }
        });
        ++k, ++s;
        step(wait01, std::false_type{}, none);
        ++k, ++s;
        if (r > 0) cnext = __builtin_amdgcn_readfirstlane(spare[0]);  // published by thread 0 two barriers ago
        TileRef nt = ct;
        if (cnext != NO_TILE) {
            nt = decode_tile<SUB>(g, tile_u(cnext));
            na = nt.offA;
            nb = nt.offB;
            nrA = rsrcA(nt);
            nrB = rsrcB(nt);
        }
        const unsigned kend = cnext != NO_TILE ? K : K - D;
        for (; k < kend; ++k, ++s) step([] { wait_vm_lgkm0<GLDS_PER_STEP *(D - 1)>(); }, std::false_type{}, none);
        for (; k < K; ++k, ++s) {  // drain of the block's last tile
            read_frags(f, rd_of(s), wr, wc, lane);
            __builtin_amdgcn_sched_barrier(0);
            wait_steps_lgkm0<GLDS_PER_STEP>(k + 2 < K ? (int)(K - k - 2) : 0);
            barrier();
            mfma_step<PRIO>(acc, f);
            barrier();
        }

        // ---- this group's epilogue: park interval, then store interval ----
        claimed = tid == 0 && cnext != NO_TILE;
        if (claimed) pos = claim();
        int etid = tid;
        asm volatile("" : "+v"(etid));
        const int elane = etid & 63, gtid = etid & 255;
        const int p = g.p[ct.j];
        uint32_t *const park = wr == 0 ? reinterpret_cast<uint32_t *>(rd_of(s - 1)) : spare;
        auto park_all = [&](auto &&res) {
            if (ABL == 3) {  // probe: the accumulators stay live (else their MFMAs are dead code)
#pragma unroll
                for (int i = 0; i < ACC_I; ++i)
#pragma unroll
                    for (int jj = 0; jj < ACC_J; ++jj) asm volatile("" ::"v"(acc[i][jj]));
                return;
            }
            // dword 4 i + q of column col (rows 16 i + 4 q ..) at col * 32 + 4 (i ^ (col & 7)) + q: the 16-byte
            // chunk i is XOR-swizzled by the column's low bits (two lanes per bank for a 16 x 16 tile's writes, no
            // permutation inside a chunk), and col & 7 = lane & 7, so a lane's eight chunk positions are eight
            // per-lane addresses computed once per tile, the four column blocks jj immediate offsets
            const int t7 = elane & 7;
            uint32_t *const pb = park + (wc * 64 + (elane & 15)) * 32 + (elane >> 4);
#pragma unroll
            for (int i = 0; i < ACC_I; ++i) {
                uint32_t *const pi = pb + 4 * (i ^ t7);
#pragma unroll
                for (int jj = 0; jj < ACC_J; ++jj) {
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w |= res(acc[i][jj][e]) << (8 * e);
                    pi[jj * 16 * 32] = w;
                }
            }
        };
        if (ABL == 1 || (g.biased && p == 256)) {
            park_all([&](int x) { return (uint32_t)x & 0xffu; });
        } else if (g.biased) {
            const double invp = g.invp[ct.j], pneg = -(double)p;
            const double cneg = __builtin_fma(-0x1p52, invp, 0x1p-8);
            park_all([&](int x) { return residue_biased_f64((uint32_t)x, invp, cneg, pneg); });
        } else {
            const int bar = g.barrett[ct.j];
            const bool p256 = (p == 256);
            park_all([&](int x) { return residue(x, p, bar, p256); });
        }
        __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0), vmcnt untouched
        barrier();
        uint8_t *out = static_cast<uint8_t *>(g.out) + ct.j * g.planeOut + ct.sb * g.subOut +
                       (size_t)ct.tn * 256 * g.ldo + (size_t)ct.tm * 256 + wr * 128;
#pragma unroll
        for (int it = 0; it < PARK_STORES; ++it) {
            if (ABL >= 2) break;
            const int chunk = gtid + 256 * it;
            const int col = chunk >> 3, c = chunk & 7;
            const uint4 v = *reinterpret_cast<const uint4 *>(park + col * 32 + ((c ^ (col & 7)) << 2));
            typedef unsigned u4v __attribute__((ext_vector_type(4)));
            const u4v val = u4v{v.x, v.y, v.z, v.w};
            u4v *dst = reinterpret_cast<u4v *>(out + (size_t)col * g.ldo + 16 * c);
            if (OZ2_RES_NTS) __builtin_nontemporal_store(val, dst);
            else *dst = val;
        }
        if (claimed) asm volatile("" ::"v"(pos));  // the claim returned (older than the 8 stores: vmcnt(8))
        __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));  // park reads done
        barrier();
        if (cnext == NO_TILE) break;
        ct = nt;
    }
    if (wr == 0) barrier();  // group 0 passed one barrier fewer (group 1's initial one)
}

// Exhaustive check of the two residue epilogues against exact arithmetic, every input and every
// modulus: path 0 = biased (x in [-2^30, 2^30], the accumulator starting at bias_i), path 1 = signed
// Barrett (every int32, conv_32i_2_8u.hpp:7-56).  Counts mismatches into *count.
__global__ void residue_selftest_kernel(int path, GemmArgs g, unsigned long long *count) {
    unsigned long long bad = 0;
    // path 2: the biased check against a deliberately wrong expectation (negative control: every
    // pair must be counted); path 3: the f64 form of the biased residue (p < 256; 256: the low byte)
    const uint64_t total = path != 1 ? ((uint64_t)1 << 31) + 1 : ((uint64_t)1 << 32);
    const int64_t lo = path != 1 ? -((int64_t)1 << 30) : -((int64_t)1 << 31);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t x = lo + (int64_t)i;
        for (int j = 0; j < OZ2_MAX_MODULI; ++j) {
            const int p = g.p[j] > 0 ? g.p[j] : 256;
            // exact x mod p in [0, p) through f64 (|x| < 2^53) with a one-step correction
            int64_t q = (int64_t)floor((double)x * (1.0 / (double)p));
            int64_t r = x - q * p;
            if (r < 0) r += p;
            if (r >= p) r -= p;
            if (path == 2) r = (r + 1) % p;
            uint32_t got;
            if (path == 3) {
                const uint32_t u = (uint32_t)((int32_t)x + g.bias[j]);
                got = p == 256 ? (u & 0xffu)
                               : residue_biased_f64(u, g.invp[j], __builtin_fma(-0x1p52, g.invp[j], 0x1p-8), -(double)p);
            } else if (path != 1) {
                got = residue_biased((uint32_t)((int32_t)x + g.bias[j]), (uint32_t)p, g.minv[j]);
            } else {
                got = residue((int)x, g.p[j], g.barrett[j], p == 256);
            }
            bad += (got != (uint32_t)r);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) bad += __shfl_xor(bad, d);
    if ((threadIdx.x & 63) == 0 && bad) atomicAdd(count, bad);
}

unsigned long long residue_selftest(int path, hipStream_t st) {
    GemmArgs g{};
    const ModParams MP = make_mod_params(OZ2_MAX_MODULI);
    for (int i = 0; i < OZ2_MAX_MODULI; ++i) {
        g.p[i] = MP.p[i];
        g.barrett[i] = MP.barrett[i];
        const uint32_t p = MP.p[i] > 0 ? (uint32_t)MP.p[i] : 256u;
        g.minv[i] = (uint32_t)((((uint64_t)1) << 32) / p);
        g.bias[i] = (int)(((((uint64_t)1) << 30) + p - 1) / p * p);
        g.invp[i] = 1.0 / (double)p;
    }
    unsigned long long *d = nullptr, h = ~0ull;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return h;
    (void)hipMemsetAsync(d, 0, sizeof(h), st);
    residue_selftest_kernel<<<4096, 256, 0, st>>>(path, g, d);
    if (hipGetLastError() != hipSuccess) {
        (void)hipFree(d);
        return ~0ull;
    }
    (void)hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    (void)hipFree(d);
    return h;
}

// CUs of the current device (one persistent block each); cached per device id below 64 (atomics: any
// host thread may launch), queried on every call beyond
static unsigned device_cu_count() {
    static std::atomic<unsigned> cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    if (dev < 64) {
        const unsigned c = cached[dev].load(std::memory_order_relaxed);
        if (c) return c;
    }
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    if (dev < 64) cached[dev].store((unsigned)n, std::memory_order_relaxed);
    return (unsigned)n;
}
// the residue-product kernel the last gemm_i8 RESIDUE launch of this process took (bench.py labels)
std::atomic<int> g_last_residue_kernel{0};
// GEMMUL8_PERSISTENT: 0 = one-tile kernel only, 1 = persistent kernel wherever it applies, unset =
// persistent when the launch has at least three tiles per CU.  g_persistent_override (probes) wins when >= 0.
int g_persistent_override = -1;
int g_prio_override = 1;  // probes: the persistent kernel's priority variant (PRIO; 1 = the default)
int g_epim_override = 0;  // probes: the persistent kernel's residue arithmetic (EPIM; 0 = the default)
int g_order_override = 0;  // probes: the persistent kernel's k order (ORD; 0 = the default)
unsigned long long *g_stamps = nullptr;  // probes: OZ2_STAMPS builds' per-wave phase sums
// the persistent kernel: per wave group epilogues (gemm_i8_persistent_pg_kernel, the default) or the block
// epilogue (gemm_i8_persistent_kernel: GEMMUL8_PG_EPILOGUE=0, read once; A/B and the kernel the stamp / EPIM /
// order probes instrument).  g_pg_override (probes) wins when >= 0; 2-4 are the per-group kernel's ablations.
int g_pg_override = -1;
static bool pg_epilogue() {
    if (g_pg_override >= 0) return g_pg_override != 0;
    static const bool env = [] {
        const char *e = getenv("GEMMUL8_PG_EPILOGUE");
        return e ? atoi(e) != 0 : true;
    }();
    return env;
}
// GEMMUL8_SMALL_TILES: 0 = never the 128 x 128 kernel, 1 = wherever it applies, unset (2) = the rule in
// gemm_i8.  g_small_override (probes) wins when >= 0.
int g_small_override = -1;
static int small_tiles_mode() {
    if (g_small_override >= 0) return g_small_override;
    static const int env = [] {
        const char *e = getenv("GEMMUL8_SMALL_TILES");
        return e ? atoi(e) : 2;
    }();
    return env;
}
static int persistent_mode() {
    if (g_persistent_override >= 0) return g_persistent_override;
    static const int env = [] {
        const char *e = getenv("GEMMUL8_PERSISTENT");
        return e ? atoi(e) : 2;
    }();
    return env;
}

// GEMMUL8_TAIL_SMALL=1 (read once): 128 x 128 tail planes (below; measured slower, so off by default)
static bool tail_small_mode() {
    static const bool on = [] {
        const char *e = getenv("GEMMUL8_TAIL_SMALL");
        return e ? atoi(e) != 0 : false;
    }();
    return on;
}
std::atomic<int> g_last_tail_small{0};

void gemm_i8(const int8_t *A8, const int8_t *B8, const Layout &L, unsigned nplanes, Epi epi, void *out,
             int32_t *rowmax, int32_t *colmax, const ModParams &MP, hipStream_t st, uint32_t *queue,
             bool queue_zeroed, bool tail_small) {
    GemmArgs g{};
    g.A = A8;
    g.B = B8;
    g.planeA = L.planeA;
    g.planeB = L.planeB;
    g.ksteps = (unsigned)L.ksteps;
    g.mtiles = (unsigned)L.mtiles;
    g.ntiles = (unsigned)L.ntiles;
    g.out = out;
    g.planeOut = L.planeR;
    g.ldo = L.ldr;
    // Karatsuba complex: the residue products run as 3 sub-products per modulus; the bound and raw
    // products always see one (the bound runs on the big-matrix geometry)
    g.nsub = epi == Epi::RESIDUE ? L.nsub : 1;
    g.subA = g.nsub > 1 ? L.subA : 0;
    g.subB = g.nsub > 1 ? L.subB : 0;
    g.subOut = g.nsub > 1 ? L.subR : 0;
    g.rowmax = rowmax;
    g.colmax = colmax;
    // |int8 product| <= 2^14 * k_pad: the biased residue path needs <= 2^30
    g.biased = L.k_pad <= ((size_t)1 << 16) ? 1 : 0;
    for (int i = 0; i < OZ2_MAX_MODULI; ++i) {
        g.p[i] = MP.p[i];
        g.barrett[i] = MP.barrett[i];
        const uint32_t p = MP.p[i] > 0 ? (uint32_t)MP.p[i] : 256u;
        g.minv[i] = (uint32_t)((((uint64_t)1) << 32) / p);
        g.bias[i] = (int)(((((uint64_t)1) << 30) + p - 1) / p * p);
        g.invp[i] = 1.0 / (double)p;
    }
    g.kstride = g.ksteps;
    g.k0 = 0;
    dim3 grid((unsigned)(L.mtiles * L.ntiles), nplanes * g.nsub);
    // GEMMUL8_FORCE_FLAT_DMA=1 takes the 64-bit path at any size (tests cover it with small shapes)
    const char *ff = getenv("GEMMUL8_FORCE_FLAT_DMA");
    const bool buf = L.planeA < ((size_t)1 << 32) && L.planeB < ((size_t)1 << 32) && !(ff && atoi(ff));
#define OZ2_GEMM1(E, B) launch(gemm_i8_kernel<E, B>, grid, dim3(NTHREADS), st, g)
#define OZ2_GEMM(E, B) (g.nsub == 3 ? launch(gemm_i8_kernel<E, B, true>, grid, dim3(NTHREADS), st, g) : OZ2_GEMM1(E, B))
    // beyond k_pad = 2^17 an int32 product can wrap (the reference's int32 C32i does): the residue
    // product then runs in k-chunks of 2^16 (biased path), each adding its residues into the planes
    // mod p.  GEMMUL8_KCHUNK (k-steps, multiple of 1) forces chunking at small k for the tests.
    static const unsigned forced_chunk = [] {
        const char *e = getenv("GEMMUL8_KCHUNK");
        return e ? (unsigned)atoi(e) : 0u;
    }();
    const unsigned chunk = forced_chunk ? forced_chunk : ((1u << 16) / KSTEP);
    if (epi == Epi::RESIDUE && (L.k_pad > ((size_t)1 << 17) || (forced_chunk && g.ksteps > forced_chunk))) {
        g_last_residue_kernel.store(3, std::memory_order_relaxed);
        g.biased = 1;
        for (unsigned k0 = 0; k0 < g.kstride; k0 += chunk) {
            g.k0 = k0;
            g.ksteps = g.kstride - k0 < chunk ? g.kstride - k0 : chunk;
            if (k0 == 0) buf ? OZ2_GEMM(0, 1) : OZ2_GEMM(0, 0);
            else buf ? OZ2_GEMM(EPI_RESIDUE_ADD, 1) : OZ2_GEMM(EPI_RESIDUE_ADD, 0);
        }
        return;
    }
    // persistent residue kernel: a tile-queue area, buffer descriptors (planes < 4 GiB),
    // >= 6 k-steps per tile (the kernel's cursor jump at k = K - 4 after its first two steps) and, by
    // default, >= 3 tiles per CU (measured, same process: cfg2 products 5.16 -> 5.04 ms, 8192^2 x 1024
    // 1.14 -> 1.01 ms, 4096^3 0.857 -> 0.842 ms; with the queue zeroed by the encode instead of a launch
    // of its own, tools/probes/persist_threshold.sh: 2048^3 (3.5 tiles per CU) 112.8 -> 110.3 us,
    // 2560^3 199.1 -> 192.0 us, 3072^3 317.0 -> 305.7 us, but 1536^3 (2 per CU) 57.6 -> 65.2 us)
    const unsigned ntiles_all = (unsigned)(L.mtiles * L.ntiles) * nplanes * g.nsub;
    const unsigned ncu = device_cu_count();
    const int pmode = persistent_mode();
    // 128 x 128 tiles, two blocks per CU (gemm_i8_small_kernel): by default the accurate-mode bound product with
    // fewer 256 x 256 tiles than CUs (1024^2: 16 tiles on 256 CUs; measured, profiles/r06/small_tiles/: the
    // accurate scaling phase at 1024^3 63.7 -> 55.2 us, 1536^3 83.3 -> 73.3, 2048^3 100.6 -> 94.5).  Residue
    // products only when forced: the 256-tile kernels are faster for them at every size measured (1024^3 22.7
    // vs 29.5 us, 1536^3 55.1 vs 63.8, 2048^3 105 vs 130).  GEMMUL8_SMALL_TILES=0 never, 1 wherever it applies
    // (residue and bound products over buffer descriptors), unset by that rule unless GEMMUL8_PERSISTENT forces
    // a 256-tile kernel.
    const int smode = small_tiles_mode();
    // Tail planes (GEMMUL8_TAIL_SMALL=1): a residue launch whose last round of 256 x 256 tiles would leave CUs idle
    // (2048^3: 896 tiles, 3.5 per CU; 1152^3: 350 on 256 CUs) runs the planes that fit one round fewer on the
    // 256-tile kernels and the rest, at most half a round of 256-tiles, as 128 x 128 tiles (two blocks per CU: one
    // round of them).  Same residues (integer sums), but slower: 2048^3 products 98.5-99.1 -> 102.7-104.0 us, 1152^3
    // 36.5-36.9 -> 38.0-38.3 us (profiles/r06/mid_sizes/tail_small_ab.txt): the 128 x 128 round costs more than the
    // half-empty 256-tile round it replaces.
    if (epi == Epi::RESIDUE && !tail_small && g.nsub == 1 && buf && smode == 2 && pmode == 2 && tail_small_mode()) {
        const unsigned T = (unsigned)(L.mtiles * L.ntiles);
        const unsigned rounds = (ntiles_all + ncu - 1) / ncu;
        if (rounds >= 2 && ntiles_all % ncu != 0) {
            const unsigned keep = (unsigned)(((size_t)(rounds - 1) * ncu) / T);
            const unsigned tail = nplanes - keep;
            if (keep >= 1 && tail >= 1 && 2 * (size_t)tail * T <= ncu) {
                gemm_i8(A8, B8, L, keep, epi, out, rowmax, colmax, MP, st, queue, queue_zeroed, false);
                const int head = g_last_residue_kernel.load(std::memory_order_relaxed);
                ModParams M2 = MP;
                for (unsigned i = 0; i < tail; ++i) {
                    M2.p[i] = MP.p[keep + i];
                    M2.barrett[i] = MP.barrett[keep + i];
                    M2.rinv_d[i] = MP.rinv_d[keep + i];
                    M2.rinv_f[i] = MP.rinv_f[keep + i];
                }
                M2.N = tail;
                gemm_i8(A8 + keep * L.planeA, B8 + keep * L.planeB, L, tail, epi,
                        static_cast<uint8_t *>(out) + keep * L.planeR, nullptr, nullptr, M2, st, nullptr, true, true);
                g_last_residue_kernel.store(head, std::memory_order_relaxed);
                g_last_tail_small.store(1, std::memory_order_relaxed);
                return;
            }
        }
    }
    if (epi == Epi::RESIDUE && !tail_small) g_last_tail_small.store(0, std::memory_order_relaxed);
    if ((epi == Epi::RESIDUE || epi == Epi::BOUND) && buf &&
        (smode == 1 || tail_small || (smode == 2 && pmode == 2 && epi == Epi::BOUND && ntiles_all < ncu))) {
        const dim3 sgrid((unsigned)(4 * L.mtiles * L.ntiles), nplanes * g.nsub);
        if (epi == Epi::RESIDUE) {
            g_last_residue_kernel.store(4, std::memory_order_relaxed);
            if (g.nsub == 3) launch(gemm_i8_small_kernel<0, true>, sgrid, dim3(SM_THREADS), st, g);
            else launch(gemm_i8_small_kernel<0, false>, sgrid, dim3(SM_THREADS), st, g);
        } else {
            launch(gemm_i8_small_kernel<1, false>, sgrid, dim3(SM_THREADS), st, g);
        }
        return;
    }
    // round 6, per-group kernel: also up to 1.5 tiles per CU when its XCD queues need no more rounds than the
    // one-tile launch (1024^3 products 22.7 -> 21.0 us, 1152^3 37.3 -> 36.3, 1280^3 44.6 -> 39.2; 1024^2 x k
    // faster from 6 k-steps on).  With fewer than 8 tiles per plane, or 9 of them, the XCD shares are uneven
    // (512^2: 4 tiles per plane on 4 XCDs, 7 blocks each for 14 tiles, 2 rounds: 13.2 -> 19.5 us; 768^3 15.8 ->
    // 22.2), so those stay one-tile; 1536^3 (2 per CU) too: 54.4 vs 60.2 (profiles/r06/mid_sizes/persistent_ab.txt)
    auto persist_balanced = [&] {
        const unsigned per_plane = (unsigned)(L.mtiles * L.ntiles), grid = std::min(ntiles_all, ncu);
        const unsigned most = nplanes * g.nsub * ((per_plane >> 3) + ((per_plane & 7) ? 1u : 0u));
        const unsigned fewest_blocks = grid >> 3;
        return fewest_blocks > 0 && (most + fewest_blocks - 1) / fewest_blocks <= (ntiles_all + ncu - 1) / ncu;
    };
    const bool persist_rule = ntiles_all >= 3 * ncu || (pg_epilogue() && 2 * ntiles_all <= 3 * ncu && persist_balanced());
    if (epi == Epi::RESIDUE && queue && buf && pmode != 0 && g.ksteps >= 6 && (pmode == 1 || persist_rule)) {
        g_last_residue_kernel.store(2, std::memory_order_relaxed);
        g.nplanes = nplanes * g.nsub;
        g.queue = queue;
        g.stamps = g_stamps;
        if (!queue_zeroed) zero_i32(reinterpret_cast<int32_t *>(queue), 8, st);
        // GEMMUL8_PERSISTENT_GRID caps the grid (tests: many tiles per block at small shapes), at no fewer
        // than 8 blocks: every XCD queue that holds tiles needs a block of its own (bid mod 8)
        static const unsigned grid_cap = [] {
            const char *e = getenv("GEMMUL8_PERSISTENT_GRID");
            return e ? (unsigned)atoi(e) : 0u;
        }();
        const dim3 pgrid(std::min(std::min(ntiles_all, ncu), grid_cap ? std::max(grid_cap, 8u) : ncu));
        // (the probe overrides below select the block-epilogue kernel's variants)
        const bool probe_variant = g_epim_override != 0 || g_prio_override != 1 || g_order_override != 0;
        if (pg_epilogue() && !probe_variant) {
#ifdef OZ2_PG_PROBES
            if (g_pg_override == 2) launch(gemm_i8_persistent_pg_kernel<false, 1, 1>, pgrid, dim3(NTHREADS), st, g);
            else if (g_pg_override == 3) launch(gemm_i8_persistent_pg_kernel<false, 1, 2>, pgrid, dim3(NTHREADS), st, g);
            else if (g_pg_override == 4) launch(gemm_i8_persistent_pg_kernel<false, 1, 3>, pgrid, dim3(NTHREADS), st, g);
            else
#endif
            if (g.nsub == 3) launch(gemm_i8_persistent_pg_kernel<true, 1>, pgrid, dim3(NTHREADS), st, g);
            else launch(gemm_i8_persistent_pg_kernel<false, 1>, pgrid, dim3(NTHREADS), st, g);
            g_last_residue_kernel.store(5, std::memory_order_relaxed);
        } else if (g.nsub == 3) launch(gemm_i8_persistent_kernel<true, 1>, pgrid, dim3(NTHREADS), st, g);
        else if (g_epim_override == 1) launch(gemm_i8_persistent_kernel<false, 1, 1>, pgrid, dim3(NTHREADS), st, g);
        else if (g_epim_override == 2) launch(gemm_i8_persistent_kernel<false, 1, 2>, pgrid, dim3(NTHREADS), st, g);
#ifdef OZ2_EPIM_PROBES
        else if (g_epim_override == 3) launch(gemm_i8_persistent_kernel<false, 1, 3>, pgrid, dim3(NTHREADS), st, g);
        else if (g_epim_override == 4) launch(gemm_i8_persistent_kernel<false, 1, 4>, pgrid, dim3(NTHREADS), st, g);
#endif
#ifdef OZ2_ORDER_PROBES
        else if (g_order_override == 1) launch(gemm_i8_persistent_kernel<false, 1, 0, 1>, pgrid, dim3(NTHREADS), st, g);
#endif
        else if (g_prio_override == 0) launch(gemm_i8_persistent_kernel<false, 0>, pgrid, dim3(NTHREADS), st, g);
        else if (g_prio_override == 2) launch(gemm_i8_persistent_kernel<false, 2>, pgrid, dim3(NTHREADS), st, g);
        else launch(gemm_i8_persistent_kernel<false, 1>, pgrid, dim3(NTHREADS), st, g);
        return;
    }
    switch (epi) {
    case Epi::RESIDUE:
        g_last_residue_kernel.store(1, std::memory_order_relaxed);
        buf ? OZ2_GEMM(0, 1) : OZ2_GEMM(0, 0);
        break;
    case Epi::BOUND: buf ? OZ2_GEMM1(1, 1) : OZ2_GEMM1(1, 0); break;
    default: buf ? OZ2_GEMM1(2, 1) : OZ2_GEMM1(2, 0); break;
    }
#undef OZ2_GEMM
#undef OZ2_GEMM1
}

}  // namespace oz2
