// gemm_i8.hip -- exact int8 x int8 -> int32 slice products on CDNA4 MFMA with fused epilogues.
//
// Replaces the reference's per-modulus hipblasGemmEx + conv_32i_2_8u pair
// (GEMMul8/src/gemmul8.cu:259-275, conv_32i_2_8u.hpp:7-71): one launch covers all
// N moduli (grid.y = modulus), each 256x256 output tile accumulates with
// v_mfma_i32_32x32x32_i8 and is reduced mod p_i in the epilogue, so the int32
// product never reaches HBM (the reference writes and re-reads 4*m*n bytes per
// modulus).  The accurate-mode bound product (scaling.hpp:3113-3121) runs the same
// main loop with a row/column-max epilogue instead of an m x n int32 buffer.
//
// Block: 256 threads = 4 waves (one per SIMD) as 2 (M) x 2 (N); each wave owns a
// 128 x 128 sub-tile = 4 x 4 fragments of 32x32 (256 accumulator registers).
// Pipeline per 64-deep k-step:
//   * operand panels (16 KiB each, pre-arranged in fragment order by split.hip)
//     stream HBM -> LDS through a 4-slot ring (128 KiB) with global_load_lds issued
//     three k-steps ahead (inline asm, one DMA per 4 MFMAs, waits counted by hand);
//     measured on MI355X: 3 slots 1.87 ms, 4 slots 1.63 ms, 5 slots 1.63 ms (N=4, 8192^3);
//   * one barrier per k-step;
//   * the next k-step's 16 fragment reads (ds_read_b128, conflict-free 1 KiB sweeps)
//     are issued between the current k-step's 32 MFMAs (register double buffer).
#include "oz2_split.hpp"

namespace oz2 {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int NTHREADS = 256;
#ifndef OZ2_STAGES
#define OZ2_STAGES 4
#endif
constexpr int STAGES = OZ2_STAGES;  // ring slots; DMA runs STAGES-1 k-steps ahead
constexpr int SLOT = 2 * PANEL;                 // A panel + B panel
constexpr int LDS_BYTES = STAGES * SLOT;        // the epilogue reuses 64 KiB of it
constexpr int GLDS_PER_STEP = 8;                // 16-B LDS-DMA per thread per k-step (4 A + 4 B)

struct GemmArgs {
    const int8_t *A;
    const int8_t *B;
    size_t planeA, planeB;
    unsigned ksteps, mtiles, ntiles;
    void *out;
    size_t planeOut, ldo;
    int32_t *rowmax, *colmax;
    int p[OZ2_MAX_MODULI];
    int barrett[OZ2_MAX_MODULI];
};

// One 16-byte-per-lane LDS-DMA: LDS[m0 + lane*16] <- gsrc (per lane).  Issued from inline asm
// so the compiler neither waits for it nor reorders it; completion is counted with vmcnt by hand.
// M0 is compiler-reserved: saved and restored inside the statement.
#ifndef OZ2_ABLATE
#define OZ2_ABLATE 0  // probe builds only: 1 = no LDS-DMA in the main loop, 2 = no MFMA
#endif
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_addr) {
    if (OZ2_ABLATE == 1) return;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}
// sched_barrier(0) after each: hipcc would otherwise move register-only MFMAs across these
// asm statements (their "memory" clobber does not order them), stretching live ranges
// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]);
// the builtin form is visible to the compiler's own waitcnt tracking of its ds_reads.
template <int N> __device__ __forceinline__ void wait_vmcnt() {
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void wait_lgkm0() {
    __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void barrier() {
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// r = x mod p in [0, p): conv_32i_2_8u.hpp:7-56 (modulus 256 = low byte, others Barrett)
__device__ __forceinline__ uint32_t residue(int x, int p, int barrett, bool p256) {
    if (p256) return (uint32_t)x & 0xffu;
    x -= __mulhi(x, barrett) * p;
    x -= (x >= p) * p;
    x += (x < 0) * p;
    return (uint32_t)x;
}

// One half-step (32-deep k-substep) of fragments: 4 row blocks of A, 4 column blocks of B.
struct Half {
    v4i a[4];
    v4i b[4];
};

__device__ __forceinline__ void read_half(Half &h, const int8_t *slot, int s, int wm, int wn, int lane) {
    const int8_t *la = slot + s * 8192 + (wm * 4) * 1024 + lane * 16;
    const int8_t *lb = slot + PANEL + s * 8192 + (wn * 4) * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h.a[i] = *reinterpret_cast<const v4i *>(la + i * 1024);
        h.b[i] = *reinterpret_cast<const v4i *>(lb + i * 1024);
    }
}

// 4 MFMAs of row block g (acc[g][0..3]) from one half-step of fragments
__device__ __forceinline__ void mfma_row(v16i (&acc)[4][4], const Half &h, int g) {
    if (OZ2_ABLATE == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[g][j][0] += h.a[g][0] ^ h.b[j][1];
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[g][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(h.a[g], h.b[j], acc[g][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
}

template <int EPI>
__global__ __launch_bounds__(NTHREADS, 1) void gemm_i8_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(1024))) int8_t smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const unsigned j = blockIdx.y;

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

    const int8_t *Ag = g.A + j * g.planeA + (size_t)tm * g.ksteps * PANEL + tid * 16;
    const int8_t *Bg = g.B + j * g.planeB + (size_t)tn * g.ksteps * PANEL + tid * 16;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int8_t *)smem;
    const uint32_t lds_wave = lds_base + wave * 1024;

    // part 0..3: quarter q of the A panel, 4..7: of the B panel (1 KiB per wave each)
    auto stage_part = [&](unsigned ks, unsigned slot, int part) {
        const int8_t *g0 = (part < 4 ? Ag : Bg) + (size_t)ks * PANEL + (part & 3) * 4096;
        glds16(g0, lds_wave + slot * SLOT + (part < 4 ? 0 : PANEL) + (part & 3) * 4096);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto stage = [&](unsigned ks, unsigned slot) {
#pragma unroll
        for (int part = 0; part < 8; ++part) stage_part(ks, slot, part);
    };

    v16i acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = v16i{};

    // Per k-step t (slot of t landed, half 0 of t in h0):
    //   issue LDS-DMA of step t+2;  MFMA(h0) || read half 1 of t -> h1;  wait lgkm
    //   wait vmcnt (step t+1 landed);  barrier
    //   MFMA(h1) || read half 0 of t+1 -> h0;  wait lgkm
    // The slot written at step t was last read before the barrier of step t-1.
    const unsigned K = g.ksteps;
    constexpr unsigned D = STAGES - 1;  // prefetch distance in k-steps
    Half h0, h1;
    if (K == 0) goto epilogue;
    // prologue: steps 0..D-1 in flight, wait for step 0
    for (unsigned s0 = 0; s0 < D; ++s0)
        if (s0 < K) stage(s0, s0);
    if (K >= D) wait_vmcnt<GLDS_PER_STEP *(D - 1)>();
    else wait_vmcnt<0>();
    barrier();
    read_half(h0, smem, 0, wm, wn, lane);
    wait_lgkm0();
    {
        unsigned slot_cur = 0, slot_next = 1, slot_issue = D;  // slots of steps t, t+1, t+D
        unsigned t = 0;
        // Steady state (step t+D exists), branch-free: the 8 LDS-DMA of step t+D are spread one
        // per 4 MFMAs over both half-steps so their issue cost hides under MFMA execution.  At the
        // end of half 0, younger than step t+1's DMA are those of steps t+2..t+D-1 (8 each) and the
        // 4 just issued: vmcnt(8*(D-2)+4).  The slot refilled at step t is that of step t-1, whose
        // last reads completed before the barrier of step t-1.
        for (; t + D < K; ++t) {
            read_half(h1, smem + slot_cur * SLOT, 1, wm, wn, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                mfma_row(acc, h0, gq);
                stage_part(t + D, slot_issue, gq);
            }
            constexpr int VM = GLDS_PER_STEP * (D - 2) + 4;
            __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (0 << 8) | ((VM >> 4) << 14));  // vmcnt(VM) lgkmcnt(0)
            __builtin_amdgcn_sched_barrier(0);
            barrier();
            read_half(h0, smem + slot_next * SLOT, 0, wm, wn, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                mfma_row(acc, h1, gq);
                stage_part(t + D, slot_issue, 4 + gq);
            }
            wait_lgkm0();
            slot_cur = slot_next;
            slot_next = slot_next == STAGES - 1 ? 0 : slot_next + 1;
            slot_issue = slot_issue == STAGES - 1 ? 0 : slot_issue + 1;
        }
        // drain: nothing left to stage (last D steps)
        for (; t + 1 < K; ++t) {
            read_half(h1, smem + slot_cur * SLOT, 1, wm, wn, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) mfma_row(acc, h0, gq);
            wait_lgkm0();
            wait_vmcnt<0>();
            barrier();
            read_half(h0, smem + slot_next * SLOT, 0, wm, wn, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) mfma_row(acc, h1, gq);
            wait_lgkm0();
            slot_cur = slot_next;
            slot_next = slot_next == STAGES - 1 ? 0 : slot_next + 1;
        }
        // last step
        read_half(h1, smem + slot_cur * SLOT, 1, wm, wn, lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) mfma_row(acc, h0, gq);
        wait_lgkm0();
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) mfma_row(acc, h1, gq);
    }
epilogue:
    barrier();  // all waves done with the ring before the epilogue reuses it

    // accumulator map (32x32 fragments): col = lane & 31, row = (r & 3) + 8*(r >> 2) + 4*(lane >> 5)
    if constexpr (EPI == (int)Epi::RESIDUE) {
        const int p = g.p[j], bar = g.barrett[j];
        const bool p256 = (p == 256);  // modulus 256: the low byte (conv_32i_2_8u.hpp:7-20)
        uint32_t *lo = reinterpret_cast<uint32_t *>(smem);  // [256 cols][64 dwords], dword index ^= col & 31
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int col = wn * 128 + jj * 32 + (lane & 31);
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w |= residue(acc[i][jj][4 * gq + e], p, bar, p256) << (8 * e);
                    const int rdw = wm * 32 + i * 8 + 2 * gq + (lane >> 5);
                    lo[col * 64 + (rdw ^ (col & 31))] = w;
                }
                __builtin_amdgcn_sched_barrier(0);  // one fragment at a time: bounded VGPR use
            }
        __syncthreads();
        uint8_t *out = static_cast<uint8_t *>(g.out) + j * g.planeOut + (size_t)tn * 256 * g.ldo + (size_t)tm * 256;
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int chunk = tid + NTHREADS * it;
            const int col = chunk >> 4, qd = chunk & 15;
            const int x = col & 31;
            const uint4 v = *reinterpret_cast<const uint4 *>(lo + col * 64 + ((4 * qd) ^ (x & ~3)));
            const uint32_t e[4] = {v.x, v.y, v.z, v.w};
            const int pm = x & 3;
            *reinterpret_cast<uint4 *>(out + (size_t)col * g.ldo + 16 * qd) =
                make_uint4(e[0 ^ pm], e[1 ^ pm], e[2 ^ pm], e[3 ^ pm]);
        }
    } else if constexpr (EPI == (int)Epi::BOUND) {
        int32_t *rmax = reinterpret_cast<int32_t *>(smem);
        int32_t *cmax = rmax + 256;
        rmax[tid] = 0;
        cmax[tid] = 0;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                int v = 0;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) v = max(v, abs(acc[i][jj][rr]));
#pragma unroll
                for (int d = 16; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 32));
                if ((lane & 31) == 0) atomicMax(&rmax[wm * 128 + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5)], v);
            }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            int v = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) v = max(v, abs(acc[i][jj][rr]));
            v = max(v, __shfl_xor(v, 32));
            if (lane < 32) atomicMax(&cmax[wn * 128 + jj * 32 + lane], v);
        }
        __syncthreads();
        atomicMax(&g.rowmax[tm * 256 + tid], rmax[tid]);
        atomicMax(&g.colmax[tn * 256 + tid], cmax[tid]);
    } else {  // RAW int32 (plane 0): validation path
        int32_t *out = static_cast<int32_t *>(g.out);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) {
                    const size_t row = (size_t)tm * 256 + wm * 128 + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
                    const size_t col = (size_t)tn * 256 + wn * 128 + jj * 32 + (lane & 31);
                    out[col * g.ldo + row] = acc[i][jj][rr];
                }
    }
}

void gemm_i8(const int8_t *A8, const int8_t *B8, const Layout &L, unsigned nplanes, Epi epi, void *out,
             int32_t *rowmax, int32_t *colmax, const ModParams &MP, hipStream_t st) {
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
    g.ldo = L.m_pad;
    g.rowmax = rowmax;
    g.colmax = colmax;
    for (int i = 0; i < OZ2_MAX_MODULI; ++i) {
        g.p[i] = MP.p[i];
        g.barrett[i] = MP.barrett[i];
    }
    dim3 grid((unsigned)(L.mtiles * L.ntiles), nplanes);
    switch (epi) {
    case Epi::RESIDUE: gemm_i8_kernel<0><<<grid, dim3(NTHREADS), 0, st>>>(g); break;
    case Epi::BOUND: gemm_i8_kernel<1><<<grid, dim3(NTHREADS), 0, st>>>(g); break;
    default: gemm_i8_kernel<2><<<grid, dim3(NTHREADS), 0, st>>>(g); break;
    }
}

}  // namespace oz2
