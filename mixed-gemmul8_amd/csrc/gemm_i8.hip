// gemm_i8.hip -- exact int8 x int8 -> int32 slice products on CDNA4 MFMA with fused epilogues.
//
// Replaces the reference's per-modulus hipblasGemmEx + conv_32i_2_8u pair
// (GEMMul8/src/gemmul8.cu:259-275, conv_32i_2_8u.hpp:7-71): one launch covers all
// N moduli (grid.y = modulus), each 256x256 output tile accumulates in AGPRs with
// v_mfma_i32_32x32x32_i8 and is reduced mod p_i in the epilogue, so the int32
// product never reaches HBM (the reference writes and re-reads 4*m*n bytes per
// modulus).  The accurate-mode bound product (scaling.hpp:3113-3121) uses the
// same main loop with a row/column-max epilogue instead of an m x n int32 buffer.
//
// Block: 512 threads = 8 waves as 2 (M) x 4 (N); wave tile 128 x 64 = 4 x 2
// fragments of 32x32.  Operand panels (16 KiB each, pre-arranged in fragment
// order by split.hip) are staged with global_load_lds into a double-buffered LDS
// ring; fragment reads are conflict-free 1 KiB ds_read_b128 sweeps.
#include "oz2_split.hpp"

namespace oz2 {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int NTHREADS = 512;
constexpr int LDS_BYTES = 4 * PANEL + 1024;  // 2 stages x (A, B) panels; epilogue reuses it

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

__device__ __forceinline__ void glds16(const int8_t *g, int8_t *l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}

// r = x mod p in [0, p): conv_32i_2_8u.hpp:7-56 (modulus 256 = low byte, others Barrett)
__device__ __forceinline__ uint32_t residue(int x, int p, int barrett, bool p256) {
    if (p256) return (uint32_t)x & 0xffu;
    x -= __mulhi(x, barrett) * p;
    x -= (x >= p) * p;
    x += (x < 0) * p;
    return (uint32_t)x;
}

template <int EPI>
__global__ __launch_bounds__(NTHREADS, 1) void gemm_i8_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) int8_t smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const unsigned j = blockIdx.y;

    // XCD-aware, bijective remap: blocks dealt round-robin over the 8 XCDs get
    // contiguous logical ids per XCD, then a grouped (4 row tiles) raster so the
    // ~32 co-resident tiles of one XCD share 4 A panels and 8 B panels in its L2.
    const unsigned nwg = gridDim.x, bid = blockIdx.x;
    const unsigned xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const unsigned wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    constexpr unsigned GM = 4;
    const unsigned grp = wgid / (GM * g.ntiles);
    const unsigned gm = min(GM, g.mtiles - grp * GM);
    const unsigned idx = wgid - grp * GM * g.ntiles;
    const unsigned tm = grp * GM + idx % gm, tn = idx / gm;

    const int8_t *Ag = g.A + j * g.planeA + (size_t)tm * g.ksteps * PANEL;
    const int8_t *Bg = g.B + j * g.planeB + (size_t)tn * g.ksteps * PANEL;

    auto stage = [&](unsigned ks, int buf) {
        const int8_t *ga = Ag + (size_t)ks * PANEL + tid * 16;
        const int8_t *gb = Bg + (size_t)ks * PANEL + tid * 16;
        int8_t *la = smem + buf * 2 * PANEL + wave * 1024;
        int8_t *lb = la + PANEL;
        glds16(ga, la);
        glds16(ga + 8192, la + 8192);
        glds16(gb, lb);
        glds16(gb + 8192, lb + 8192);
    };

    v16i acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj] = v16i{};

    stage(0, 0);
    __syncthreads();
    for (unsigned t = 0; t < g.ksteps; ++t) {
        const int cur = t & 1;
        if (t + 1 < g.ksteps) stage(t + 1, cur ^ 1);
        const int8_t *la = smem + cur * 2 * PANEL;
        const int8_t *lb = la + PANEL;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            v4i a[4], b[2];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const v4i *>(la + s * 8192 + (wm * 4 + i) * 1024 + lane * 16);
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) b[jj] = *reinterpret_cast<const v4i *>(lb + s * 8192 + (wn * 2 + jj) * 1024 + lane * 16);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) acc[i][jj] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[jj], acc[i][jj], 0, 0, 0);
        }
        __syncthreads();
    }

    // accumulator map (32x32 fragments): col = lane & 31, row = (r & 3) + 8*(r >> 2) + 4*(lane >> 5)
    if constexpr (EPI == (int)Epi::RESIDUE) {
        const int p = g.p[j], bar = g.barrett[j];
        const bool p256 = (j == 0);
        uint32_t *lo = reinterpret_cast<uint32_t *>(smem);  // [256 cols][64 dwords], dword index ^= col & 31
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const int col = wn * 64 + jj * 32 + (lane & 31);
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w |= residue(acc[i][jj][4 * gq + e], p, bar, p256) << (8 * e);
                    const int rdw = wm * 32 + i * 8 + 2 * gq + (lane >> 5);
                    lo[col * 64 + (rdw ^ (col & 31))] = w;
                }
            }
        __syncthreads();
        uint8_t *out = static_cast<uint8_t *>(g.out) + j * g.planeOut + (size_t)tn * 256 * g.ldo + (size_t)tm * 256;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
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
        if (tid < 512) rmax[tid] = 0;  // covers rmax[0..255] and cmax[0..255]
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                int v = max(abs(acc[i][0][rr]), abs(acc[i][1][rr]));
#pragma unroll
                for (int d = 16; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 32));
                if ((lane & 31) == 0) atomicMax(&rmax[wm * 128 + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5)], v);
            }
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            int v = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) v = max(v, abs(acc[i][jj][rr]));
            v = max(v, __shfl_xor(v, 32));
            if (lane < 32) atomicMax(&cmax[wn * 64 + jj * 32 + lane], v);
        }
        __syncthreads();
        if (tid < 256) {
            atomicMax(&g.rowmax[tm * 256 + tid], rmax[tid]);
            atomicMax(&g.colmax[tn * 256 + tid], cmax[tid]);
        }
    } else {  // RAW int32 (plane 0): validation path
        int32_t *out = static_cast<int32_t *>(g.out);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) {
                    const size_t row = (size_t)tm * 256 + wm * 128 + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
                    const size_t col = (size_t)tn * 256 + wn * 64 + jj * 32 + (lane & 31);
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
