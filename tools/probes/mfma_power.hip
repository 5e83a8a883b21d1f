// Data-dependent MFMA power probe: v_mfma_i32_32x32x32_i8 throughput and clock when the operand
// bytes follow different distributions.  Each wave holds 8 A and 8 B fragments in registers and
// cycles through all 64 (A, B) pairs, so operands change every instruction with no VALU work in
// the loop.  dist: 0 uniform [-128,127]; 1 symmetric residues mod 173 [-86,86]; 2 the same residues
// as [-45,127] (r + 173 for r < -45); 3 [0,127]; 4 [-64,63]; 5 constant bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int pick(unsigned x, int dist) {
    const int u = (int)(x >> 24);  // 0..255
    switch (dist) {
    case 0: return u - 128;
    case 1: return (int)((x >> 8) % 173u) - 86;
    case 2: { const int r = (int)((x >> 8) % 173u) - 86; return r < -45 ? r + 173 : r; }
    case 3: return u & 127;
    case 4: return (u & 127) - 64;
    default: return 3;
    }
}

__global__ __launch_bounds__(256) void k(int dist, int iters, int *out, long long *clk) {
    unsigned x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + 12345u;
    v4i A[8], B[8];
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int wa = 0, wb = 0;
            for (int b = 0; b < 4; ++b) {
                x = x * 1664525u + 1013904223u;
                wa |= (pick(x, dist) & 0xff) << (8 * b);
                x = x * 1664525u + 1013904223u;
                wb |= (pick(x, dist) & 0xff) << (8 * b);
            }
            A[f][q] = wa;
            B[f][q] = wb;
        }
    v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
    long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[0], B[j], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[1], B[(j + 1) & 7], c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[2], B[(j + 2) & 7], c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[3], B[(j + 3) & 7], c3, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[4], B[(j + 4) & 7], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[5], B[(j + 5) & 7], c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[6], B[(j + 6) & 7], c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[7], B[(j + 7) & 7], c3, 0, 0, 0);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

typedef int v4o __attribute__((ext_vector_type(4)));
// the same operand cycling with v_mfma_i32_16x16x64_i8 (16 cycles, half the ops of 32x32x32):
// 8 independent accumulators per wave
template <int NACC>
__global__ __launch_bounds__(256) void k16(int dist, int iters, int *out, long long *clk) {
    unsigned x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + 12345u;
    v4i A[8], B[8];
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int wa = 0, wb = 0;
            for (int b = 0; b < 4; ++b) {
                x = x * 1664525u + 1013904223u;
                wa |= (pick(x, dist) & 0xff) << (8 * b);
                x = x * 1664525u + 1013904223u;
                wb |= (pick(x, dist) & 0xff) << (8 * b);
            }
            A[f][q] = wa;
            B[f][q] = wb;
        }
    v4o c[NACC] = {};
    long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int f = 0; f < 8; ++f) {
                const int ci = (j * 8 + f) % NACC;
                c[ci] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[f], B[(j + f) & 7], c[ci], 0, 0, 0);
            }
    }
    long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    int sacc = 0;
    for (int f = 0; f < NACC; ++f) sacc += c[f][f & 3];
    out[blockIdx.x * 256 + threadIdx.x] = sacc;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
    const int blocks = 256 * 2, iters = 4000;
    int *out; long long *clk;
    (void)hipMalloc(&out, blocks * 256 * 4);
    (void)hipMalloc(&clk, blocks * 16);
    static long long h[2 * 512];
    const char *names[6] = {"uniform [-128,127]", "mod173 [-86,86]", "mod173 [-45,127]", "[0,127]", "[-64,63]", "constant"};
    for (int pass = 0; pass < 2; ++pass)
        for (int d = 0; d < 6; ++d) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            k<<<blocks, 256>>>(d, iters, out, clk);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
            double cyc = 0, rt = 0;
            for (int i = 0; i < blocks; ++i) { cyc += h[2 * i]; rt += h[2 * i + 1]; }
            const double total = 2.0 * 32 * 32 * 32 * 64.0 * iters * blocks * 4;
            if (pass) printf("%-20s %8.3f ms  %7.1f TOPS  clk %.3f GHz\n", names[d], ms, total / ms / 1e9, cyc / rt * 0.1);
        }
    // 16x16x64: 64 MFMAs per iteration of half the ops each; twice the iterations for the same work
    for (int acc : {8, 16, 32})
    for (int pass = 0; pass < 2; ++pass)
        for (int d : {0, 5}) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            if (acc == 8) k16<8><<<blocks, 256>>>(d, 2 * iters, out, clk);
            else if (acc == 16) k16<16><<<blocks, 256>>>(d, 2 * iters, out, clk);
            else k16<32><<<blocks, 256>>>(d, 2 * iters, out, clk);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
            double cyc = 0, rt = 0;
            for (int i = 0; i < blocks; ++i) { cyc += h[2 * i]; rt += h[2 * i + 1]; }
            const double total = 2.0 * 16 * 16 * 64 * 64.0 * 2 * iters * blocks * 4;
            if (pass) printf("16x16x64 acc%-2d %-9s %8.3f ms  %7.1f TOPS  clk %.3f GHz\n", acc, d == 0 ? "uniform" : "constant", ms,
                             total / ms / 1e9, cyc / rt * 0.1);
        }
    return 0;
}
