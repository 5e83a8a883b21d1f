// Microbenchmark: sustained MFMA rate per instruction shape on gfx950 (operands in registers).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v4o __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ __launch_bounds__(256) void k(int iters, int *out, long long *clk) {
    v4i a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
    long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (SHAPE == 3) {  // 32x32x32 i8 with random operands that change every iteration
        unsigned x = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
        v4i ra, rb;
        for (int q = 0; q < 4; ++q) { x = x * 1664525u + 1013904223u; ra[q] = (int)x; x = x * 1664525u + 1013904223u; rb[q] = (int)x; }
        v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ra, rb, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(rb, ra, c1, 0, 0, 0);
            ra = ra.yzwx ^ (v4i){i, 0x5a5a5a5a, i * 3, 0x3c3c3c3c};
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ra, rb, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(rb, ra, c3, 0, 0, 0);
            rb = rb.wxyz ^ ra;
        }
        out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    } else if (SHAPE == 0) {  // 32x32x32 i8, 4 independent chains
        v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
        }
        out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    } else if (SHAPE == 1) {  // 16x16x64 i8
        v4o c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
        }
        out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    } else {  // 32x32x16 bf16
        v8s ab = {1, 2, 3, 4, 5, 6, 7, (short)threadIdx.x};
        v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, ab, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, ab, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, ab, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, ab, c3, 0, 0, 0);
        }
        out[blockIdx.x * 256 + threadIdx.x] = (int)(c0[0] + c1[1] + c2[2] + c3[3]);
    }
    long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
    const int blocks = 256 * 2, iters = 100000;
    int *out; long long *clk; hipMalloc(&out, blocks * 256 * 4); hipMalloc(&clk, blocks * 16);
    long long h[2 * 512];
    const char *names[4] = {"i32_32x32x32_i8", "i32_16x16x64_i8", "f32_32x32x16_bf16", "i8 32x32x32 random"};
    const double ops_per[4] = {2.0 * 32 * 32 * 32, 2.0 * 16 * 16 * 64, 2.0 * 32 * 32 * 16, 2.0 * 32 * 32 * 32};
    for (int s = 0; s < 4; ++s) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            if (s == 0) k<0><<<blocks, 256>>>(iters, out, clk);
            else if (s == 1) k<1><<<blocks, 256>>>(iters, out, clk);
            else if (s == 2) k<2><<<blocks, 256>>>(iters, out, clk);
            else k<3><<<blocks, 256>>>(iters, out, clk);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
            double cyc = 0, rt = 0; for (int i = 0; i < blocks; ++i) { cyc += h[2*i]; rt += h[2*i+1]; }
            cyc /= blocks; rt /= blocks;
            const double total = ops_per[s] * 4.0 * iters * blocks * 4;  // 4 waves/block
            printf("%-20s %8.3f ms  %8.1f TOPS   clk %.3f GHz   cycles/MFMA/wave %.1f\n", names[s], ms, total / ms / 1e9,
                   cyc / rt * 0.1, cyc / (4.0 * iters));
        }
    }
    return 0;
}
