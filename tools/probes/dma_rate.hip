// Per-CU rate of 16-B/lane LDS-DMA (global_load_lds_dwordx4) and of global_load_dwordx4 into
// VGPRs, one block per CU, from an L2-resident source (each block re-reads its own 64 KiB) or a
// streamed one.  Prints bytes per CU per shader clock (clock from s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}

template <int MODE, int INFLIGHT>
__global__ void rate_kernel(const int8_t *src, size_t span, int iters, long long *clk, int *sink) {
    __shared__ __attribute__((aligned(1024))) int8_t smem[128 * 1024];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
    const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int8_t *)smem;
    const int8_t *base = src + (span == 65536 ? 0 : (size_t)blockIdx.x * span);
    long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    v4i acc = {0, 0, 0, 0};
#pragma unroll 8
    for (int it = 0; it < iters; ++it) {
        const size_t off = ((size_t)(it * nw + wave) * 1024) % span;
        if (MODE == 0) {
            glds16(base + off + lane * 16, lds + ((it * nw + wave) % 128) * 1024);
            __builtin_amdgcn_s_waitcnt((INFLIGHT & 15) | (7 << 4) | (15 << 8) | ((INFLIGHT >> 4) << 14));
        } else if (MODE == 1) {
            v4i x = *reinterpret_cast<const v4i *>(base + off + lane * 16);
            acc ^= x;
        } else {  // register staging: global_load_dwordx4 + ds_write_b128
            v4i x = *reinterpret_cast<const v4i *>(base + off + lane * 16);
            *reinterpret_cast<v4i *>(smem + ((it * nw + wave) % 128) * 1024 + lane * 16) = x;
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
    if (acc[0] == 12345) sink[0] = acc[1];
}

int main(int argc, char **argv) {
    const int mode = atoi(argv[1]);      // 0 = LDS-DMA, 1 = global_load_dwordx4
    const int threads = atoi(argv[2]);   // 256 / 512 / 1024
    const bool l2 = !strcmp(argv[3], "l2");
    const int blocks = 256, iters = 8192 * 512 / threads;
    const size_t span = l2 ? 65536 : (size_t)iters * (threads / 64) * 1024;
    int8_t *src;
    long long *clk;
    int *sink;
    (void)hipMalloc(&src, l2 ? 65536 : span * blocks);
    (void)hipMemset(src, 1, l2 ? 65536 : span * blocks);
    (void)hipMalloc(&clk, blocks * 16);
    (void)hipMalloc(&sink, 4);
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        if (mode == 0) rate_kernel<0, 8><<<blocks, threads>>>(src, span, iters, clk, sink);
        else if (mode == 1) rate_kernel<1, 8><<<blocks, threads>>>(src, span, iters, clk, sink);
        else rate_kernel<2, 8><<<blocks, threads>>>(src, span, iters, clk, sink);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        long long h[512];
        (void)hipMemcpy(h, clk, blocks * 16, hipMemcpyDeviceToHost);
        double cyc = 0, rt = 0;
        for (int b = 0; b < blocks; ++b) { cyc += h[2 * b]; rt += h[2 * b + 1]; }
        cyc /= blocks; rt /= blocks;
        const double bytes = (double)iters * (threads / 64) * 1024;
        printf("mode=%s threads=%d src=%s: %.3f ms, %.1f B/clk/CU, clock %.2f GHz, %.1f GB/s/CU\n",
               mode == 2 ? "vgpr+ds_write" : mode ? "vgpr" : "lds-dma", threads, l2 ? "l2" : "stream", ms, bytes / cyc, cyc / rt * 0.1,
               bytes / (ms * 1e-3) / 1e9);
    }
    return 0;
}
