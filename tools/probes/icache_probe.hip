// Is the instruction cache cold at every dispatch?  Straight-line kernels of NI independent VALU ops
// (8 bytes each) on 256 blocks x 256 threads, launched back to back (100 launches each, events): if the time per
// launch grows with the code size well beyond NI x 4 cycles, the code is fetched from L2 at every dispatch.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NI>
__global__ void straight(int *out, int x) {
    int a = x + threadIdx.x, b = x ^ 5, c = x * 3, d = x - 7;
#pragma unroll
    for (int i = 0; i < NI / 4; ++i) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(b) : "v"(c));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(c) : "v"(d));
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(a));
    }
    if (a + b + c + d == 0x12345) out[threadIdx.x] = a;
}

template <int NI>
void run(int *o) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 5; ++w) straight<NI><<<256, 256>>>(o, w);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 100; ++i) straight<NI><<<256, 256>>>(o, i);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("NI=%6d code ~%6d B: %8.2f us per launch (%.1f ns per instruction)\n", NI, NI * 8, ms * 10.0,
           ms * 1e4 / NI);
}

int main() {
    int *o;
    if (hipMalloc(&o, 4096) != hipSuccess) return 1;
    run<64>(o);
    run<256>(o);
    run<1024>(o);
    run<2048>(o);
    run<4096>(o);
    run<8192>(o);
    return 0;
}
