// VALU issue cost of the instructions a residue epilogue can be built from (wave64 cycles per
// instruction on one SIMD): v_mul_hi_u32, v_mul_u32_u24, v_fma_f64, v_floor_f64, v_cvt_f64_u32,
// v_add_f64, v_perm_b32.  One wave per SIMD (4 per CU), 8 independent chains per lane, clock64
// around the loop.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void rate(unsigned *out, unsigned seed, long long *cyc) {
    unsigned u[8];
    double d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u[i] = seed * (threadIdx.x + 1) * (i + 3);
        d[i] = (double)(u[i] & 0xffff) + 0.25;
    }
    const double c1 = 0.003921568627450980, c2 = -3.0;
    const long long t0 = clock64();
#pragma unroll 1
    for (int it = 0; it < 1024; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) u[i] = __umulhi(u[i], 0x01010101u + i);
            if (OP == 1) u[i] = __umul24(u[i], 0x10101u + i);
            if (OP == 2) d[i] = __builtin_fma(d[i], c1, c2);
            if (OP == 3) d[i] = __builtin_floor(d[i] * 1.0000001);  // floor + mul
            if (OP == 4) d[i] = d[i] * 1.0000001;                    // mul alone (baseline for 3)
            if (OP == 5) d[i] = (double)(u[i] + (unsigned)it);        // cvt_f64_u32 (+ add)
            if (OP == 6) u[i] = __builtin_amdgcn_perm(u[i], u[(i + 1) & 7], 0x05040100u + i);
            if (OP == 7) u[i] = u[i] + (unsigned)it;                  // add (baseline for 5)
        }
    }
    const long long t1 = clock64();
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += u[i] + (unsigned)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    unsigned *out;
    long long *cyc, h;
    (void)hipMalloc(&out, 256 * 256 * 4);
    (void)hipMalloc(&cyc, 8);
    const char *names[] = {"v_mul_hi_u32", "v_mul_u32_u24", "v_fma_f64", "v_mul_f64+v_floor_f64", "v_mul_f64",
                           "v_add_u32+v_cvt_f64_u32", "v_perm_b32", "v_add_u32"};
#define RUN(op)                                                                                                  \
    for (int rep = 0; rep < 3; ++rep) {                                                                           \
        rate<op><<<256, 256>>>(out, 12345u, cyc);                                                                 \
        (void)hipDeviceSynchronize();                                                                             \
    }                                                                                                             \
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);                                                           \
    printf("%-26s %.2f cycles per wave-instruction (8 chains)\n", names[op], (double)h / (1024.0 * 8));
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7)
    return 0;
}
