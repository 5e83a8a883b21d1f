// Is the CRT at the copy rate?  cfg2's CRT (m = n = 8192, N = 14 residue planes, f64 C) against a
// kernel with the same memory pattern and no arithmetic: per lane one 8-byte non-temporal load from each of the N
// planes (8 rows of one column), then 64 bytes of C as four 16-byte non-temporal stores (8 rows x 8 B), 256-thread
// blocks, 4 columns per block as the CRT's default from n = 4096.  Interleaved, 10 rounds, events.
#include "../../mixed-gemmul8_amd/csrc/crt.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

template <unsigned N>
__global__ __launch_bounds__(256) void copy_pattern(const uint8_t *R, size_t planeR, size_t ldr, size_t m, size_t n,
                                                    double *C, size_t ldc) {
    typedef const __attribute__((address_space(1))) uint64_t *GW;
    const size_t r0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (r0 >= m) return;
    for (size_t col = blockIdx.y; col < n; col += gridDim.y) {
        uint64_t w[N];
#pragma unroll
        for (unsigned i = 0; i < N; ++i) w[i] = __builtin_nontemporal_load((GW)(R + i * planeR + col * ldr + r0));
        uint64_t x = 0;
#pragma unroll
        for (unsigned i = 0; i < N; ++i) x ^= w[i];
        // C stores as the CRT issues them after its LDS transpose: 16 bytes per lane, lanes adjacent (the wave's
        // 512 rows = 4 KiB of the column in four 1 KiB store instructions)
        typedef int i4v __attribute__((ext_vector_type(4)));
        i4v v = {(int)x, (int)(x >> 32), (int)x, (int)(x >> 32)};
        const int lane = threadIdx.x & 63;
        i4v *dst = reinterpret_cast<i4v *>(C + col * ldc + (r0 - (size_t)lane * 8));
#pragma unroll
        for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(v, dst + q * 64 + lane);
    }
}

int main() {
    const size_t m = 8192, n = 8192, k = 8192;
    const unsigned N = 14;
    oz2::Layout L = oz2::make_layout(m, n, k, N, false);
    uint8_t *R;
    double *C;
    int16_t *sft;
    if (hipMalloc(&R, L.planeR * N) || hipMalloc(&C, m * n * 8) || hipMalloc(&sft, (m + n) * 2)) return 1;
    (void)hipMemset(R, 3, L.planeR * N);
    (void)hipMemset(sft, 0, (m + n) * 2);
    const oz2::CrtParams CP = oz2::make_crt_params(N, false);
    const double one = 1.0, zero = 0.0;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> tc, tp;
    const double bytes = (double)N * m * n + 8.0 * m * n;
    for (int rep = 0; rep < 11; ++rep) {
        float ms;
        (void)hipEventRecord(e0);
        oz2::crt_inverse(R, L, sft, sft + m, CP, oz2::OutType::F64, &one, &zero, C, m, nullptr, 0);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep) tc.push_back(ms);
        (void)hipEventRecord(e0);
        copy_pattern<14><<<dim3((unsigned)(m / 2048), (unsigned)(n / 4)), 256>>>(R, L.planeR, L.ldr, m, n, C, m);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep) tp.push_back(ms);
    }
    std::sort(tc.begin(), tc.end());
    std::sort(tp.begin(), tp.end());
    printf("cfg2 CRT        median %.4f ms  %.2f TB/s (%.3f GB)\n", tc[5], bytes / tc[5] / 1e9, bytes / 1e9);
    printf("copy pattern    median %.4f ms  %.2f TB/s\n", tp[5], bytes / tp[5] / 1e9);
    printf("CRT / copy = %.3f\n", tc[5] / tp[5]);
    return 0;
}
