// Where the one-tile residue product kernel's time goes at small sizes: m = n = argv[2]
// (default 1024), N = argv[1] planes (default 14), k in {64, 256, 1024, 2048}, 50 back-to-back launches per
// timing (events), random operand bytes; built per variant with -DOZ2_ABLATE (0 full, 10 no epilogue, 9 no
// residue stores, 7 residues = low byte, 6 no DMA in the main loop, 2 no MFMA, 1 no LDS-DMA at all), plus an
// empty kernel on the same grid (launch + dispatch floor).
#include "../../mixed-gemmul8_amd/csrc/gemm_i8.hip"
#include <cstdio>

namespace oz2 {  // split.hip's helper (not linked into this probe)
__global__ void zero_probe_kernel(int32_t *p, size_t n) {
    if (threadIdx.x < n) p[threadIdx.x] = 0;
}
void zero_i32(int32_t *p, size_t n, hipStream_t st) { zero_probe_kernel<<<1, 64, 0, st>>>(p, n); }
}  // namespace oz2

__global__ void fill_rand(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
        p[i] = x;
    }
}
__global__ __launch_bounds__(512, 1) void empty_kernel(int *p) {
    __shared__ int s[32768];
    if (threadIdx.x == 1023) p[0] = s[blockIdx.x];
}

int main(int argc, char **argv) {
    const unsigned N = argc > 1 ? atoi(argv[1]) : 14;
    const size_t m = argc > 2 ? atoll(argv[2]) : 1024, n = m;
    const size_t ks[] = {64, 256, 1024, 2048};
    oz2::g_persistent_override = 0;
    oz2::g_small_override = 0;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (size_t k : ks) {
        oz2::Layout L = oz2::make_layout(m, n, k, N, false);
        void *w;
        if (hipMalloc(&w, L.total) != hipSuccess) return 1;
        fill_rand<<<4096, 256>>>((uint32_t *)w, L.total / 4, 12345u);
        oz2::ModParams MP = oz2::make_mod_params(N);
        int8_t *b = (int8_t *)w;
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            for (int i = 0; i < 50; ++i)
                oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, b + L.offR, nullptr, nullptr, MP, nullptr);
            (void)hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) return 2;
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        float bestE = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            for (int i = 0; i < 50; ++i) empty_kernel<<<dim3((unsigned)(L.mtiles * L.ntiles), N), 512>>>((int *)w);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            bestE = ms < bestE ? ms : bestE;
        }
        printf("ABLATE=%d N=%u m=n=%zu k=%5zu ksteps=%3zu: %8.2f us per launch (empty kernel, same grid: %.2f us)\n",
               OZ2_ABLATE, N, m, k, L.ksteps, best * 20.0, bestE * 20.0);
        (void)hipFree(w);
    }
    return 0;
}
