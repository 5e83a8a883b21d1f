// Ablation probe for gemm_i8_kernel: times cfg2-shaped launches (8192^3, N planes) of the
// product kernel compiled with -DOZ2_ABLATE=0/1/2 (full / no LDS-DMA / no MFMA), on constant
// or random operand bytes (argv[2] = "rand": random data lowers the sustained clock).
#include "../../mixed-gemmul8_amd/csrc/gemm_i8.hip"
#include <cstdio>
#include <cstring>

__global__ void fill_rand(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
        p[i] = x;
    }
}

int main(int argc, char **argv) {
    const size_t m = 8192, n = 8192, k = argc > 3 ? atoll(argv[3]) : 8192;
    const unsigned N = argc > 1 ? atoi(argv[1]) : 4;
    const bool rnd = argc > 2 && !strcmp(argv[2], "rand");
    oz2::Layout L = oz2::make_layout(m, n, k, N, false);
    void *w;
    if (hipMalloc(&w, L.total) != hipSuccess) return 1;
    if (rnd) fill_rand<<<4096, 256>>>((uint32_t *)w, L.total / 4, 12345u);
    else (void)hipMemset(w, 1, L.total);
    oz2::ModParams MP = oz2::make_mod_params(N);
    int8_t *b = (int8_t *)w;
    for (int rep = 0; rep < 4; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, b + L.offR, nullptr, nullptr, MP, nullptr);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep) printf("%s stages=%d N=%u k=%zu %s: %.3f ms  %.0f TOPS\n", argv[0], OZ2_STAGES, N, k,
                        rnd ? "rand" : "const", ms, 2.0 * m * n * k * N / ms / 1e9);
    }
    return 0;
}
