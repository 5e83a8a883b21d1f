// Ablation probe for gemm_i8_kernel: times one cfg2-shaped launch (8192^3, N planes) of the
// product kernel compiled with -DOZ2_ABLATE=0/1/2 (full / no LDS-DMA / no MFMA).
#include "../../mixed-gemmul8_amd/csrc/gemm_i8.hip"
#include <cstdio>
int main(int argc, char **argv) {
    const size_t m = 8192, n = 8192, k = 8192;
    const unsigned N = argc > 1 ? atoi(argv[1]) : 4;
    oz2::Layout L = oz2::make_layout(m, n, k, N, false);
    void *w;
    if (hipMalloc(&w, L.total) != hipSuccess) return 1;
    (void)hipMemset(w, 1, L.total);
    oz2::ModParams MP = oz2::make_mod_params(N);
    int8_t *b = (int8_t *)w;
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, b + L.offR, nullptr, nullptr, MP, nullptr);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("ablate=%d N=%u: %.3f ms  %.0f TOPS\n", OZ2_ABLATE, N, ms, 2.0 * m * n * k * N / ms / 1e9);
    }
    return 0;
}
