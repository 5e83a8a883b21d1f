// Fixed cost of the one-tile residue product kernel at small shapes: m = n = 1024 (224 tiles at
// N = 14, one round over 256 CUs), k = 64 and 1024; builds with -DOZ2_ABLATE=0 / 9 (no residue
// stores) / 10 (no epilogue) / 1 (no LDS-DMA).  Back-to-back launches (stream time per launch) and
// single launches after a sync.
#include "../../mixed-gemmul8_amd/csrc/gemm_i8.hip"
#include <cstdio>

namespace oz2 {
void zero_i32(int32_t *p, size_t n, hipStream_t st) { (void)hipMemsetAsync(p, 0, n * 4, st); }
}  // namespace oz2

__global__ void fill_rand(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
        p[i] = x;
    }
}
__global__ void empty_kernel() {}

int main() {
    const unsigned N = 14;
    const size_t shapes[][2] = {{1024, 64}, {1024, 1024}, {1024, 4096}, {2048, 2048}, {1536, 1536}};
    for (auto &sh : shapes) {
        const size_t m = sh[0], n = sh[0], k = sh[1];
        oz2::Layout L = oz2::make_layout(m, n, k, N, false);
        void *w;
        if (hipMalloc(&w, L.total) != hipSuccess) return 1;
        fill_rand<<<4096, 256>>>((uint32_t *)w, L.total / 4, 12345u);
        oz2::ModParams MP = oz2::make_mod_params(N);
        int8_t *b = (int8_t *)w;
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        auto run = [&] { oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, b + L.offR, nullptr, nullptr, MP, nullptr); };
        for (int i = 0; i < 10; ++i) run();
        (void)hipDeviceSynchronize();
        const int R = 200;
        (void)hipEventRecord(e0);
        for (int i = 0; i < R; ++i) run();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        float single = 0;
        for (int i = 0; i < 20; ++i) {
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            run();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float s;
            (void)hipEventElapsedTime(&s, e0, e1);
            single += s / 20;
        }
        printf("stages=%d ablate=%d m=n=%zu k=%4zu N=14: back-to-back %.2f us/launch, single %.2f us\n", OZ2_STAGES, OZ2_ABLATE, m, k,
               ms * 1e3 / R, single * 1e3);
        (void)hipFree(w);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 200; ++i) empty_kernel<<<224, 512>>>();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("empty kernel 224 x 512: %.2f us/launch\n", ms * 1e3 / 200);
    return 0;
}
