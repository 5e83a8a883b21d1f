// Encode-kernel probe: times split_encode (fast mode, MODE 0) of an 8192 x 8192 f64 operand into
// 14 slice planes, for A (op N, strided vectors) and B (op N, contiguous vectors).
// Build variants with -DOZ2_ENC_ABLATE=1 (no residue arithmetic) / 2 (no loads).
#include "../../mixed-gemmul8_amd/csrc/split.hip"
#include <cstdio>
#include <algorithm>

__global__ void fill(double *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13;
        p[i] = ((double)(x & 0xffffff) / 16777216.0 - 0.5) * (1.0 + (double)((x >> 24) & 7));
    }
}
__global__ void fills(int16_t *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = -40;
}

int main() {
    using namespace oz2;
    const size_t m = 8192, n = 8192, k = 8192;
    const unsigned N = 14;
    Layout L = make_layout(m, n, k, N, false);
    double *X;
    int16_t *sft;
    int8_t *out;
    (void)hipMalloc(&X, m * k * 8);
    (void)hipMalloc(&sft, 16384 * 2);
    (void)hipMalloc(&out, L.planeA * N);
    fill<<<4096, 256>>>(X, m * k);
    fills<<<64, 256>>>(sft, 16384);
    ModParams MP = make_mod_params(N);
    for (int which = 0; which < 2; ++which) {
        OperandDesc d{X, which == 0 ? m : k, which == 1, true, false, false};
        float t[21];
        for (int rep = 0; rep < 21; ++rep) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            split_encode(d, which == 0, which == 0 ? m : n, k, sft, out, L.planeA, L, 0, MP, nullptr, false);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&t[rep], e0, e1);
        }
        std::sort(t + 1, t + 21);
        const float ms = t[10];
        printf("encode %s: median %.3f ms (min %.3f max %.3f)  %.2f TB/s\n", which ? "B (contig)" : "A (strided)", ms, t[1],
               t[20], (m * k * 8.0 + N * (double)m * k) / ms / 1e9);
    }
    return 0;
}
