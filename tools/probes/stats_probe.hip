// Stats pass (fast-mode shifts of A rows + B columns, stats_pair_kernel) timed alone across sizes,
// with a checksum of the shifts so that builds with different loads in flight can be compared:
//   hipcc ... -DOZ2_STRIDED_LOADS=16 -DOZ2_CONTIG_LOADS=8 stats_probe.hip
#include "../../mixed-gemmul8_amd/csrc/split.hip"
#include <cstdio>
#include <vector>

__global__ void fill(double *x, size_t n, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
        h ^= h >> 31; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 27;
        const double u = (double)(h >> 11) * 0x1p-53;
        x[i] = (u - 0.5) * exp2((double)((int)(h & 15) - 8));
    }
}

int main() {
    const size_t sizes[] = {1024, 2048, 4096, 8192};
    for (size_t s : sizes) {
        const size_t m = s, n = s, k = s;
        double *A, *B;
        int16_t *sft;
        hipMalloc(&A, m * k * 8);
        hipMalloc(&B, k * n * 8);
        hipMalloc(&sft, (m + n) * 2);
        fill<<<4096, 256>>>(A, m * k, 1);
        fill<<<4096, 256>>>(B, k * n, 2);
        oz2::OperandDesc dA{A, m, false, true, false, false}, dB{B, k, true, true, false, false};
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int i = 0; i < 5; ++i) oz2::split_stats_pair(dA, m, dB, n, k, 128, 30.5f, sft, sft + m, nullptr);
        const int R = 50;
        hipEventRecord(e0, nullptr);
        for (int i = 0; i < R; ++i) oz2::split_stats_pair(dA, m, dB, n, k, 128, 30.5f, sft, sft + m, nullptr);
        hipEventRecord(e1, nullptr);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<int16_t> h(m + n);
        hipMemcpy(h.data(), sft, (m + n) * 2, hipMemcpyDeviceToHost);
        uint64_t cs = 0;
        for (size_t i = 0; i < m + n; ++i) cs = cs * 1000003 + (uint16_t)h[i];
        const double us = ms * 1e3 / R;
        printf("strided %d contig %d size %5zu: %8.2f us  %5.2f TB/s  checksum %016llx\n", OZ2_STRIDED_LOADS,
               OZ2_CONTIG_LOADS, s, us, 2.0 * s * s * 8 / (us * 1e-6) / 1e12, (unsigned long long)cs);
        hipFree(A);
        hipFree(B);
        hipFree(sft);
    }
    return 0;
}
