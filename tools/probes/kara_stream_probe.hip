// Probe: read bandwidth of the complex CRT's residue access patterns (cfg5: m = n = 4096, N = 12).
// Each lane reads one 8-byte word per stream for 8 consecutive rows of one column, as crt_kernel does,
// and folds them into one word (the CRT arithmetic left out).  Patterns:
//   0  Karatsuba sub-planes: N planes x 3 sub-planes of [n][m]          (36 streams of 512 B per wave)
//   1  the same bytes with P1 | P2 | P3 interleaved per 512-row chunk   (12 streams of 1.5 KB per wave)
//   2  big matrix: N planes of [n][2m], rows r and r + m                 (24 streams of 512 B per wave)
//   3  real: N planes of [n][m]                                           (12 streams)
// hipcc -O3 --offload-arch=gfx950 kara_stream_probe.hip -o kara_stream_probe && ./kara_stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int N = 12;
constexpr size_t M = 4096, NC = 4096;

template <int PAT>
__global__ __launch_bounds__(256) void probe(const uint8_t *R, uint64_t *out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t col = blockIdx.y;
    const size_t rows = PAT == 2 ? 2 * M : M;
    const size_t r0 = ((size_t)blockIdx.x * 256 + wv * 64) * 8 + lane * 8;
    if (r0 >= M) return;
    uint64_t acc = 0;
    if (PAT == 0) {
        const size_t plane = 3 * M * NC, sub = M * NC;
#pragma unroll
        for (int j = 0; j < N; ++j)
#pragma unroll
            for (int s = 0; s < 3; ++s) acc ^= *(const uint64_t *)(R + j * plane + s * sub + col * M + r0);
    } else if (PAT == 1) {
        const size_t plane = 3 * M * NC;
        const size_t base = col * 3 * M + (r0 / 512) * 1536 + r0 % 512;
#pragma unroll
        for (int j = 0; j < N; ++j)
#pragma unroll
            for (int s = 0; s < 3; ++s) acc ^= *(const uint64_t *)(R + j * plane + base + s * 512);
    } else if (PAT == 2) {
        const size_t plane = rows * NC;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            acc ^= *(const uint64_t *)(R + j * plane + col * rows + r0);
            acc ^= *(const uint64_t *)(R + j * plane + col * rows + M + r0);
        }
    } else {
        const size_t plane = M * NC;
#pragma unroll
        for (int j = 0; j < N; ++j) acc ^= *(const uint64_t *)(R + j * plane + col * M + r0);
    }
    if (acc == 0x123456789abcdefull) out[0] = acc;  // keeps the loads
}

template <int PAT> double run(const uint8_t *R, uint64_t *out, size_t bytes) {
    dim3 grid((unsigned)(M / 2048), (unsigned)NC);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) probe<PAT><<<grid, 256>>>(R, out);
    hipEventRecord(a);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) probe<PAT><<<grid, 256>>>(R, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return bytes / (ms / reps * 1e-3) / 1e9;
}

int main() {
    const size_t total = (size_t)N * 3 * M * NC;
    uint8_t *R;
    uint64_t *out;
    if (hipMalloc(&R, total) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(R, 1, total);
    printf("karatsuba sub-planes (36 streams): %.0f GB/s\n", run<0>(R, out, total));
    printf("interleaved sub-planes (12 x 1.5 KB): %.0f GB/s\n", run<1>(R, out, total));
    printf("big matrix (24 streams): %.0f GB/s\n", run<2>(R, out, (size_t)N * 2 * M * NC));
    printf("real (12 streams): %.0f GB/s\n", run<3>(R, out, (size_t)N * M * NC));
    printf("karatsuba again: %.0f GB/s\n", run<0>(R, out, total));
    printf("interleaved again: %.0f GB/s\n", run<1>(R, out, total));
    hipFree(R);
    hipFree(out);
    return 0;
}
