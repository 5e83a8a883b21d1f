// Infinity-Cache (MALL) reuse probe for the split: does the encode's read of an operand band hit
// the MALL when the stats pass has just read it?  For bands of B (contiguous columns, k = 8192)
// of 256..8192 columns: time stats(band) -> encode(band) back to back, against the same encode
// after a 1 GiB sweep that flushes the MALL.
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
__global__ void sweep(const double4 *p, size_t n, double *sink) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i].x;
    if (s == 12345.678) *sink = s;
}

int main() {
    using namespace oz2;
    const size_t k = 8192, N = 14, nmax = 8192;
    double *X, *F, *sink;
    int16_t *sft;
    (void)hipMalloc(&X, nmax * k * 8);
    (void)hipMalloc(&F, (size_t)1 << 30);
    (void)hipMalloc(&sink, 8);
    (void)hipMalloc(&sft, nmax * 2);
    fill<<<4096, 256>>>(X, nmax * k);
    fill<<<4096, 256>>>(F, ((size_t)1 << 30) / 8);
    const ModParams MP = make_mod_params(N);
    for (size_t n : {256, 512, 1024, 2048, 4096, 8192}) {
        Layout L = make_layout(8192, n, k, N, false);
        int8_t *out;
        (void)hipMalloc(&out, L.planeB * N);
        OperandDesc d{X, k, true, true, false, false};
        hipEvent_t e[4];
        for (auto &x : e) (void)hipEventCreate(&x);
        float hot[9], cold[9], st[9];
        for (int rep = 0; rep < 9; ++rep) {
            sweep<<<4096, 256>>>((const double4 *)F, ((size_t)1 << 30) / 32, sink);
            (void)hipEventRecord(e[0]);
            split_stats(d, k, n, 128, false, oz2_log2M_fast[N - 2], sft, nullptr);
            (void)hipEventRecord(e[1]);
            split_encode(d, false, n, k, sft, out, L.planeB, L, 0, MP, nullptr);
            (void)hipEventRecord(e[2]);
            sweep<<<4096, 256>>>((const double4 *)F, ((size_t)1 << 30) / 32, sink);
            (void)hipEventRecord(e[3]);
            split_encode(d, false, n, k, sft, out, L.planeB, L, 0, MP, nullptr);
            hipEvent_t e4;
            (void)hipEventCreate(&e4);
            (void)hipEventRecord(e4);
            (void)hipEventSynchronize(e4);
            (void)hipEventElapsedTime(&st[rep], e[0], e[1]);
            (void)hipEventElapsedTime(&hot[rep], e[1], e[2]);
            (void)hipEventElapsedTime(&cold[rep], e[3], e4);
            (void)hipEventDestroy(e4);
        }
        std::sort(st, st + 9);
        std::sort(hot, hot + 9);
        std::sort(cold, cold + 9);
        const double bytes = n * k * 8.0;
        printf("band %5zu cols (%5.0f MB): stats %7.1f us (%.2f TB/s)  encode after stats %7.1f us  encode cold %7.1f us\n",
               n, bytes / 1e6, st[4] * 1e3, bytes / st[4] / 1e9, hot[4] * 1e3, cold[4] * 1e3);
        (void)hipFree(out);
    }
    return 0;
}
