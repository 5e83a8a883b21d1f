// A/B of the persistent residue product kernel's k order in one process (interleaved rounds, random operand
// bytes): ORD 0 (every tile k ascending, the default) and ORD 1 (serpentine: every other round of a queue k
// descending, so its first k-steps re-read the A panels the previous round read last); cfg2-shaped launches
// (m = n = 8192, N planes, k from argv[2]); checks that both write identical residues.  argv[6] = 0 / 1: that
// variant only (PMC passes: L2 hit rate and memory-side bytes per variant).
#define OZ2_ORDER_PROBES 1
#include "../../mixed-gemmul8_amd/csrc/gemm_i8.hip"
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>

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

int main(int argc, char **argv) {
    const unsigned N = argc > 1 ? atoi(argv[1]) : 14;
    const size_t k = argc > 2 ? atoll(argv[2]) : 8192;
    const size_t m = argc > 3 ? atoll(argv[3]) : 8192, n = argc > 4 ? atoll(argv[4]) : m;
    const int rounds = argc > 5 ? atoi(argv[5]) : 6;
    oz2::Layout L = oz2::make_layout(m, n, k, N, false);
    void *w;
    if (hipMalloc(&w, L.total) != hipSuccess) return 1;
    fill_rand<<<4096, 256>>>((uint32_t *)w, L.total / 4, 12345u);
    oz2::ModParams MP = oz2::make_mod_params(N);
    int8_t *b = (int8_t *)w;
    const size_t rbytes = (size_t)N * L.planeR;
    constexpr int NV = 2;
    const int only = argc > 6 ? atoi(argv[6]) : -1;
    uint8_t *R2[NV];
    for (int v = 0; v < NV; ++v)
        if (hipMalloc(&R2[v], rbytes) != hipSuccess) return 1;
    uint32_t *queue = reinterpret_cast<uint32_t *>(b + L.offQueue);
    std::vector<float> t[NV];
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < rounds; ++rep)
        for (int v = 0; v < NV; ++v) {
            if (only >= 0 && v != only) continue;
            oz2::g_persistent_override = 1;
            oz2::g_order_override = v;
            (void)hipEventRecord(e0);
            oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, (void *)R2[v], nullptr,
                         nullptr, MP, nullptr, queue);
            (void)hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return 2; }
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep) t[v].push_back(ms);
        }
    std::vector<uint8_t> h1(rbytes), h2(rbytes);
    bool same = true;
    (void)hipMemcpy(h1.data(), R2[0], rbytes, hipMemcpyDeviceToHost);
    for (int v = 1; v < NV && only < 0; ++v) {
        (void)hipMemcpy(h2.data(), R2[v], rbytes, hipMemcpyDeviceToHost);
        same = same && memcmp(h1.data(), h2.data(), rbytes) == 0;
    }
    for (int v = 0; v < NV; ++v) {
        if (t[v].empty()) continue;
        std::sort(t[v].begin(), t[v].end());
        printf("%s N=%u m=%zu n=%zu k=%zu: median %.3f ms min %.3f ms  %.0f TOPS\n", v == 0 ? "k ascending " : "k serpentine", N,
               m, n, k, t[v][t[v].size() / 2], t[v][0], 2.0 * m * n * L.k_pad * N / t[v][t[v].size() / 2] / 1e9);
    }
    printf("residues identical: %s\n", same ? "yes" : "NO");
    return same ? 0 : 3;
}
