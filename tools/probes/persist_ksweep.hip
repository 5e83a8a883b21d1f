// Per-tile overhead of the persistent residue product kernel, measured as time per MAC against k-steps per tile
// (under the power cap, time ~ energy: DESIGN.md 9.2).  One process, interleaved rounds, random operand bytes,
// m = n = 8192 (argv[3]), N planes (argv[1]); for each k of {1024, 2048, 4096, 8192, 16384} the same kernel on a
// layout of that k inside one workspace.  A fit of ns per GMAC = Y + X / ksteps gives the per-tile overhead X in
// k-step equivalents.  argv[2] = EPIM variant (0 default f64 residue, 1 low byte only).
#define OZ2_EPIM_PROBES 1
#include "../../mixed-gemmul8_amd/csrc/gemm_i8.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

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
    oz2::g_epim_override = argc > 2 ? atoi(argv[2]) : 0;
    const size_t m = argc > 3 ? atoll(argv[3]) : 8192, n = m;
    const int rounds = argc > 4 ? atoi(argv[4]) : 5;
    const size_t ks[] = {1024, 2048, 4096, 8192, 16384};
    constexpr int NK = 5;
    oz2::Layout Ls[NK];
    size_t total = 0;
    for (int i = 0; i < NK; ++i) {
        Ls[i] = oz2::make_layout(m, n, ks[i], N, false);
        total = std::max(total, Ls[i].total);
    }
    void *w;
    if (hipMalloc(&w, total) != hipSuccess) return 1;
    fill_rand<<<4096, 256>>>((uint32_t *)w, total / 4, 12345u);
    oz2::ModParams MP = oz2::make_mod_params(N);
    oz2::g_persistent_override = 1;
    oz2::g_pg_override = 0;  // the block-epilogue kernel (this probe instruments it)
    std::vector<float> t[NK];
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < rounds; ++rep)
        for (int i = 0; i < NK; ++i) {
            const oz2::Layout &L = Ls[i];
            int8_t *b = (int8_t *)w;
            uint32_t *queue = reinterpret_cast<uint32_t *>(b + L.offQueue);
            (void)hipEventRecord(e0);
            oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, (void *)(b + L.offR), nullptr, nullptr, MP,
                         nullptr, queue);
            (void)hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return 2; }
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep) t[i].push_back(ms);
        }
    printf("EPIM=%d N=%u m=n=%zu\n", oz2::g_epim_override, N, m);
    double sx = 0, sy = 0, sxx = 0, sxy = 0;
    for (int i = 0; i < NK; ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med = t[i][t[i].size() / 2];
        const double gmac = (double)m * n * Ls[i].k_pad * N / 1e9;
        const double nspg = med * 1e6 / gmac;  // ns per GMAC
        const double inv = 1.0 / (double)Ls[i].ksteps;
        sx += inv; sy += nspg; sxx += inv * inv; sxy += inv * nspg;
        printf("k=%6zu ksteps=%4zu median %8.3f ms min %8.3f ms  %.4f ns/GMAC  %.0f TOPS\n", ks[i], Ls[i].ksteps, med, t[i][0],
               nspg, 2.0 * gmac / med / 1e3);
    }
    const double slope = (NK * sxy - sx * sy) / (NK * sxx - sx * sx), icpt = (sy - slope * sx) / NK;
    printf("fit ns/GMAC = %.4f + %.4f / ksteps: per-tile overhead = %.1f k-step equivalents\n", icpt, slope,
           slope / icpt);
    return 0;
}
