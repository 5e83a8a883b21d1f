// A/B of the persistent residue product's epilogue (round 6): gemm_i8_persistent_kernel (block-wide epilogue after
// realigning the two wave groups; variant 0) against gemm_i8_persistent_pg_kernel (per-group epilogues, no
// realignment, accumulators started by the first MFMA; variant 1), in one process, interleaved rounds, random
// operand bytes, m = n = argv[2] (default 8192), N = argv[1] planes (default 14), k in {1024 ... 16384}.
// Prints per variant the ns per GMAC for each k and the fit Y + X / ksteps (X / Y = the per-tile overhead in k-step
// equivalents, as tools/probes/persist_ksweep.hip), and checks that both variants write identical residue planes.
// argv[4] = 5 adds the ablations of variant 1: residues reduced to the low byte, no residue stores, no park / stores.
#define OZ2_PG_PROBES 1
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
__global__ void hash_kernel(const uint32_t *p, size_t n, unsigned long long *out) {
    unsigned long long h = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        h += (unsigned long long)p[i] * (2 * i + 1);
    for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, h);
}

int main(int argc, char **argv) {
    const unsigned N = argc > 1 ? atoi(argv[1]) : 14;
    const size_t m = argc > 2 ? atoll(argv[2]) : 8192, n = m;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const int NV = argc > 4 ? atoi(argv[4]) : 2;  // 2: variants 0, 1; 5: also the ablations 2, 3, 4 of variant 1
    const size_t ks[] = {1024, 2048, 4096, 8192, 16384};
    constexpr int NK = 5;
    oz2::Layout Ls[NK];
    size_t total = 0;
    for (int i = 0; i < NK; ++i) {
        Ls[i] = oz2::make_layout(m, n, ks[i], N, false);
        total = std::max(total, Ls[i].total);
    }
    void *w;
    unsigned long long *hd;
    if (hipMalloc(&w, total) != hipSuccess || hipMalloc(&hd, 8) != hipSuccess) return 1;
    fill_rand<<<4096, 256>>>((uint32_t *)w, total / 4, 12345u);
    oz2::ModParams MP = oz2::make_mod_params(N);
    oz2::g_persistent_override = 1;
    std::vector<float> t[5][NK];
    unsigned long long hs[5][NK] = {};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < rounds; ++rep)
        for (int i = 0; i < NK; ++i)
            for (int v = 0; v < NV; ++v) {
                oz2::g_pg_override = v;
                const oz2::Layout &L = Ls[i];
                int8_t *b = (int8_t *)w;
                uint32_t *queue = reinterpret_cast<uint32_t *>(b + L.offQueue);
                (void)hipMemsetAsync(b + L.offR, 0x5a, L.planeR * N, nullptr);
                (void)hipEventRecord(e0);
                oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, (void *)(b + L.offR), nullptr, nullptr,
                             MP, nullptr, queue);
                (void)hipEventRecord(e1);
                if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return 2; }
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (rep) t[v][i].push_back(ms);
                if (rep == 0) {
                    (void)hipMemset(hd, 0, 8);
                    hash_kernel<<<1024, 256>>>((const uint32_t *)(b + L.offR), L.planeR * N / 4, hd);
                    (void)hipMemcpy(&hs[v][i], hd, 8, hipMemcpyDeviceToHost);
                }
            }
    int bad = 0;
    for (int v = 0; v < NV; ++v) {
        static const char *names[] = {"block epilogue", "per-group epilogue", "per-group, residues = low byte (wrong)",
                                      "per-group, no residue stores", "per-group, no park / stores"};
        printf("variant %d (%s) N=%u m=n=%zu\n", v, names[v], N, m);
        double sx = 0, sy = 0, sxx = 0, sxy = 0;
        for (int i = 0; i < NK; ++i) {
            std::sort(t[v][i].begin(), t[v][i].end());
            const double med = t[v][i][t[v][i].size() / 2];
            const double gmac = (double)m * n * Ls[i].k_pad * N / 1e9;
            const double nspg = med * 1e6 / gmac;
            const double inv = 1.0 / (double)Ls[i].ksteps;
            sx += inv; sy += nspg; sxx += inv * inv; sxy += inv * nspg;
            printf("k=%6zu ksteps=%4zu median %8.4f ms min %8.4f ms  %.4f ns/GMAC  residue hash %016llx%s\n", ks[i],
                   Ls[i].ksteps, med, t[v][i][0], nspg, hs[v][i], hs[v][i] == hs[0][i] || v >= 2 ? "" : "  MISMATCH");
            bad += v < 2 && hs[v][i] != hs[0][i];
        }
        const double slope = (NK * sxy - sx * sy) / (NK * sxx - sx * sx), icpt = (sy - slope * sx) / NK;
        printf("fit ns/GMAC = %.4f + %.4f / ksteps: per-tile overhead = %.2f k-step equivalents\n", icpt, slope,
               slope / icpt);
    }
    printf(bad ? "RESIDUES DIFFER\n" : "residues identical\n");
    return bad ? 3 : 0;
}
