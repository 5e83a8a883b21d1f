// Where a persistent product block's cycles go per tile: the kernel built with OZ2_STAMPS=1 sums
// s_memtime deltas per wave over [0] realign barriers, [1] residues -> LDS, [2] park barrier,
// [3] residue stores + barrier, [4] accumulator reset + stagger barrier, [5] k-step 0, [6] k-step 1,
// [7] the other k-steps; printed per tile, averaged over blocks, for wave 0 (group 0) and wave 4
// (group 1).  Random operand bytes, cfg2-shaped launch (m = n from argv[3], N, k from argv).
// (The barrier-free epilogue variant it was also run on lives in git history, commit 39a29fd.)
#define OZ2_STAMPS 1
#include "../../mixed-gemmul8_amd/csrc/gemm_i8.hip"
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
    const size_t k = argc > 2 ? atoll(argv[2]) : 8192;
    const size_t m = argc > 3 ? atoll(argv[3]) : 8192, n = m;
    oz2::Layout L = oz2::make_layout(m, n, k, N, false);
    void *w;
    if (hipMalloc(&w, L.total) != hipSuccess) return 1;
    fill_rand<<<4096, 256>>>((uint32_t *)w, L.total / 4, 12345u);
    oz2::ModParams MP = oz2::make_mod_params(N);
    int8_t *b = (int8_t *)w;
    const size_t nst = 4096 * 8 * 9;
    unsigned long long *st;
    if (hipMalloc(&st, nst * 8) != hipSuccess) return 1;
    (void)hipMemset(st, 0, nst * 8);
    oz2::g_persistent_override = 1;
    oz2::g_pg_override = 0;  // the block-epilogue kernel (this probe instruments it)
    uint32_t *queue = reinterpret_cast<uint32_t *>(b + L.offQueue);
    for (int rep = 0; rep < 4; ++rep) {
        oz2::g_stamps = rep == 3 ? st : nullptr;  // the last launch records
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        oz2::gemm_i8(b + L.offA, b + L.offB, L, N, oz2::Epi::RESIDUE, b + L.offR, nullptr, nullptr, MP, nullptr, queue);
        (void)hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return 2; }
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("launch %d: %.3f ms\n", rep, ms);
    }
    std::vector<unsigned long long> h(nst);
    (void)hipMemcpy(h.data(), st, nst * 8, hipMemcpyDeviceToHost);
    const char *names[8] = {"realign", "residues->LDS", "park barrier", "stores+barrier", "acc reset+stagger",
                            "k-step 0", "k-step 1", "other k-steps"};
    for (int wv : {0, 4}) {
        double sum[9] = {};
        int blocks = 0;
        for (int blk = 0; blk < 4096; ++blk) {
            const unsigned long long *q = &h[((size_t)blk * 8 + wv) * 9];
            if (q[8] == 0) continue;
            ++blocks;
            for (int i = 0; i < 9; ++i) sum[i] += (double)q[i];
        }
        if (!blocks) continue;
        const double tiles = sum[8];
        printf("wave %d (%d blocks, %.1f tiles per block), cycles per tile:\n", wv, blocks, tiles / blocks);
        double tot = 0;
        for (int i = 0; i < 8; ++i) tot += sum[i];
        for (int i = 0; i < 8; ++i)
            printf("  %-18s %9.0f  (%4.1f %%)\n", names[i], sum[i] / tiles, 100.0 * sum[i] / tot);
        printf("  %-18s %9.0f  (per k-step in the other k-steps: %.0f)\n", "total", tot / tiles,
               sum[7] / tiles / ((double)L.ksteps - 2));
    }
    return 0;
}
