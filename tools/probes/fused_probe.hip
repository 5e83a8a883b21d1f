// One-pass shift + slices of a contiguous f64 operand (split_fused_contig, defined here; measured
// and NOT taken into the library) against the two-pass form (stats_contig + encode), and the pair
// kernels of the current real NN fast split for scale: times (median of 21) and a bit-for-bit
// comparison of the shifts and the 14 slice planes.  Result (MI355X, 8192^3, N = 14,
// profiles/r02_probes/fused_*.txt): bit-identical, but 0.83 ms against 0.39 ms for the two passes;
// without slice stores (-DOZ2_ENC_ABLATE=4) still 0.41 ms: with a 64 KiB column per block only two
// blocks fit a CU, too few waves to hide the encode arithmetic, which the two-pass encode kernel
// (16 waves per CU) overlaps with its HBM traffic.
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off -DOCML_BASIC_ROUNDED_OPERATIONS \
//         -o fused_probe tools/probes/fused_probe.hip
#include "../../mixed-gemmul8_amd/csrc/split.hip"
#include <algorithm>
#include <cstdio>
#include <functional>
#include <vector>

namespace oz2 {
// ------------------------------------------------------------------
// Contiguous real f64 vectors (B op N, A op T) in fast mode with k <= 8192: shift and slices in ONE
// pass, so the operand is read from HBM once instead of twice.  A 256-thread block walks a list of
// vectors; each is staged in LDS (64 KiB + one pad double per 16 elements, so the chains' strided
// reads and the encode's 16-element reads are both conflict-free), its shift is computed from that
// copy exactly as the contiguous stats pass does (VT = 128 chains of round-up fmas in element order,
// the reference's wave tree and lane-1 / lane-33 pickup, compute_sft), and its slices are encoded
// from the same copy.  The next vector's loads are issued into registers before the current one's
// shift and slices, so the block's HBM reads never wait for its arithmetic.
// Vectors are dealt XCD-aware: the blocks of one XCD walk one contiguous range of vectors in
// lockstep, so the 16-B slice pieces of neighbouring vectors (which share 128-B lines of the panel
// layout) are written by co-running blocks of that XCD and merge in its L2.
// ------------------------------------------------------------------
constexpr int FUSED_KMAX = 8192;
constexpr int FUSED_NT = 256;
constexpr int FUSED_LOADS = FUSED_KMAX / FUSED_NT;  // prefetch registers per thread (doubles)
__device__ __forceinline__ int fused_idx(int e) { return e + (e >> 4); }
struct FusedShared {
    double col[FUSED_KMAX + FUSED_KMAX / 16];
    double grp[32];
    double gmax[8];
    int s;
};

__global__ __launch_bounds__(FUSED_NT, 2) void split_fused_contig_kernel(const double *__restrict__ X, size_t ld,
                                                                        size_t nvec, size_t len, size_t kblk,
                                                                        size_t vpad, float log2M,
                                                                        int16_t *__restrict__ sft_out,
                                                                        int8_t *__restrict__ out, size_t plane,
                                                                        size_t ksteps, ModParams MP, ModGroups G) {
    __shared__ FusedShared sh;
    // this block's vectors: XCD x owns the x-th of 8 contiguous ranges of [0, vpad); its nb blocks
    // take vectors lo + lb, lo + lb + nb, ...
    const unsigned nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7;
    const unsigned nb = (nwg >> 3) + (xcd < (nwg & 7) ? 1u : 0u), lb = bid >> 3;
    const size_t q8 = vpad >> 3, r8 = vpad & 7;
    const size_t lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
    const size_t hi = lo + q8 + (xcd < r8 ? 1 : 0);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int K = (int)kblk;

    double r[FUSED_LOADS];
    auto fetch = [&](size_t v) {  // elements [0, kblk) of vector v into registers (zeros beyond len / nvec)
        const int n = v < nvec ? (int)len : 0;
        const double *__restrict__ x = X + (v < nvec ? v : 0) * ld;
        if (n == FUSED_KMAX) {
#pragma unroll
            for (int u = 0; u < FUSED_LOADS; ++u) r[u] = x[u * FUSED_NT + tid];
        } else {
#pragma unroll
            for (int u = 0; u < FUSED_LOADS; ++u) {
                const int e = u * FUSED_NT + tid;
                r[u] = e < n ? x[e] : 0.0;
            }
        }
    };
    size_t v = lo + lb;
    if (v < hi) fetch(v);
    for (; v < hi; v += nb) {
        const bool valid = v < nvec;
        const int n = valid ? (int)len : 0;
#pragma unroll
        for (int u = 0; u < FUSED_LOADS; ++u) {
            const int e = u * FUSED_NT + tid;
            if (e < K) sh.col[fused_idx(e)] = r[u];
        }
        __syncthreads();
        if (v + nb < hi) fetch(v + nb);  // in flight under this vector's shift and slices

        // shift: stats_contig_body<double, false, 128, false> on the LDS copy (threads 0..127 are its
        // virtual threads; the others carry zeros through the same tree)
        double amax = 0, sum = 0;
        if (tid < 128)
            for (int e = tid; e < n; e += 128) accum<double, false>(sh.col[fused_idx(e)], 0.0, amax, sum);
        amax = wave_max<double>(amax);
        sum = ref_wave_sum<double>(sum);
        if (w < 2) {
            if (lane == 1) sh.grp[2 * w] = sum;
            if (lane == 33) sh.grp[2 * w + 1] = sum;
            if (lane == 0) sh.gmax[w] = amax;
        }
        __syncthreads();
        if (w == 0) {
            double mx = lane < 2 ? sh.gmax[lane] : 0.0;
            mx = wave_max<double>(mx);
            double s2 = (lane >= 32 && lane - 32 < 4) ? sh.grp[lane - 32] : 0.0;
            s2 = ref_wave_sum<double>(s2);
            const double nrm = __shfl(s2, 32);
            if (lane == 0) {
                const int sf = compute_sft(mx, nrm, log2M);
                sh.s = valid ? sf : 0;
                if (valid) sft_out[v] = (int16_t)(-sf);
            }
        }
        __syncthreads();

        // slices of the 16-element chunks c = tid, tid + 256, ...
        const int s = sh.s;
        for (int c = tid; c < K / 16; c += FUSED_NT) {
            double yr[16], yi[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                yr[q] = trunc(scalbn(sh.col[17 * c + q], s));  // fused_idx(16 c + q)
                yi[q] = 0.0;
            }
            encode_vec16<double, false, false, 0>(yr, yi, v, (size_t)16 * c, nvec, len, out, plane, ksteps, kblk,
                                                  vpad, 0, MP, G);
        }
        __syncthreads();  // the LDS copy is rewritten by the next vector
    }
}

bool split_fused_contig(const OperandDesc &d, bool is_A, size_t nvec, size_t len, int VT, float log2M, int16_t *sft,
                        int8_t *out, size_t plane, const Layout &L, const ModParams &MP, hipStream_t st) {
    if (!d.dbl || d.cplx || !d.contig || VT != 128 || L.kara || L.kblk == 0 || L.kblk > (size_t)FUSED_KMAX)
        return false;
    const size_t vpad = is_A ? L.m_pad : L.n_pad;
    const ModGroups G = make_groups(MP, L.N);
    // two blocks per CU (LDS), as many as there are vectors
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        ncu = 256;
    const size_t nblk = std::min(vpad, (size_t)(2 * ncu));
    split_fused_contig_kernel<<<dim3((unsigned)nblk), dim3(FUSED_NT), 0, st>>>(
        static_cast<const double *>(d.ptr), d.ld, nvec, len, L.kblk, vpad, log2M, sft, out, plane, L.ksteps, MP, G);
    return true;
}

}  // namespace oz2

__global__ void fill(double *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
        const double u = (double)(x & 0xffffff) / 16777216.0 - 0.5;
        p[i] = u * exp2((double)((int)((x >> 24) & 15) - 8) * 0.5);
    }
}

static float time_ms(const std::function<void()> &f) {
    float t[21];
    for (int rep = 0; rep < 21; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        f();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&t[rep], e0, e1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    std::sort(t + 1, t + 21);
    return t[10];
}

int main(int argc, char **argv) {
    using namespace oz2;
    const size_t m = argc > 1 ? atol(argv[1]) : 8192, n = argc > 2 ? atol(argv[2]) : 8192, k = argc > 3 ? atol(argv[3]) : 8192;
    const unsigned N = argc > 4 ? atoi(argv[4]) : 14;
    const Layout L = make_layout(m, n, k, N, false);
    const ModParams MP = make_mod_params(N);
    const float log2M = oz2_log2M_fast[N - 2];
    double *A, *B;
    int16_t *sA, *sB, *sB2;
    int8_t *outA, *outB, *outB2;
    (void)hipMalloc(&A, m * k * 8);
    (void)hipMalloc(&B, k * n * 8);
    (void)hipMalloc(&sA, L.m_pad * 2);
    (void)hipMalloc(&sB, L.n_pad * 2);
    (void)hipMalloc(&sB2, L.n_pad * 2);
    (void)hipMalloc(&outA, L.planeA * N);
    (void)hipMalloc(&outB, L.planeB * N);
    (void)hipMalloc(&outB2, L.planeB * N);
    fill<<<4096, 256>>>(A, m * k, 1);
    fill<<<4096, 256>>>(B, k * n, 2);
    (void)hipMemset(outB, 0x5a, L.planeB * N);
    (void)hipMemset(outB2, 0xa5, L.planeB * N);
    (void)hipMemset(sB, 0x11, L.n_pad * 2);
    (void)hipMemset(sB2, 0x22, L.n_pad * 2);
    OperandDesc dA{A, m, false, true, false, false};
    OperandDesc dB{B, k, true, true, false, false};

    const float tBs = time_ms([&] { split_stats(dB, k, n, 128, false, log2M, sB, nullptr); });
    const float tBe = time_ms([&] { split_encode(dB, false, n, k, sB, outB, L.planeB, L, 0, MP, nullptr); });
    const float tB2 = time_ms([&] {
        split_stats(dB, k, n, 128, false, log2M, sB, nullptr);
        split_encode(dB, false, n, k, sB, outB, L.planeB, L, 0, MP, nullptr);
    });
    bool ok = true;
    const float tF = time_ms([&] {
        ok = split_fused_contig(dB, false, n, k, 128, log2M, sB2, outB2, L.planeB, L, MP, nullptr);
    });
    const float tAs = time_ms([&] { split_stats(dA, k, m, 128, false, log2M, sA, nullptr); });
    const float tAe = time_ms([&] { split_encode(dA, true, m, k, sA, outA, L.planeA, L, 0, MP, nullptr); });
    const float tP = time_ms([&] {
        split_stats_pair(dA, m, dB, n, k, 128, log2M, sA, sB, nullptr);
        split_encode_pair(dA, m, dB, n, k, sA, sB, outA, outB, L, MP, nullptr);
    });
    const float tN = time_ms([&] {
        split_stats(dA, k, m, 128, false, log2M, sA, nullptr);
        split_encode(dA, true, m, k, sA, outA, L.planeA, L, 0, MP, nullptr);
        split_fused_contig(dB, false, n, k, 128, log2M, sB2, outB2, L.planeB, L, MP, nullptr);
    });
    const float tSP = time_ms([&] { split_stats_pair(dA, m, dB, n, k, 128, log2M, sA, sB, nullptr); });
    const float tS2 = time_ms([&] {
        split_stats(dA, k, m, 128, false, log2M, sA, nullptr);
        split_stats(dB, k, n, 128, false, log2M, sB, nullptr);
    });
    const float tEP = time_ms([&] { split_encode_pair(dA, m, dB, n, k, sA, sB, outA, outB, L, MP, nullptr); });
    const float tS2EP = time_ms([&] {
        split_stats(dA, k, m, 128, false, log2M, sA, nullptr);
        split_stats(dB, k, n, 128, false, log2M, sB, nullptr);
        split_encode_pair(dA, m, dB, n, k, sA, sB, outA, outB, L, MP, nullptr);
    });
    (void)hipDeviceSynchronize();
    if (hipGetLastError() != hipSuccess) { printf("HIP error\n"); return 1; }

    std::vector<int16_t> h1(n), h2(n);
    (void)hipMemcpy(h1.data(), sB, n * 2, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2.data(), sB2, n * 2, hipMemcpyDeviceToHost);
    std::vector<int8_t> p1(L.planeB * N), p2(L.planeB * N);
    (void)hipMemcpy(p1.data(), outB, p1.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(p2.data(), outB2, p2.size(), hipMemcpyDeviceToHost);
    size_t dsft = 0, dpl = 0;
    for (size_t i = 0; i < n; ++i) dsft += h1[i] != h2[i];
    for (size_t i = 0; i < p1.size(); ++i) dpl += p1[i] != p2[i];
    const double bB = k * n * 8.0, bS = N * (double)L.planeB;
    printf("shape m=%zu n=%zu k=%zu N=%u fused_applies=%d\n", m, n, k, N, (int)ok);
    printf("B stats (contig)        %.4f ms  %.2f TB/s\n", tBs, bB / tBs / 1e9);
    printf("B encode                %.4f ms  %.2f TB/s\n", tBe, (bB + bS) / tBe / 1e9);
    printf("B stats + encode        %.4f ms  %.2f TB/s (alg. 2 reads)\n", tB2, (2 * bB + bS) / tB2 / 1e9);
    printf("B fused                 %.4f ms  %.2f TB/s (1 read)\n", tF, (bB + bS) / tF / 1e9);
    printf("A stats (strided)       %.4f ms\n", tAs);
    printf("A encode                %.4f ms\n", tAe);
    printf("pair split (current)    %.4f ms\n", tP);
    printf("A stats+encode, B fused %.4f ms\n", tN);
    printf("stats pair              %.4f ms\n", tSP);
    printf("stats A; stats B        %.4f ms\n", tS2);
    printf("encode pair             %.4f ms\n", tEP);
    printf("stats A; stats B; enc pair %.4f ms\n", tS2EP);
    printf("mismatch: sft %zu of %zu, slice bytes %zu of %zu\n", dsft, n, dpl, p1.size());
    return 0;
}
