// Write-bandwidth probe for the encode's store pattern: 940 MB of 16-byte stores into 14 planes.
//   pattern 0: linear (each wave stores 1 KiB contiguous, grid-stride)
//   pattern 1: the encode's A order (64-vector x 64-k tile -> per plane two 2 KiB pieces in one
//              16 KiB panel; consecutive blocks walk vectors: panels 2 MiB apart)
//   pattern 2: the encode's B order (k-first: consecutive blocks walk k -> consecutive panels)
// Each with the plane stride exact (power of two) or padded by `pad` bytes, plain or nt stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr size_t M = 8192, K = 8192, NPL = 14;
constexpr size_t PANEL = 16384, KSTEPS = K / 64;

__device__ __forceinline__ size_t panel_offset(size_t v, size_t kk) {
    const size_t tile = v >> 8, vb = v & 255, blk = vb >> 5, r = vb & 31;
    const size_t ks = kk >> 6, kin = kk & 63, s = kin >> 5, h = (kin >> 4) & 1;
    return (tile * KSTEPS + ks) * PANEL + s * 8192 + blk * 1024 + h * 512 + r * 16;
}

template <int PAT, bool NT>
__global__ __launch_bounds__(256) void wr(int8_t *out, size_t plane) {
    const int tid = threadIdx.x;
    const v4u val = {(unsigned)tid, blockIdx.x, blockIdx.y, 7u};
    if (PAT == 0) {
        // same number of 16-B stores per block as the encode (14 per thread), linear
        const size_t blin = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
        for (int j = 0; j < (int)NPL; ++j) {
            v4u *p = reinterpret_cast<v4u *>(out + j * plane + blin * 4096 + tid * 16);
            if (NT) __builtin_nontemporal_store(val, p); else *p = val;
        }
        return;
    }
    const bool kfirst = PAT == 2;
    const size_t v0 = (size_t)(kfirst ? blockIdx.y : blockIdx.x) * 64;
    const size_t e0 = (size_t)(kfirst ? blockIdx.x : blockIdx.y) * 64;
    const int vl = tid & 63, c = tid >> 6;
    const size_t off = panel_offset(v0 + vl, e0 + 16 * c);
    for (int j = 0; j < (int)NPL; ++j) {
        v4u *p = reinterpret_cast<v4u *>(out + j * plane + off);
        if (NT) __builtin_nontemporal_store(val, p); else *p = val;
    }
}

int main() {
    const size_t base = M * K;  // 64 MiB per plane
    int8_t *out;
    (void)hipMalloc(&out, NPL * (base + (1 << 20)));
    const size_t pads[3] = {0, 4096 + 256, 1 << 20};
    for (int pat = 0; pat < 3; ++pat)
        for (int nt = 0; nt < 2; ++nt)
            for (int pi = 0; pi < 3; ++pi) {
                const size_t plane = base + pads[pi];
                dim3 grid = pat == 2 ? dim3(K / 64, M / 64) : dim3(M / 64, K / 64);
                float t[11];
                for (int rep = 0; rep < 11; ++rep) {
                    hipEvent_t e0, e1;
                    (void)hipEventCreate(&e0);
                    (void)hipEventCreate(&e1);
                    (void)hipEventRecord(e0);
                    if (pat == 0) { if (nt) wr<0, true><<<grid, 256>>>(out, plane); else wr<0, false><<<grid, 256>>>(out, plane); }
                    else if (pat == 1) { if (nt) wr<1, true><<<grid, 256>>>(out, plane); else wr<1, false><<<grid, 256>>>(out, plane); }
                    else { if (nt) wr<2, true><<<grid, 256>>>(out, plane); else wr<2, false><<<grid, 256>>>(out, plane); }
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    (void)hipEventElapsedTime(&t[rep], e0, e1);
                }
                std::sort(t + 1, t + 11);
                printf("pattern %d nt %d pad %7zu: %.3f ms  %.2f TB/s\n", pat, nt, pads[pi], t[5], NPL * base / t[5] / 1e9);
            }
    return 0;
}
