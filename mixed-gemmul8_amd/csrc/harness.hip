// harness.hip -- bench/test utilities exported through the C ABI (not on the emulation path).
//
//  * gemmul8_randmat: the reference test drivers' input generator
//    (GEMMul8/testing/make_matrix.hpp:8-71): hiprand XORWOW, init(seed, idx, 0),
//    x = (u - 0.5) * exp(phi * n); same library, same stream of draws.
//  * gemmul8_dd_gemm: double-double reference product (testing/eval.hpp:265-308),
//    TwoProd + double-double accumulation, LDS-tiled.
//  * gemmul8_relerr_dd: |C - Cref| / |Cref| in double-double (eval.hpp:317-338).
//  * gemmul8_time_gemm / gemmul8_time_vendor_gemm: the drivers' timing loop in native code
//    (test_double.cu:318-331, 422-431): per call a device sync, the host clock, the call, a device sync,
//    the clock -- without the Python binding's per-call overhead, for the emulation and the vendor GEMM alike.
#include <hip/hip_runtime.h>
#include <hipblas/hipblas.h>
#include <hiprand/hiprand_kernel.h>

#include <chrono>
#include <mutex>

#include "../../include/gemmul8_c.h"

namespace oz2h {

template <typename T>
__global__ void randmat_kernel(size_t total, T *A, double phi, unsigned long long seed) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    hiprandState_t state;
    hiprand_init(seed, idx, 0, &state);
    const T u = static_cast<T>(hiprand_uniform_double(&state));
    const T nn = static_cast<T>(hiprand_normal_double(&state));
    A[idx] = static_cast<T>((u - 0.5) * exp(nn * static_cast<T>(phi)));
}

template <typename T>
__global__ void randmat_c_kernel(size_t total, T *A, double phi, unsigned long long seed) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    hiprandState_t state;
    hiprand_init(seed, idx, 0, &state);
    const T ur = static_cast<T>(hiprand_uniform_double(&state));
    const T nr = static_cast<T>(hiprand_normal_double(&state));
    const T ui = static_cast<T>(hiprand_uniform_double(&state));
    const T ni = static_cast<T>(hiprand_normal_double(&state));
    A[2 * idx] = static_cast<T>((ur - 0.5) * exp(nr * static_cast<T>(phi)));
    A[2 * idx + 1] = static_cast<T>((ui - 0.5) * exp(ni * static_cast<T>(phi)));
}

// ---- double-double helpers (eval.hpp:22-110 semantics) ----
__device__ __forceinline__ void two_sum(double a, double b, double &c, double &d) {
    c = a + b;
    const double s = c - a, t = b - s, u = c - s;
    d = (a - u) + t;
}
__device__ __forceinline__ void fast_two_sum(double a, double b, double &c, double &d) {
    c = a + b;
    d = (a - c) + b;
}
__device__ __forceinline__ void dd_add(double a1, double a2, double b1, double b2, double &c1, double &c2) {
    two_sum(a1, b1, c1, c2);
    c2 += a2;
    c2 += b2;
    fast_two_sum(c1, c2, c1, c2);
}

// C1 + C2 = A * B, 64x64 output tile per 256-thread block, 4x4 outputs per thread
__global__ __launch_bounds__(256) void dd_gemm_kernel(size_t m, size_t n, size_t k, const double *__restrict__ A,
                                                      const double *__restrict__ B, double *C1, double *C2) {
    __shared__ double As[16][65];
    __shared__ double Bs[16][65];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const size_t r0 = (size_t)blockIdx.x * 64, c0 = (size_t)blockIdx.y * 64;
    double s1[4][4] = {}, s2[4][4] = {};
    for (size_t kk = 0; kk < k; kk += 16) {
        for (int i = threadIdx.x; i < 16 * 64; i += 256) {
            const int rr = i & 63, kq = i >> 6;
            const size_t r = r0 + rr, kx = kk + kq;
            As[kq][rr] = (r < m && kx < k) ? A[kx * m + r] : 0.0;
            const int cc = i >> 4, kq2 = i & 15;
            const size_t c = c0 + cc, ky = kk + kq2;
            Bs[kq2][cc] = (c < n && ky < k) ? B[c * k + ky] : 0.0;
        }
        __syncthreads();
#pragma unroll 4
        for (int q = 0; q < 16; ++q) {
            double a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[q][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[q][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double p1 = a[i] * b[j];
                    const double p2 = __builtin_fma(a[i], b[j], -p1);
                    dd_add(p1, p2, s1[i][j], s2[i][j], s1[i][j], s2[i][j]);
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const size_t r = r0 + ty + 16 * i, c = c0 + tx + 16 * j;
            if (r < m && c < n) {
                C1[c * m + r] = s1[i][j];
                C2[c * m + r] = s2[i][j];
            }
        }
}

__global__ void relerr_kernel(size_t count, const double *C, const double *C1, const double *C2, double *err) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    // dd::sub(C, 0, C1, C2) then dd::div(., C1, C2) (eval.hpp:65-110, 317-338)
    double d1, d2;
    {
        const double a1 = C[i], b1 = C1[i], b2 = C2[i];
        d1 = a1 - b1;
        const double s = d1 - a1, t = b1 + s, u = d1 - s;
        d2 = (a1 - u) - t;
        d2 -= b2;
        fast_two_sum(d1, d2, d1, d2);
    }
    const double b1 = C1[i], b2 = C2[i];
    double q1 = d1 / b1;
    const double s = q1 * b1, t = __builtin_fma(q1, b1, -s);
    double u = d1 - s;
    u -= t;
    u += d2;
    u = __builtin_fma(-q1, b2, u);
    u /= b1;
    double q2;
    fast_two_sum(q1, u, q1, q2);
    err[i] = fabs(q1);
}

// The product kernel's data-bound ceiling: v_mfma_i32_32x32x32_i8 alone, 8 A and 8 B fragments of
// uniformly random bytes (the residue distribution) held in registers and cycled through so the
// operands change every instruction, two waves per SIMD, no memory traffic in the loop
// (tools/probes/mfma_power.hip).  The clock the chip holds on it bounds what any int8 GEMM on
// such operands can reach.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(256) void mfma_ceiling_kernel(int iters, int *out) {
    unsigned x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + 12345u;
    v4i A[8], B[8];
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            x = x * 1664525u + 1013904223u;
            A[f][q] = (int)x;
            x = x * 1664525u + 1013904223u;
            B[f][q] = (int)x;
        }
    v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[0], B[j], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[1], B[(j + 1) & 7], c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[2], B[(j + 2) & 7], c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[3], B[(j + 3) & 7], c3, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[4], B[(j + 4) & 7], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[5], B[(j + 5) & 7], c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[6], B[(j + 6) & 7], c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[7], B[(j + 7) & 7], c3, 0, 0, 0);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
// the same with v_mfma_i32_16x16x64_i8 (the product kernel's instruction), 8 accumulators
__global__ __launch_bounds__(256) void mfma16_ceiling_kernel(int iters, int *out) {
    unsigned x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + 12345u;
    v4i A[8], B[8];
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            x = x * 1664525u + 1013904223u;
            A[f][q] = (int)x;
            x = x * 1664525u + 1013904223u;
            B[f][q] = (int)x;
        }
    v4i c[8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int f = 0; f < 8; ++f) c[f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[f], B[(j + f) & 7], c[f], 0, 0, 0);
    }
    int s = 0;
#pragma unroll
    for (int f = 0; f < 8; ++f) s += c[f][f & 3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

}  // namespace oz2h

extern "C" {

// int8 ops per second (TOPS) over the whole chip of the better of the two MFMA forms alone on random
// operand bytes (32x32x32 and 16x16x64, the same ops per run); < 0 on failure
double gemmul8_mfma_ceiling(void *stream, int iters) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
        return -1.0;
    const int blocks = 2 * cus;  // 8 waves per CU = 2 per SIMD
    int *out = nullptr;
    if (hipMalloc(&out, (size_t)blocks * 256 * sizeof(int)) != hipSuccess) return -1.0;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double ops = 2.0 * 32 * 32 * 32 * 64.0 * iters * (double)blocks * 4;
    double best = -1.0;
    for (int form = 0; form < 2; ++form) {
        auto launch = [&](int it) {
            if (form == 0) oz2h::mfma_ceiling_kernel<<<blocks, 256, 0, st>>>(it, out);
            else oz2h::mfma16_ceiling_kernel<<<blocks, 256, 0, st>>>(2 * it, out);  // half the ops per MFMA
        };
        launch(iters / 4 + 1);  // warm-up
        (void)hipEventRecord(e0, st);
        launch(iters);
        (void)hipEventRecord(e1, st);
        float ms = 0.f;
        if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0.f) {
            const double tops = ops / (ms * 1e-3) / 1e12;
            if (tops > best) best = tops;
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
    return best;
}

int gemmul8_randmat(void *stream, int dtype, size_t m, size_t n, void *A, double phi, unsigned long long seed) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t total = m * n;
    if (total == 0) return GEMMUL8_OK;
    const unsigned grid = (unsigned)((total + 255) / 256);
    switch (dtype) {
    case GEMMUL8_R_64F: oz2h::randmat_kernel<double><<<grid, 256, 0, st>>>(total, (double *)A, phi, seed); break;
    case GEMMUL8_R_32F: oz2h::randmat_kernel<float><<<grid, 256, 0, st>>>(total, (float *)A, phi, seed); break;
    case GEMMUL8_C_64F: oz2h::randmat_c_kernel<double><<<grid, 256, 0, st>>>(total, (double *)A, phi, seed); break;
    case GEMMUL8_C_32F: oz2h::randmat_c_kernel<float><<<grid, 256, 0, st>>>(total, (float *)A, phi, seed); break;
    default: return GEMMUL8_E_TYPES;
    }
    return hipGetLastError() == hipSuccess ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_dd_gemm(void *stream, size_t m, size_t n, size_t k, const double *A, const double *B, double *C1,
                    double *C2) {
    dim3 grid((unsigned)((m + 63) / 64), (unsigned)((n + 63) / 64));
    oz2h::dd_gemm_kernel<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(m, n, k, A, B, C1, C2);
    return hipGetLastError() == hipSuccess ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_time_gemm(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                      int type_c, const void *alpha, const void *A, size_t lda, const void *B, size_t ldb,
                      const void *beta, void *C, size_t ldc, unsigned num_moduli, int fastmode, void *work,
                      int compute_type, int iters, double *sec, double *phase_ns) {
    if (iters <= 0 || !sec) return GEMMUL8_E_SIZE;
    // the total is timed on calls that record no phase events (what an application's call costs; the events and
    // their read-back add ~10 us per call at 1024^3); the phase times come from a second loop of the same length
    double ph[4] = {0, 0, 0, 0}, total = 0.0;
    for (int pass = 0; pass < (phase_ns ? 2 : 1); ++pass) {
        for (int it = 0; it < iters; ++it) {
            if (hipDeviceSynchronize() != hipSuccess) return GEMMUL8_E_HIP;
            double p[4] = {0, 0, 0, 0};
            const auto t0 = std::chrono::steady_clock::now();
            const int rc = gemmul8_gemm(stream, op_a, op_b, m, n, k, type_a, type_b, type_c, alpha, A, lda, B, ldb,
                                        beta, C, ldc, num_moduli, fastmode, work, compute_type, pass ? p : nullptr);
            if (hipDeviceSynchronize() != hipSuccess) return GEMMUL8_E_HIP;
            const auto t1 = std::chrono::steady_clock::now();
            if (rc != GEMMUL8_OK) return rc;
            if (pass == 0) total += std::chrono::duration<double>(t1 - t0).count();
            for (int i = 0; i < 4; ++i) ph[i] += p[i];
        }
    }
    *sec = total / iters;
    if (phase_ns)
        for (int i = 0; i < 4; ++i) phase_ns[i] = ph[i] / iters;
    return GEMMUL8_OK;
}

// the vendor routine of the drivers: hipblasGemmEx, op N / N, alpha = 1, beta = 0, column-major operands of one
// type (GEMMUL8_R_64F: DGEMM, R_32F: SGEMM, C_32F: CGEMM, C_64F: ZGEMM) with lda = m, ldb = k, ldc = m
int gemmul8_time_vendor_gemm(void *stream, int type, size_t m, size_t n, size_t k, const void *A, const void *B,
                             void *C, int iters, double *sec) {
    static std::mutex mu;
    static hipblasHandle_t handle = nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (iters <= 0 || !sec) return GEMMUL8_E_SIZE;
    if (!handle && hipblasCreate(&handle) != HIPBLAS_STATUS_SUCCESS) return GEMMUL8_E_HIP;
    if (hipblasSetStream(handle, static_cast<hipStream_t>(stream)) != HIPBLAS_STATUS_SUCCESS) return GEMMUL8_E_HIP;
    hipDataType dt;
    hipblasComputeType_t ct;
    switch (type) {
    case GEMMUL8_R_64F: dt = HIP_R_64F; ct = HIPBLAS_COMPUTE_64F; break;
    case GEMMUL8_R_32F: dt = HIP_R_32F; ct = HIPBLAS_COMPUTE_32F; break;
    case GEMMUL8_C_64F: dt = HIP_C_64F; ct = HIPBLAS_COMPUTE_64F; break;
    case GEMMUL8_C_32F: dt = HIP_C_32F; ct = HIPBLAS_COMPUTE_32F; break;
    default: return GEMMUL8_E_TYPES;
    }
    const double one_d[2] = {1.0, 0.0}, zero_d[2] = {0.0, 0.0};
    const float one_f[2] = {1.0f, 0.0f}, zero_f[2] = {0.0f, 0.0f};
    const bool dbl = type == GEMMUL8_R_64F || type == GEMMUL8_C_64F;
    const void *al = dbl ? (const void *)one_d : (const void *)one_f;
    const void *be = dbl ? (const void *)zero_d : (const void *)zero_f;
    auto call = [&] {
        return hipblasGemmEx(handle, HIPBLAS_OP_N, HIPBLAS_OP_N, (int)m, (int)n, (int)k, al, A, dt, (int)m, B, dt,
                             (int)k, be, C, dt, (int)m, ct, HIPBLAS_GEMM_DEFAULT);
    };
    if (call() != HIPBLAS_STATUS_SUCCESS) return GEMMUL8_E_HIP;  // (the drivers' accuracy call precedes the loop)
    double total = 0.0;
    for (int it = 0; it < iters; ++it) {
        if (hipDeviceSynchronize() != hipSuccess) return GEMMUL8_E_HIP;
        const auto t0 = std::chrono::steady_clock::now();
        const hipblasStatus_t rc = call();
        if (hipDeviceSynchronize() != hipSuccess) return GEMMUL8_E_HIP;
        const auto t1 = std::chrono::steady_clock::now();
        if (rc != HIPBLAS_STATUS_SUCCESS) return GEMMUL8_E_HIP;
        total += std::chrono::duration<double>(t1 - t0).count();
    }
    *sec = total / iters;
    return GEMMUL8_OK;
}

int gemmul8_relerr_dd(void *stream, size_t count, const double *C, const double *C1, const double *C2, double *err) {
    if (count == 0) return GEMMUL8_OK;
    oz2h::relerr_kernel<<<(unsigned)((count + 255) / 256), 256, 0, static_cast<hipStream_t>(stream)>>>(count, C, C1,
                                                                                                       C2, err);
    return hipGetLastError() == hipSuccess ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

}  // extern "C"
