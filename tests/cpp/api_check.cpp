// C++ drop-in surface check (run by tests/test_gpu_cpp_api.py on the GPU box): code written against
// the reference's GEMMul8/include/gemmul8.hpp -- workSize + gemm<TA,TB,TC> with a hipBLAS handle --
// compiled against include/gemmul8.hpp and linked with libgemmul8_amd.so.  Each product must be
// bit-identical to the C ABI's (itself pinned against the oracle); an invalid compute type must return
// {0,0,0,0} and leave C untouched.  Prints "OK" on success.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gemmul8.hpp"
#include "gemmul8_c.h"

#define CHECK(x)                                                                  \
    do {                                                                          \
        if (!(x)) {                                                               \
            std::fprintf(stderr, "FAILED %s (line %d)\n", #x, __LINE__);          \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

template <typename T> static T *upload(const std::vector<T> &h) {
    T *d;
    CHECK(hipMalloc(&d, h.size() * sizeof(T)) == hipSuccess);
    CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess);
    return d;
}
template <typename T> static std::vector<T> download(const T *d, size_t n) {
    std::vector<T> h(n);
    CHECK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost) == hipSuccess);
    return h;
}
static double rnd(unsigned &s) {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) / 16777216.0 - 0.5) * (1.0 + (s & 7));
}

// GEMMUL8_TIMERS=0 (run with argv[1] == "async"): gemmul8::gemm returns {0,0,0,0} before its kernels finish;
// otherwise (the default contract) it returns after them.  Two back-to-back calls, bits against the C ABI.
static int check_async(hipblasHandle_t h, hipStream_t st, bool async) {
    const size_t s = 4096;  // ~1.5 ms of GPU work per call: the enqueue returns long before that
    const unsigned N = 14;
    unsigned seed = 11;
    std::vector<double> hA(s * s), hC(s * s, 0.0);
    for (auto &x : hA) x = rnd(seed);
    double *A = upload(hA), *C = upload(hC), *C3 = upload(hC), *Cr = upload(hC);
    void *work;
    CHECK(hipMalloc(&work, gemmul8::workSize(s, s, s, N)) == hipSuccess);
    const double one = 1.0, zero = 0.0;
    CHECK(hipDeviceSynchronize() == hipSuccess);
    std::vector<double> t1 = gemmul8::gemm<double>(h, HIPBLAS_OP_N, HIPBLAS_OP_N, s, s, s, &one, A, s, A, s, &zero, C, s,
                                                   N, true, work);
    std::vector<double> t2 = gemmul8::gemm<double>(h, HIPBLAS_OP_N, HIPBLAS_OP_T, s, s, s, &one, A, s, A, s, &zero, C3,
                                                   s, N, true, work);
    const hipError_t q = hipStreamQuery(st);  // right after the second call returned
    if (async) {
        CHECK(q == hipErrorNotReady);  // its kernels were still queued or running
        CHECK(t1 == std::vector<double>(4, 0.0) && t2 == std::vector<double>(4, 0.0));
    } else {
        // the synchronous contract: the phase times are read from the call's own completed events (the stream
        // itself may report its last completion signal a few microseconds after the event the call waited for)
        (void)q;
        CHECK(t1[1] > 0.0 && t2[1] > 0.0 && t1[3] > 0.0 && t2[3] > 0.0);
    }
    CHECK(hipStreamSynchronize(st) == hipSuccess);
    CHECK(gemmul8_gemm(st, GEMMUL8_OP_N, GEMMUL8_OP_N, s, s, s, GEMMUL8_R_64F, GEMMUL8_R_64F, GEMMUL8_R_64F, &one, A, s, A,
                       s, &zero, Cr, s, N, 1, work, GEMMUL8_REAL_DEFAULT, nullptr) == GEMMUL8_OK);
    CHECK(hipStreamSynchronize(st) == hipSuccess);
    CHECK(download(C, s * s) == download(Cr, s * s));
    CHECK(gemmul8_gemm(st, GEMMUL8_OP_N, GEMMUL8_OP_T, s, s, s, GEMMUL8_R_64F, GEMMUL8_R_64F, GEMMUL8_R_64F, &one, A, s, A,
                       s, &zero, Cr, s, N, 1, work, GEMMUL8_REAL_DEFAULT, nullptr) == GEMMUL8_OK);
    CHECK(hipStreamSynchronize(st) == hipSuccess);
    CHECK(download(C3, s * s) == download(Cr, s * s));
    CHECK(hipFree(A) == hipSuccess && hipFree(C) == hipSuccess && hipFree(C3) == hipSuccess && hipFree(Cr) == hipSuccess);
    CHECK(hipFree(work) == hipSuccess);
    std::printf("%s OK\n", async ? "async" : "sync");
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && (std::strcmp(argv[1], "async") == 0 || std::strcmp(argv[1], "sync") == 0)) {
        hipStream_t st;
        CHECK(hipStreamCreate(&st) == hipSuccess);
        hipblasHandle_t h;
        CHECK(hipblasCreate(&h) == HIPBLAS_STATUS_SUCCESS);
        CHECK(hipblasSetStream(h, st) == HIPBLAS_STATUS_SUCCESS);
        return check_async(h, st, std::strcmp(argv[1], "async") == 0);
    }
    const size_t m = 300, n = 260, k = 513;
    const unsigned N = 14;
    unsigned seed = 7;
    std::vector<double> hA(m * k), hB(k * n), hC(m * n, 0.0);
    for (auto &x : hA) x = rnd(seed);
    for (auto &x : hB) x = rnd(seed);
    std::vector<float> hBf(hB.begin(), hB.end());
    double *A = upload(hA), *B = upload(hB), *C = upload(hC), *C2 = upload(hC);
    float *Bf = upload(hBf);

    hipStream_t st;
    CHECK(hipStreamCreate(&st) == hipSuccess);
    hipblasHandle_t h;
    CHECK(hipblasCreate(&h) == HIPBLAS_STATUS_SUCCESS);
    CHECK(hipblasSetStream(h, st) == HIPBLAS_STATUS_SUCCESS);

    const size_t ws = gemmul8::workSize(m, n, k, N);
    CHECK(ws > 0 && ws == gemmul8_work_size(m, n, k, N, GEMMUL8_REAL_DEFAULT));
    void *work;
    CHECK(hipMalloc(&work, ws) == hipSuccess);
    const double one = 1.0, zero = 0.0;

    // DGEMM, both ops N, fast and accurate
    for (int fast = 1; fast >= 0; --fast) {
        std::vector<double> t = gemmul8::gemm<double>(h, HIPBLAS_OP_N, HIPBLAS_OP_N, m, n, k, &one, A, m, B, k, &zero, C,
                                                      m, N, fast != 0, work);
        CHECK(t.size() == 4 && t[1] > 0.0);
        CHECK(gemmul8_gemm(st, GEMMUL8_OP_N, GEMMUL8_OP_N, m, n, k, GEMMUL8_R_64F, GEMMUL8_R_64F, GEMMUL8_R_64F, &one, A,
                           m, B, k, &zero, C2, m, N, fast, work, GEMMUL8_REAL_DEFAULT, nullptr) == GEMMUL8_OK);
        CHECK(hipStreamSynchronize(st) == hipSuccess);
        CHECK(download(C, m * n) == download(C2, m * n));
    }
    // mixed double x float -> double (gemm<double, float, double>), op T on B
    {
        std::vector<double> t = gemmul8::gemm<double, float, double>(h, HIPBLAS_OP_N, HIPBLAS_OP_T, m, n, k, &one, A, m,
                                                                     Bf, n, &zero, C, m, 10, true, work);
        CHECK(t.size() == 4);
        CHECK(gemmul8_gemm(st, GEMMUL8_OP_N, GEMMUL8_OP_T, m, n, k, GEMMUL8_R_64F, GEMMUL8_R_32F, GEMMUL8_R_64F, &one, A,
                           m, Bf, n, &zero, C2, m, 10, 1, work, GEMMUL8_REAL_DEFAULT, nullptr) == GEMMUL8_OK);
        CHECK(hipStreamSynchronize(st) == hipSuccess);
        CHECK(download(C, m * n) == download(C2, m * n));
    }
    // complex double, big-matrix encode, op C x op N
    {
        const size_t mc = 90, nc = 70, kc = 110;
        std::vector<hipDoubleComplex> hZa(kc * mc), hZb(kc * nc), hZc(mc * nc);
        for (auto &z : hZa) z = make_hipDoubleComplex(rnd(seed), rnd(seed));
        for (auto &z : hZb) z = make_hipDoubleComplex(rnd(seed), rnd(seed));
        hipDoubleComplex *Za = upload(hZa), *Zb = upload(hZb), *Zc = upload(hZc), *Zc2 = upload(hZc);
        const size_t wz = gemmul8::workSize(mc, nc, kc, 12, gemmul8::COMPLEX_BIG_MATRIX_ENCODE);
        void *wkz;
        CHECK(hipMalloc(&wkz, wz) == hipSuccess);
        const hipDoubleComplex z1 = make_hipDoubleComplex(1.0, 0.0), z0 = make_hipDoubleComplex(0.0, 0.0);
        std::vector<double> t = gemmul8::gemm<hipDoubleComplex>(h, HIPBLAS_OP_C, HIPBLAS_OP_N, mc, nc, kc, &z1, Za, kc,
                                                                Zb, kc, &z0, Zc, mc, 12, true, wkz,
                                                                gemmul8::COMPLEX_BIG_MATRIX_ENCODE);
        CHECK(t.size() == 4 && t[1] > 0.0);
        CHECK(gemmul8_gemm(st, GEMMUL8_OP_C, GEMMUL8_OP_N, mc, nc, kc, GEMMUL8_C_64F, GEMMUL8_C_64F, GEMMUL8_C_64F, &z1,
                           Za, kc, Zb, kc, &z0, Zc2, mc, 12, 1, wkz, GEMMUL8_COMPLEX_BIG_MATRIX_ENCODE,
                           nullptr) == GEMMUL8_OK);
        CHECK(hipStreamSynchronize(st) == hipSuccess);
        std::vector<hipDoubleComplex> a = download(Zc, mc * nc), b = download(Zc2, mc * nc);
        CHECK(std::memcmp(a.data(), b.data(), a.size() * sizeof(hipDoubleComplex)) == 0);
        // a real compute type for complex operands: rejected like the reference (gemmul8.cu:142-145)
        CHECK(hipMemset(Zc, 0x3c, mc * nc * sizeof(hipDoubleComplex)) == hipSuccess);
        t = gemmul8::gemm<hipDoubleComplex>(h, HIPBLAS_OP_N, HIPBLAS_OP_N, mc, nc, kc, &z1, Za, mc, Zb, kc, &z0, Zc, mc,
                                            12, true, wkz, gemmul8::REAL_DEFAULT);
        CHECK(t == std::vector<double>(4, 0.0));
        CHECK(hipDeviceSynchronize() == hipSuccess);
        std::vector<unsigned char> raw(mc * nc * sizeof(hipDoubleComplex));
        CHECK(hipMemcpy(raw.data(), Zc, raw.size(), hipMemcpyDeviceToHost) == hipSuccess);
        for (unsigned char c : raw) CHECK(c == 0x3c);
    }
    // the C++ API inside a HIP graph capture on the handle's stream: zero phase times (no readback
    // inside the capture), and the instantiated graph reproduces the direct call's bits
    for (int fast = 1; fast >= 0; --fast) {
        CHECK(hipMemset(C, 0, m * n * sizeof(double)) == hipSuccess);
        CHECK(hipDeviceSynchronize() == hipSuccess);
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal) == hipSuccess);
        std::vector<double> t = gemmul8::gemm<double>(h, HIPBLAS_OP_N, HIPBLAS_OP_N, m, n, k, &one, A, m, B, k, &zero, C,
                                                      m, N, fast != 0, work);
        CHECK(hipStreamEndCapture(st, &g) == hipSuccess);
        CHECK(t == std::vector<double>(4, 0.0));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess);
        CHECK(hipGraphLaunch(ge, st) == hipSuccess);
        CHECK(gemmul8_gemm(st, GEMMUL8_OP_N, GEMMUL8_OP_N, m, n, k, GEMMUL8_R_64F, GEMMUL8_R_64F, GEMMUL8_R_64F, &one, A,
                           m, B, k, &zero, C2, m, N, fast, work, GEMMUL8_REAL_DEFAULT, nullptr) == GEMMUL8_OK);
        CHECK(hipStreamSynchronize(st) == hipSuccess);
        CHECK(download(C, m * n) == download(C2, m * n));
        CHECK(hipGraphExecDestroy(ge) == hipSuccess);
        CHECK(hipGraphDestroy(g) == hipSuccess);
    }
    std::printf("OK\n");
    return 0;
}
