// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
// extern "C" shim around the REFERENCE's own gemmul8::gemm (compiled from
// /root/reference/GEMMul8/src/gemmul8.cu by oracle/ref/Makefile into oracle/_ref/),
// used on the GPU box to pin the CPU oracle with golden vectors.  Never linked
// into the product.
#include <cstdio>
#include <hip/hip_complex.h>
#include <hipblas/hipblas.h>

#include "gemmul8.hpp"  // the reference's header (-I/root/reference/GEMMul8/include)

static hipblasHandle_t handle() {
    static hipblasHandle_t h = nullptr;
    if (!h) hipblasCreate(&h);
    return h;
}

template <typename TA, typename TB, typename TC>
static int call(int opA, int opB, size_t m, size_t n, size_t k, const void *alpha, const void *A, size_t lda,
                const void *B, size_t ldb, const void *beta, void *C, size_t ldc, unsigned N, int fast, int ctype,
                void *work, double *times) {
    auto op = [](int o) { return o == 0 ? HIPBLAS_OP_N : (o == 1 ? HIPBLAS_OP_T : HIPBLAS_OP_C); };
    std::vector<double> t = gemmul8::gemm<TA, TB, TC>(handle(), op(opA), op(opB), m, n, k, (const TC *)alpha,
                                                      (const TA *)A, lda, (const TB *)B, ldb, (const TC *)beta,
                                                      (TC *)C, ldc, N, fast != 0, work,
                                                      (gemmul8::computeType_t)ctype);
    if (times)
        for (int i = 0; i < 4; ++i) times[i] = t[i];
    return hipDeviceSynchronize() == hipSuccess ? 0 : -6;
}

extern "C" {
// type codes as include/gemmul8_c.h: 0 f64, 1 f32, 2 c64, 3 c32
int ref_gemm(int ta, int tb, int tc, int opA, int opB, size_t m, size_t n, size_t k, const void *alpha,
             const void *A, size_t lda, const void *B, size_t ldb, const void *beta, void *C, size_t ldc,
             unsigned N, int fast, int ctype, void *work, double *times) {
    using cd = hipDoubleComplex;
    using cf = hipFloatComplex;
#define C_(a, b, c, TA, TB, TC)                                                                                   \
    if (ta == a && tb == b && tc == c)                                                                            \
        return call<TA, TB, TC>(opA, opB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, N, fast, ctype, work, times);
    C_(0, 0, 0, double, double, double)
    C_(1, 1, 1, float, float, float)
    C_(0, 1, 0, double, float, double)
    C_(1, 0, 0, float, double, double)
    C_(0, 1, 1, double, float, float)
    C_(1, 0, 1, float, double, float)
    C_(3, 3, 3, cf, cf, cf)
    C_(2, 2, 2, cd, cd, cd)
    C_(3, 2, 2, cf, cd, cd)
    C_(2, 3, 2, cd, cf, cd)
    C_(2, 3, 3, cd, cf, cf)
    C_(3, 2, 3, cf, cd, cf)
#undef C_
    return -2;
}

size_t ref_work_size(size_t m, size_t n, size_t k, unsigned N, int ctype) {
    return gemmul8::workSize(m, n, k, N, (gemmul8::computeType_t)ctype);
}
}
