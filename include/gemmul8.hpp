// gemmul8.hpp -- drop-in C++ API of the MI355X-native Ozaki-scheme-II GEMM emulator.
//
// Same declarations (names, parameter types, defaults, return type) as the
// reference's GEMMul8/include/gemmul8.hpp:7-287, so code compiled against the
// reference links against libgemmul8_amd.so unchanged (identical mangled names,
// checked by tests/test_abi.py).
//
//   size_t bytes = gemmul8::workSize(m, n, k, num_moduli);            // gemmul8.hpp:18-22
//   std::vector<double> t = gemmul8::gemm<double>(handle, HIPBLAS_OP_N, HIPBLAS_OP_N,
//        m, n, k, &alpha, dA, lda, dB, ldb, &beta, dC, ldc, num_moduli, fastmode, dwork);
//
// Semantics kept from the reference:
//   * column-major device operands, host alpha/beta, caller-owned workspace of
//     at least workSize(...) bytes (the library never allocates);
//   * returns the 4 phase times {scaling, int8 products, residue conversion,
//     inverse scaling} in nanoseconds; conversion is fused into the products on
//     MI355X, so entry 2 is 0;
//   * an unsupported computeType / type combination prints to stderr and
//     returns {0,0,0,0} without touching C.
// Differences (deliberate): all work is enqueued on the hipBLAS handle's stream
// (null stream when handle == nullptr) with no device-wide synchronisation; the
// call waits only for its own last event to fill the timers.  With the environment
// variable GEMMUL8_TIMERS=0 (read once per process) it does not wait at all and
// returns {0,0,0,0}: the call is then asynchronous on that stream, as the C ABI's
// gemmul8_gemm with phase_ns = NULL.  alpha/beta follow
// BLAS semantics for every value (the reference mis-applies some).
// num_moduli outside [2, 20] or k beyond the int32-exact bound is rejected.
#pragma once
#include <cstddef>
#include <vector>

#include <hip/hip_complex.h>
#include <hip/hip_runtime.h>
#include <hipblas/hipblas.h>

namespace gemmul8 {

typedef enum {
    REAL_DEFAULT,
    COMPLEX_BIG_MATRIX_ENCODE,
    COMPLEX_CLASSIC_MULT,
    COMPLEX_KARATSUBA_MULT
} computeType_t;

size_t workSize(const size_t m, const size_t n, const size_t k, const unsigned num_moduli,
                const computeType_t computeType = REAL_DEFAULT);

template <typename TA, typename TB = TA, typename TC = TA>
std::vector<double> gemm(hipblasHandle_t handle, const hipblasOperation_t op_A, const hipblasOperation_t op_B,
                         const size_t m, const size_t n, const size_t k, const TC *alpha, const TA *const A,
                         const size_t lda, const TB *const B, const size_t ldb, const TC *beta, TC *const C,
                         const size_t ldc, const unsigned num_moduli, const bool fastmode, void *const work,
                         const computeType_t computeType = REAL_DEFAULT);

#define GEMMUL8_DECLARE(TA_, TB_, TC_)                                                                            \
    template <>                                                                                                   \
    std::vector<double> gemm<TA_, TB_, TC_>(hipblasHandle_t, const hipblasOperation_t, const hipblasOperation_t,   \
                                            const size_t, const size_t, const size_t, const TC_ *, const TA_ *const, \
                                            const size_t, const TB_ *const, const size_t, const TC_ *, TC_ *const,   \
                                            const size_t, const unsigned, const bool, void *const,                 \
                                            const computeType_t);

GEMMUL8_DECLARE(double, double, double)
GEMMUL8_DECLARE(float, float, float)
GEMMUL8_DECLARE(double, float, double)
GEMMUL8_DECLARE(float, double, double)
GEMMUL8_DECLARE(double, float, float)
GEMMUL8_DECLARE(float, double, float)
GEMMUL8_DECLARE(hipFloatComplex, hipFloatComplex, hipFloatComplex)
GEMMUL8_DECLARE(hipDoubleComplex, hipDoubleComplex, hipDoubleComplex)
GEMMUL8_DECLARE(hipFloatComplex, hipDoubleComplex, hipDoubleComplex)
GEMMUL8_DECLARE(hipDoubleComplex, hipFloatComplex, hipDoubleComplex)
GEMMUL8_DECLARE(hipDoubleComplex, hipFloatComplex, hipFloatComplex)
GEMMUL8_DECLARE(hipFloatComplex, hipDoubleComplex, hipFloatComplex)
#undef GEMMUL8_DECLARE

}  // namespace gemmul8
