// Known-good comparison: hipBLAS int8 GEMM (what the reference calls per modulus,
// gemmul8.cu:265) on random int8 data at 8192^3, C32 = A^T B (OP_T, OP_N), K padded like the reference.
#include <hip/hip_runtime.h>
#include <hipblas/hipblas.h>
#include <cstdio>
#include <vector>
#include <cstdlib>
int main() {
    const int m = 8192, n = 8192, k = 8256;
    int8_t *A, *B; int32_t *C;
    (void)hipMalloc(&A, (size_t)m * k); (void)hipMalloc(&B, (size_t)n * k); (void)hipMalloc(&C, (size_t)m * n * 4);
    std::vector<int8_t> h((size_t)m * k);
    for (auto &x : h) x = (int8_t)(rand() % 255 - 127);
    (void)hipMemcpy(A, h.data(), h.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(B, h.data(), h.size(), hipMemcpyHostToDevice);
    hipblasHandle_t hd; hipblasCreate(&hd);
    int32_t one = 1, zero = 0;
    for (int rep = 0; rep < 5; ++rep) {
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        for (int i = 0; i < 4; ++i)
            hipblasGemmEx(hd, HIPBLAS_OP_T, HIPBLAS_OP_N, m, n, k, &one, A, HIP_R_8I, k, B, HIP_R_8I, k, &zero, C,
                          HIP_R_32I, m, HIPBLAS_COMPUTE_32I, HIPBLAS_GEMM_DEFAULT);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("hipblasGemmEx i8->i32 8192x8192x8256: %.3f ms per GEMM, %.0f TOPS\n", ms / 4, 2.0 * m * n * k * 4 / ms / 1e9);
    }
    return 0;
}
