// Cost of phase-timing events between dependent kernels on one stream: plain launches, hipEventRecord
// markers (timing / disable-timing events), and events attached to the kernel dispatches themselves
// (hipExtLaunchKernelGGL start/stop).  4 kernels of ~8 us per iteration, 300 iterations.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

__global__ void work(float *x, int iters) {
    float v = x[blockIdx.x * blockDim.x + threadIdx.x];
    for (int i = 0; i < iters; ++i) v = v * 1.0001f + 0.5f;
    x[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

int main() {
    float *x;
    hipMalloc(&x, 1024 * 256 * sizeof(float));
    hipMemset(x, 0, 1024 * 256 * sizeof(float));
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipEvent_t ev[8], evn[8];
    for (int i = 0; i < 8; ++i) {
        hipEventCreate(&ev[i]);
        hipEventCreateWithFlags(&evn[i], hipEventDisableTiming);
    }
    const int ITER = 300, WORK = 3000;
    for (int mode = 0; mode < 5; ++mode) {
        for (int pass = 0; pass < 2; ++pass) {
            hipDeviceSynchronize();
            auto t0 = std::chrono::steady_clock::now();
            for (int it = 0; it < ITER; ++it) {
                if (mode == 0) {
                    for (int k = 0; k < 4; ++k) work<<<1024, 256, 0, st>>>(x, WORK);
                } else if (mode == 1 || mode == 2) {
                    hipEvent_t *e = mode == 1 ? ev : evn;
                    hipEventRecord(e[0], st);
                    for (int k = 0; k < 4; ++k) {
                        work<<<1024, 256, 0, st>>>(x, WORK);
                        hipEventRecord(e[1 + k], st);
                    }
                } else if (mode == 3) {
                    // start event on the first kernel, stop events on every kernel
                    for (int k = 0; k < 4; ++k)
                        hipExtLaunchKernelGGL(work, dim3(1024), dim3(256), 0, st, k == 0 ? ev[0] : nullptr, ev[1 + k], 0, x, WORK);
                } else {
                    // mode 4: events on the first and the last kernel only
                    for (int k = 0; k < 4; ++k)
                        hipExtLaunchKernelGGL(work, dim3(1024), dim3(256), 0, st, k == 0 ? ev[0] : nullptr, k == 3 ? ev[4] : nullptr, 0, x, WORK);
                }
            }
            auto t1 = std::chrono::steady_clock::now();
            hipStreamSynchronize(st);
            auto t2 = std::chrono::steady_clock::now();
            if (pass == 1) {
                float ms = 0;
                if (mode == 1 || mode >= 3) hipEventElapsedTime(&ms, ev[0], ev[4]);
                printf("mode %d: %.2f us/iter (host issue %.2f us/iter), last iter events %.2f us\n", mode,
                       std::chrono::duration<double, std::micro>(t2 - t0).count() / ITER,
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / ITER, ms * 1000);
            }
        }
    }
    return 0;
}
