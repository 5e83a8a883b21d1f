// hijack.cpp -- LD_PRELOAD interception of hipBLAS / rocBLAS {D,Z,S,C}GEMM, routed to the
// emulator (the caller side of the path).  An unmodified application --
// PyTorch's torch.matmul on float64 tensors calls hipblasDgemm -- runs its DGEMMs as Ozaki-II
// int8 products:
//
//     LD_PRELOAD=.../gemmul8/libgemmul8_hijack.so GEMMUL8_COMPUTE_MODE=fp64_int8_14 app
//
// The pattern follows the reference repository's companion libraries (ozIMMU_EF/src/cublas.cu,
// cuMpSGEMM/src/cumpsgemm_cublas.cu): the intercepted symbol decides per call whether to emulate,
// otherwise forwards to the next definition (dlsym(RTLD_NEXT)).
//
// Environment:
//   GEMMUL8_COMPUTE_MODE          D and Z GEMM: "dgemm" (forward) or "fp64_int8_<N>[_accu]",
//                                 default fp64_int8_14 (fast mode)
//   GEMMUL8_COMPUTE_MODE_SGEMM    S and C GEMM: "sgemm" (forward, default) or "fp32_int8_<N>[_accu]"
//   GEMMUL8_COMPLEX_TYPE          big_matrix (default) | classic | karatsuba
//   GEMMUL8_INTERCEPT_THRESHOLD_M / _N / _K   emulate only when m, n, k are all >= (default 128)
//   GEMMUL8_INFO=1                one line per call on stderr
// Calls with device-resident alpha/beta (pointer mode device), sizes below the thresholds or
// arguments the emulator rejects go to the vendor routine unchanged.
//
// The interposer has no link-time dependency on the HIP runtime or the BLAS libraries: a
// preloaded object that pulled in its own libamdhip64 would put a second HIP runtime into a
// process whose framework bundles one (PyTorch's torch/lib).  Every runtime entry point is
// looked up in the process at the first intercepted call, and the emulator library
// (libgemmul8_amd.so, next to this file) is dlopen'ed then, so it binds to the runtime the
// application already loaded.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipblas/hipblas.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "../../include/gemmul8_c.h"

namespace {

// runtime entry points, resolved in the running process at first use
struct Api {
    bool ok = false;
    decltype(&hipGetDevice) getDevice = nullptr;
    hipError_t (*malloc_)(void **, size_t) = nullptr;
    decltype(&hipFree) free_ = nullptr;
    decltype(&hipStreamSynchronize) streamSync = nullptr;
    decltype(&hipStreamIsCapturing) isCapturing = nullptr;
    decltype(&hipblasGetStream) hbGetStream = nullptr;
    decltype(&hipblasGetPointerMode) hbGetPointerMode = nullptr;
    decltype(&rocblas_get_stream) rbGetStream = nullptr;
    decltype(&rocblas_get_pointer_mode) rbGetPointerMode = nullptr;
    decltype(&gemmul8_gemm) gemm = nullptr;
    decltype(&gemmul8_work_size) workSize = nullptr;
    void *hip = nullptr, *hipblas = nullptr, *rocblas = nullptr;  // the application's own copies
    Api() {
        // frameworks load their runtime privately (Python extensions: RTLD_LOCAL), so look the
        // libraries up by soname among the loaded objects instead of in the global scope
        auto loaded = [](std::initializer_list<const char *> names) -> void * {
            for (const char *n : names)
                if (void *h = dlopen(n, RTLD_NOLOAD | RTLD_LAZY)) return h;
            return nullptr;
        };
        hip = loaded({"libamdhip64.so.7", "libamdhip64.so"});
        hipblas = loaded({"libhipblas.so.3", "libhipblas.so"});
        rocblas = loaded({"librocblas.so.5", "librocblas.so"});
        auto sym = [](void *h, const char *n) { return h ? dlsym(h, n) : dlsym(RTLD_DEFAULT, n); };
        getDevice = reinterpret_cast<decltype(getDevice)>(sym(hip, "hipGetDevice"));
        malloc_ = reinterpret_cast<decltype(malloc_)>(sym(hip, "hipMalloc"));
        free_ = reinterpret_cast<decltype(free_)>(sym(hip, "hipFree"));
        streamSync = reinterpret_cast<decltype(streamSync)>(sym(hip, "hipStreamSynchronize"));
        isCapturing = reinterpret_cast<decltype(isCapturing)>(sym(hip, "hipStreamIsCapturing"));
        hbGetStream = reinterpret_cast<decltype(hbGetStream)>(sym(hipblas, "hipblasGetStream"));
        hbGetPointerMode = reinterpret_cast<decltype(hbGetPointerMode)>(sym(hipblas, "hipblasGetPointerMode"));
        rbGetStream = reinterpret_cast<decltype(rbGetStream)>(sym(rocblas, "rocblas_get_stream"));
        rbGetPointerMode = reinterpret_cast<decltype(rbGetPointerMode)>(sym(rocblas, "rocblas_get_pointer_mode"));
        // the emulator library lives next to this one
        Dl_info info{};
        if (dladdr(reinterpret_cast<void *>(&cfg_anchor), &info) && info.dli_fname) {
            std::string dir(info.dli_fname);
            dir = dir.substr(0, dir.find_last_of('/') + 1);
            if (void *h = dlopen((dir + "libgemmul8_amd.so").c_str(), RTLD_NOW | RTLD_LOCAL)) {
                gemm = reinterpret_cast<decltype(gemm)>(dlsym(h, "gemmul8_gemm"));
                workSize = reinterpret_cast<decltype(workSize)>(dlsym(h, "gemmul8_work_size"));
            }
        }
        ok = getDevice && malloc_ && free_ && streamSync && gemm && workSize;
        if (!ok) fprintf(stderr, "[gemmul8] interposer inactive: HIP runtime or libgemmul8_amd.so not found\n");
    }
    static void cfg_anchor() {}
};

const Api &api() {
    static Api a;
    return a;
}

struct Mode {
    bool on = false;
    unsigned N = 14;
    int fast = 1;
};

Mode parse_mode(const char *name, const char *prefix, bool default_on) {
    Mode md;
    md.on = default_on;
    const char *v = getenv(name);
    if (!v || !*v) return md;
    std::string s(v);
    const std::string pre(prefix);
    if (s.compare(0, pre.size(), pre) != 0) {
        md.on = false;  // "dgemm" / "sgemm" / anything else: forward
        return md;
    }
    std::string rest = s.substr(pre.size());
    const size_t us = rest.find('_');
    if (us != std::string::npos) {
        md.fast = rest.substr(us + 1) == "accu" ? 0 : 1;
        rest = rest.substr(0, us);
    }
    const long n = strtol(rest.c_str(), nullptr, 10);
    md.on = n >= 2 && n <= 20;
    md.N = (unsigned)n;
    return md;
}

struct Config {
    Mode d, s;
    int ctype = GEMMUL8_COMPLEX_BIG_MATRIX_ENCODE;
    long tm = 128, tn = 128, tk = 128;
    bool info = false;
    Config() {
        d = parse_mode("GEMMUL8_COMPUTE_MODE", "fp64_int8_", true);
        s = parse_mode("GEMMUL8_COMPUTE_MODE_SGEMM", "fp32_int8_", false);
        if (const char *c = getenv("GEMMUL8_COMPLEX_TYPE")) {
            if (!strcmp(c, "classic")) ctype = GEMMUL8_COMPLEX_CLASSIC_MULT;
            else if (!strcmp(c, "karatsuba")) ctype = GEMMUL8_COMPLEX_KARATSUBA_MULT;
        }
        auto num = [](const char *e, long dflt) {
            const char *v = getenv(e);
            return v && *v ? strtol(v, nullptr, 10) : dflt;
        };
        tm = num("GEMMUL8_INTERCEPT_THRESHOLD_M", 128);
        tn = num("GEMMUL8_INTERCEPT_THRESHOLD_N", 128);
        tk = num("GEMMUL8_INTERCEPT_THRESHOLD_K", 128);
        info = num("GEMMUL8_INFO", 0) != 0;
    }
};

const Config &cfg() {
    static Config c;
    return c;
}

// one workspace per (device, stream): calls on one stream are ordered, so reuse is safe
void *workspace(size_t bytes, hipStream_t st) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, std::pair<void *, size_t>> pool;
    const Api &a = api();
    int dev = 0;
    (void)a.getDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    auto &e = pool[{dev, st}];
    if (e.second < bytes) {
        // growing the workspace synchronises and allocates: not while the stream is captured into a
        // graph (the call is forwarded to the vendor routine instead)
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (a.isCapturing && (a.isCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone)) return nullptr;
        if (e.first) {
            (void)a.streamSync(st);
            (void)a.free_(e.first);
        }
        e.first = nullptr;
        e.second = 0;
        if (a.malloc_(&e.first, bytes) != hipSuccess) return nullptr;
        e.second = bytes;
    }
    return e.first;
}

int op_code(int op) { return op == 111 ? GEMMUL8_OP_N : (op == 112 ? GEMMUL8_OP_T : GEMMUL8_OP_C); }

// true when the call was emulated
bool emulate(const char *fn, const Mode &md, hipStream_t st, int opa, int opb, long m, long n, long k, int type,
             const void *alpha, const void *A, long lda, const void *B, long ldb, const void *beta, void *C, long ldc) {
    const Config &c = cfg();
    if (!md.on || m < c.tm || n < c.tn || k < c.tk || !api().ok) return false;
    const bool cplx = type == GEMMUL8_C_64F || type == GEMMUL8_C_32F;
    const int ct = cplx ? c.ctype : GEMMUL8_REAL_DEFAULT;
    const size_t ws = api().workSize(m, n, k, md.N, ct);
    void *work = ws ? workspace(ws, st) : nullptr;
    if (!work) return false;
    const int rc = api().gemm(st, op_code(opa), op_code(opb), m, n, k, type, type, type, alpha, A, lda, B, ldb, beta,
                                C, ldc, md.N, md.fast, work, ct, nullptr);
    if (c.info)
        fprintf(stderr, "[gemmul8] %s m=%ld n=%ld k=%ld -> %s (num_moduli=%u, %s)\n", fn, m, n, k,
                rc == GEMMUL8_OK ? "emulated" : "forwarded", md.N, md.fast ? "fast" : "accurate");
    return rc == GEMMUL8_OK;
}

// the vendor definition: in the application's hipBLAS / rocBLAS, else the next one in the global scope
template <typename F> F next_symbol(const char *name) {
    const Api &a = api();
    void *lib = name[0] == 'h' ? a.hipblas : a.rocblas;
    void *f = lib ? dlsym(lib, name) : nullptr;
    return reinterpret_cast<F>(f ? f : dlsym(RTLD_NEXT, name));
}

// the handle's stream, when its scalars are host pointers (the emulator's alpha/beta contract)
bool host_stream(hipblasHandle_t h, hipStream_t *st) {
    const Api &a = api();
    hipblasPointerMode_t pm = HIPBLAS_POINTER_MODE_DEVICE;
    return a.ok && a.hbGetPointerMode && a.hbGetStream && a.hbGetPointerMode(h, &pm) == HIPBLAS_STATUS_SUCCESS &&
           pm == HIPBLAS_POINTER_MODE_HOST && a.hbGetStream(h, st) == HIPBLAS_STATUS_SUCCESS;
}
bool host_stream(rocblas_handle h, hipStream_t *st) {
    const Api &a = api();
    rocblas_pointer_mode pm = rocblas_pointer_mode_device;
    return a.ok && a.rbGetPointerMode && a.rbGetStream && a.rbGetPointerMode(h, &pm) == rocblas_status_success &&
           pm == rocblas_pointer_mode_host && a.rbGetStream(h, st) == rocblas_status_success;
}

}  // namespace

// ---------------------------------------------------------------- hipBLAS
#define OZ2_HIPBLAS_GEMM(NAME, T, TYPE, MODE)                                                                      \
    hipblasStatus_t NAME(hipblasHandle_t handle, hipblasOperation_t transA, hipblasOperation_t transB, int m,     \
                         int n, int k, const T *alpha, const T *A, int lda, const T *B, int ldb, const T *beta,  \
                         T *C, int ldc) {                                                                          \
        static auto real = next_symbol<decltype(&NAME)>(#NAME);                                                    \
        hipStream_t st = nullptr;                                                                                  \
        if (host_stream(handle, &st) &&                                                                            \
            emulate(#NAME, cfg().MODE, st, (int)transA, (int)transB, m, n, k, TYPE, alpha, A, lda, B, ldb, beta,  \
                    C, ldc))                                                                                       \
            return HIPBLAS_STATUS_SUCCESS;                                                                         \
        return real ? real(handle, transA, transB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc)                  \
                    : HIPBLAS_STATUS_NOT_SUPPORTED;                                                                \
    }

#define OZ2_HIPBLAS_GEMM_SB(NAME, T, TYPE, MODE)                                                                   \
    hipblasStatus_t NAME(hipblasHandle_t handle, hipblasOperation_t transA, hipblasOperation_t transB, int m,     \
                         int n, int k, const T *alpha, const T *A, int lda, long long strideA, const T *B,       \
                         int ldb, long long strideB, const T *beta, T *C, int ldc, long long strideC,            \
                         int batchCount) {                                                                         \
        static auto real = next_symbol<decltype(&NAME)>(#NAME);                                                    \
        hipStream_t st = nullptr;                                                                                  \
        int b = 0;                                                                                                 \
        if (batchCount > 0 && host_stream(handle, &st))                                                           \
            for (; b < batchCount; ++b)                                                                            \
                if (!emulate(#NAME, cfg().MODE, st, (int)transA, (int)transB, m, n, k, TYPE, alpha,               \
                             A + b * strideA, lda, B + b * strideB, ldb, beta, C + b * strideC, ldc))             \
                    break;                                                                                         \
        if (b == batchCount && batchCount > 0) return HIPBLAS_STATUS_SUCCESS;                                      \
        /* the batches not emulated (all of them, or those after a rejected one) go to the vendor routine */     \
        return real ? real(handle, transA, transB, m, n, k, alpha, A + b * strideA, lda, strideA, B + b * strideB, \
                           ldb, strideB, beta, C + b * strideC, ldc, strideC, batchCount - b)                      \
                    : HIPBLAS_STATUS_NOT_SUPPORTED;                                                                \
    }

extern "C" {
OZ2_HIPBLAS_GEMM(hipblasDgemm, double, GEMMUL8_R_64F, d)
OZ2_HIPBLAS_GEMM(hipblasZgemm, hipDoubleComplex, GEMMUL8_C_64F, d)
OZ2_HIPBLAS_GEMM(hipblasSgemm, float, GEMMUL8_R_32F, s)
OZ2_HIPBLAS_GEMM(hipblasCgemm, hipComplex, GEMMUL8_C_32F, s)
OZ2_HIPBLAS_GEMM_SB(hipblasDgemmStridedBatched, double, GEMMUL8_R_64F, d)
OZ2_HIPBLAS_GEMM_SB(hipblasZgemmStridedBatched, hipDoubleComplex, GEMMUL8_C_64F, d)
}

// ---------------------------------------------------------------- rocBLAS
#define OZ2_ROCBLAS_GEMM(NAME, T, TYPE, MODE)                                                                      \
    rocblas_status NAME(rocblas_handle handle, rocblas_operation transA, rocblas_operation transB, rocblas_int m, \
                        rocblas_int n, rocblas_int k, const T *alpha, const T *A, rocblas_int lda, const T *B,   \
                        rocblas_int ldb, const T *beta, T *C, rocblas_int ldc) {                                  \
        static auto real = next_symbol<decltype(&NAME)>(#NAME);                                                    \
        hipStream_t st = nullptr;                                                                                  \
        if (host_stream(handle, &st) &&                                                                            \
            emulate(#NAME, cfg().MODE, st, (int)transA, (int)transB, m, n, k, TYPE, alpha, A, lda, B, ldb, beta,  \
                    C, ldc))                                                                                       \
            return rocblas_status_success;                                                                         \
        return real ? real(handle, transA, transB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc)                  \
                    : rocblas_status_not_implemented;                                                              \
    }

extern "C" {
OZ2_ROCBLAS_GEMM(rocblas_dgemm, double, GEMMUL8_R_64F, d)
OZ2_ROCBLAS_GEMM(rocblas_zgemm, rocblas_double_complex, GEMMUL8_C_64F, d)
OZ2_ROCBLAS_GEMM(rocblas_sgemm, float, GEMMUL8_R_32F, s)
OZ2_ROCBLAS_GEMM(rocblas_cgemm, rocblas_float_complex, GEMMUL8_C_32F, s)
}
