// hijack.cpp -- LD_PRELOAD interception of hipBLAS / rocBLAS {D,Z,S,C}GEMM (plain, strided batched
// and the Ex forms), routed to the emulator (the caller side of the path).  An unmodified application --
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
//   GEMMUL8_INTERCEPT_THRESHOLD_M / _N / _K   emulate only when m, n, k are all >= (default 1280: the
//                                 measured square crossover on MI355X, below which rocBLAS DGEMM is as fast
//                                 or faster -- INTEGRATION.md section 3)
//   GEMMUL8_INFO=1                one line per call on stderr
// Calls with device-resident alpha/beta (pointer mode device), sizes below the thresholds or
// arguments the emulator rejects (nothing enqueued) go to the vendor routine unchanged.  The Ex forms
// (hipblasGemmEx, hipblasGemmStridedBatchedEx, rocblas_gemm_ex, rocblas_gemm_strided_batched_ex) are
// emulated when A, B and C share one of the four types and the compute type is that precision "at
// least" (HIPBLAS_COMPUTE_64F / _32F; rocBLAS: the same datatype); pedantic compute types, mixed types
// and rocBLAS calls whose output D is not C in place are forwarded (the reference's companion
// interposer hooks cublasGemmEx and cublasGemmStridedBatchedEx the same way, ozIMMU_EF/src/cublas.cu:135, 318).  A call
// whose kernels were enqueued and then failed to launch is never forwarded (the vendor routine
// would apply beta to a C the emulator may already have written): it returns an execution error.
//
// Workspaces: an eager call uses one buffer per (device, stream), grown on demand (calls on one
// stream are ordered, so reuse is safe; the lookup and the call's enqueue happen under one lock, so
// a call of another thread on the same stream cannot free the buffer between them).  A call captured into a graph never uses that buffer (a
// later, larger eager call would free it under the graph, and graphs captured on one stream would
// share it and race when replayed on different streams): each (device, capture, stream) gets a
// buffer of its own, allocated during the capture under relaxed capture mode and never freed,
// since the graph may be replayed at any time.
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

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
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
    decltype(&hipStreamGetCaptureInfo) captureInfo = nullptr;
    decltype(&hipThreadExchangeStreamCaptureMode) exchangeCaptureMode = nullptr;
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
        captureInfo = reinterpret_cast<decltype(captureInfo)>(sym(hip, "hipStreamGetCaptureInfo"));
        exchangeCaptureMode =
            reinterpret_cast<decltype(exchangeCaptureMode)>(sym(hip, "hipThreadExchangeStreamCaptureMode"));
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
    static constexpr long DEFAULT_THRESHOLD = 1280;
    long tm = DEFAULT_THRESHOLD, tn = DEFAULT_THRESHOLD, tk = DEFAULT_THRESHOLD;
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
        tm = num("GEMMUL8_INTERCEPT_THRESHOLD_M", DEFAULT_THRESHOLD);
        tn = num("GEMMUL8_INTERCEPT_THRESHOLD_N", DEFAULT_THRESHOLD);
        tk = num("GEMMUL8_INTERCEPT_THRESHOLD_K", DEFAULT_THRESHOLD);
        info = num("GEMMUL8_INFO", 0) != 0;
    }
};

const Config &cfg() {
    static Config c;
    return c;
}

std::atomic<void *> last_workspace{nullptr};  // test hook: gemmul8_hijack_last_workspace()

// held from the workspace lookup until the call using it is enqueued: growing a stream's eager
// buffer frees the old one (after a stream sync), which must not happen between another thread's
// lookup and its enqueue on the same stream
std::mutex ws_mu;

// workspace of one call (see the header comment); nullptr: none available, forward the call.
// The caller holds ws_mu.
void *workspace(size_t bytes, hipStream_t st) {
    static std::map<std::pair<int, hipStream_t>, std::pair<void *, size_t>> eager;
    // (device, capture id, stream) -> the capture's current buffer; every buffer ever handed to a
    // capture stays allocated (the graph's nodes hold its address)
    static std::map<std::tuple<int, unsigned long long, hipStream_t>, std::pair<void *, size_t>> captured;
    const Api &a = api();
    int dev = 0;
    (void)a.getDevice(&dev);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (a.captureInfo) {
        if (a.captureInfo(st, &cap, &id) != hipSuccess) return nullptr;
    } else if (a.isCapturing && a.isCapturing(st, &cap) != hipSuccess) {
        return nullptr;
    }
    if (cap != hipStreamCaptureStatusNone) {
        if (cap != hipStreamCaptureStatusActive || !a.captureInfo || !a.exchangeCaptureMode) return nullptr;
        auto &e = captured[{dev, id, st}];
        if (e.second >= bytes) return e.first;
        // an allocation is not a stream operation, but global capture mode forbids it as "unsafe":
        // relaxed mode for this thread around it (as PyTorch's caching allocator does)
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        (void)a.exchangeCaptureMode(&mode);
        void *p = nullptr;
        const bool ok = a.malloc_(&p, bytes) == hipSuccess;
        (void)a.exchangeCaptureMode(&mode);
        if (!ok) return nullptr;
        e = {p, bytes};  // a smaller earlier buffer of this capture stays allocated
        return p;
    }
    auto &e = eager[{dev, st}];
    if (e.second < bytes) {
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

enum class Outcome { emulated, forward, failed };

// emulated: done; forward: nothing was enqueued, the vendor routine takes the call; failed: the
// emulator's kernels were enqueued and a launch failed (never forwarded)
Outcome emulate(const char *fn, const Mode &md, hipStream_t st, int opa, int opb, long m, long n, long k, int type,
                const void *alpha, const void *A, long lda, const void *B, long ldb, const void *beta, void *C,
                long ldc) {
    const Config &c = cfg();
    if (!md.on || m < c.tm || n < c.tn || k < c.tk || !api().ok) return Outcome::forward;
    const bool cplx = type == GEMMUL8_C_64F || type == GEMMUL8_C_32F;
    const int ct = cplx ? c.ctype : GEMMUL8_REAL_DEFAULT;
    const size_t ws = api().workSize(m, n, k, md.N, ct);
    int rc;
    {
        std::lock_guard<std::mutex> g(ws_mu);
        void *work = ws ? workspace(ws, st) : nullptr;
        if (!work) return Outcome::forward;
        last_workspace.store(work);
        rc = api().gemm(st, op_code(opa), op_code(opb), m, n, k, type, type, type, alpha, A, lda, B, ldb, beta, C, ldc,
                        md.N, md.fast, work, ct, nullptr);
    }
    const Outcome o = rc == GEMMUL8_OK ? Outcome::emulated : (rc == GEMMUL8_E_HIP ? Outcome::failed : Outcome::forward);
    if (c.info)
        fprintf(stderr, "[gemmul8] %s m=%ld n=%ld k=%ld -> %s (num_moduli=%u, %s)\n", fn, m, n, k,
                o == Outcome::emulated ? "emulated" : (o == Outcome::failed ? "launch failed" : "forwarded"), md.N,
                md.fast ? "fast" : "accurate");
    return o;
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

// the emulator's type of an Ex call whose three matrices share a type the emulator covers and whose
// compute type asks for at least that precision; -1: forward
int ex_type(hipDataType a, hipDataType b, hipDataType c, hipblasComputeType_t ct) {
    if (a != b || a != c) return -1;
    if (ct == HIPBLAS_COMPUTE_64F) return a == HIP_R_64F ? GEMMUL8_R_64F : (a == HIP_C_64F ? GEMMUL8_C_64F : -1);
    if (ct == HIPBLAS_COMPUTE_32F) return a == HIP_R_32F ? GEMMUL8_R_32F : (a == HIP_C_32F ? GEMMUL8_C_32F : -1);
    return -1;
}
int ex_type(rocblas_datatype a, rocblas_datatype b, rocblas_datatype c, rocblas_datatype d, rocblas_datatype ct) {
    if (a != b || a != c || a != d || a != ct) return -1;
    switch (a) {
    case rocblas_datatype_f64_r: return GEMMUL8_R_64F;
    case rocblas_datatype_f64_c: return GEMMUL8_C_64F;
    case rocblas_datatype_f32_r: return GEMMUL8_R_32F;
    case rocblas_datatype_f32_c: return GEMMUL8_C_32F;
    default: return -1;
    }
}
const Mode &mode_of(int type) { return type == GEMMUL8_R_64F || type == GEMMUL8_C_64F ? cfg().d : cfg().s; }
size_t elem_bytes(int type) {
    return type == GEMMUL8_C_64F ? 16 : (type == GEMMUL8_R_32F ? 4 : 8);
}
const char *cbyte(const void *p, long long elems, int type) {
    return static_cast<const char *>(p) + elems * (long long)elem_bytes(type);
}

}  // namespace

// ---------------------------------------------------------------- hipBLAS
#define OZ2_HIPBLAS_GEMM(NAME, T, TYPE, MODE)                                                                      \
    hipblasStatus_t NAME(hipblasHandle_t handle, hipblasOperation_t transA, hipblasOperation_t transB, int m,     \
                         int n, int k, const T *alpha, const T *A, int lda, const T *B, int ldb, const T *beta,  \
                         T *C, int ldc) {                                                                          \
        static auto real = next_symbol<decltype(&NAME)>(#NAME);                                                    \
        hipStream_t st = nullptr;                                                                                  \
        if (host_stream(handle, &st)) {                                                                            \
            const Outcome o = emulate(#NAME, cfg().MODE, st, (int)transA, (int)transB, m, n, k, TYPE, alpha, A,   \
                                      lda, B, ldb, beta, C, ldc);                                                  \
            if (o == Outcome::emulated) return HIPBLAS_STATUS_SUCCESS;                                             \
            if (o == Outcome::failed) return HIPBLAS_STATUS_EXECUTION_FAILED;                                      \
        }                                                                                                          \
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
            for (; b < batchCount; ++b) {                                                                          \
                const Outcome o = emulate(#NAME, cfg().MODE, st, (int)transA, (int)transB, m, n, k, TYPE, alpha,  \
                                          A + b * strideA, lda, B + b * strideB, ldb, beta, C + b * strideC, ldc); \
                if (o == Outcome::failed) return HIPBLAS_STATUS_EXECUTION_FAILED;                                  \
                if (o == Outcome::forward) break;                                                                  \
            }                                                                                                      \
        if (b == batchCount && batchCount > 0) return HIPBLAS_STATUS_SUCCESS;                                      \
        /* the batches not emulated (all of them, or those after a rejected one) go to the vendor routine */     \
        return real ? real(handle, transA, transB, m, n, k, alpha, A + b * strideA, lda, strideA, B + b * strideB, \
                           ldb, strideB, beta, C + b * strideC, ldc, strideC, batchCount - b)                      \
                    : HIPBLAS_STATUS_NOT_SUPPORTED;                                                                \
    }

extern "C" {
// the workspace the interposer handed to its latest emulated call (tests check that a captured
// call never shares the eager buffer of its stream)
void *gemmul8_hijack_last_workspace(void) { return last_workspace.load(); }

OZ2_HIPBLAS_GEMM(hipblasDgemm, double, GEMMUL8_R_64F, d)
OZ2_HIPBLAS_GEMM(hipblasZgemm, hipDoubleComplex, GEMMUL8_C_64F, d)
OZ2_HIPBLAS_GEMM(hipblasSgemm, float, GEMMUL8_R_32F, s)
OZ2_HIPBLAS_GEMM(hipblasCgemm, hipComplex, GEMMUL8_C_32F, s)
OZ2_HIPBLAS_GEMM_SB(hipblasDgemmStridedBatched, double, GEMMUL8_R_64F, d)
OZ2_HIPBLAS_GEMM_SB(hipblasZgemmStridedBatched, hipDoubleComplex, GEMMUL8_C_64F, d)
OZ2_HIPBLAS_GEMM_SB(hipblasSgemmStridedBatched, float, GEMMUL8_R_32F, s)
OZ2_HIPBLAS_GEMM_SB(hipblasCgemmStridedBatched, hipComplex, GEMMUL8_C_32F, s)

hipblasStatus_t hipblasGemmEx(hipblasHandle_t handle, hipblasOperation_t transA, hipblasOperation_t transB, int m, int n,
                              int k, const void *alpha, const void *A, hipDataType aType, int lda, const void *B,
                              hipDataType bType, int ldb, const void *beta, void *C, hipDataType cType, int ldc,
                              hipblasComputeType_t computeType, hipblasGemmAlgo_t algo) {
    static auto real = next_symbol<decltype(&hipblasGemmEx)>("hipblasGemmEx");
    const int t = ex_type(aType, bType, cType, computeType);
    hipStream_t st = nullptr;
    if (t >= 0 && host_stream(handle, &st)) {
        const Outcome o = emulate("hipblasGemmEx", mode_of(t), st, (int)transA, (int)transB, m, n, k, t, alpha, A, lda,
                                  B, ldb, beta, C, ldc);
        if (o == Outcome::emulated) return HIPBLAS_STATUS_SUCCESS;
        if (o == Outcome::failed) return HIPBLAS_STATUS_EXECUTION_FAILED;
    }
    return real ? real(handle, transA, transB, m, n, k, alpha, A, aType, lda, B, bType, ldb, beta, C, cType, ldc,
                       computeType, algo)
                : HIPBLAS_STATUS_NOT_SUPPORTED;
}

hipblasStatus_t hipblasGemmStridedBatchedEx(hipblasHandle_t handle, hipblasOperation_t transA,
                                            hipblasOperation_t transB, int m, int n, int k, const void *alpha,
                                            const void *A, hipDataType aType, int lda, hipblasStride strideA,
                                            const void *B, hipDataType bType, int ldb, hipblasStride strideB,
                                            const void *beta, void *C, hipDataType cType, int ldc,
                                            hipblasStride strideC, int batchCount, hipblasComputeType_t computeType,
                                            hipblasGemmAlgo_t algo) {
    static auto real = next_symbol<decltype(&hipblasGemmStridedBatchedEx)>("hipblasGemmStridedBatchedEx");
    const int t = ex_type(aType, bType, cType, computeType);
    hipStream_t st = nullptr;
    int b = 0;
    if (t >= 0 && batchCount > 0 && host_stream(handle, &st))
        for (; b < batchCount; ++b) {
            const Outcome o = emulate("hipblasGemmStridedBatchedEx", mode_of(t), st, (int)transA, (int)transB, m, n, k,
                                      t, alpha, cbyte(A, b * strideA, t), lda, cbyte(B, b * strideB, t), ldb, beta,
                                      const_cast<char *>(cbyte(C, b * strideC, t)), ldc);
            if (o == Outcome::failed) return HIPBLAS_STATUS_EXECUTION_FAILED;
            if (o == Outcome::forward) break;
        }
    if (b == batchCount && batchCount > 0) return HIPBLAS_STATUS_SUCCESS;
    if (!real) return HIPBLAS_STATUS_NOT_SUPPORTED;
    const int tt = t >= 0 ? t : GEMMUL8_R_64F;  // (b = 0 whenever the type is not one of the emulated four)
    return real(handle, transA, transB, m, n, k, alpha, cbyte(A, b * strideA, tt), aType, lda, strideA,
                cbyte(B, b * strideB, tt), bType, ldb, strideB, beta, const_cast<char *>(cbyte(C, b * strideC, tt)),
                cType, ldc, strideC, batchCount - b, computeType, algo);
}
}

// ---------------------------------------------------------------- rocBLAS
#define OZ2_ROCBLAS_GEMM(NAME, T, TYPE, MODE)                                                                      \
    rocblas_status NAME(rocblas_handle handle, rocblas_operation transA, rocblas_operation transB, rocblas_int m, \
                        rocblas_int n, rocblas_int k, const T *alpha, const T *A, rocblas_int lda, const T *B,   \
                        rocblas_int ldb, const T *beta, T *C, rocblas_int ldc) {                                  \
        static auto real = next_symbol<decltype(&NAME)>(#NAME);                                                    \
        hipStream_t st = nullptr;                                                                                  \
        if (host_stream(handle, &st)) {                                                                            \
            const Outcome o = emulate(#NAME, cfg().MODE, st, (int)transA, (int)transB, m, n, k, TYPE, alpha, A,   \
                                      lda, B, ldb, beta, C, ldc);                                                  \
            if (o == Outcome::emulated) return rocblas_status_success;                                             \
            if (o == Outcome::failed) return rocblas_status_internal_error;                                        \
        }                                                                                                          \
        return real ? real(handle, transA, transB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc)                  \
                    : rocblas_status_not_implemented;                                                              \
    }

#define OZ2_ROCBLAS_GEMM_SB(NAME, T, TYPE, MODE)                                                                   \
    rocblas_status NAME(rocblas_handle handle, rocblas_operation transA, rocblas_operation transB, rocblas_int m, \
                        rocblas_int n, rocblas_int k, const T *alpha, const T *A, rocblas_int lda,               \
                        rocblas_stride strideA, const T *B, rocblas_int ldb, rocblas_stride strideB,             \
                        const T *beta, T *C, rocblas_int ldc, rocblas_stride strideC, rocblas_int batchCount) {  \
        static auto real = next_symbol<decltype(&NAME)>(#NAME);                                                    \
        hipStream_t st = nullptr;                                                                                  \
        int b = 0;                                                                                                 \
        if (batchCount > 0 && host_stream(handle, &st))                                                           \
            for (; b < batchCount; ++b) {                                                                          \
                const Outcome o = emulate(#NAME, cfg().MODE, st, (int)transA, (int)transB, m, n, k, TYPE, alpha,  \
                                          A + b * strideA, lda, B + b * strideB, ldb, beta, C + b * strideC, ldc); \
                if (o == Outcome::failed) return rocblas_status_internal_error;                                    \
                if (o == Outcome::forward) break;                                                                  \
            }                                                                                                      \
        if (b == batchCount && batchCount > 0) return rocblas_status_success;                                      \
        return real ? real(handle, transA, transB, m, n, k, alpha, A + b * strideA, lda, strideA, B + b * strideB, \
                           ldb, strideB, beta, C + b * strideC, ldc, strideC, batchCount - b)                      \
                    : rocblas_status_not_implemented;                                                              \
    }

#undef rocblas_gemm_ex
#undef rocblas_gemm_strided_batched_ex

extern "C" {
OZ2_ROCBLAS_GEMM(rocblas_dgemm, double, GEMMUL8_R_64F, d)
OZ2_ROCBLAS_GEMM(rocblas_zgemm, rocblas_double_complex, GEMMUL8_C_64F, d)
OZ2_ROCBLAS_GEMM(rocblas_sgemm, float, GEMMUL8_R_32F, s)
OZ2_ROCBLAS_GEMM(rocblas_cgemm, rocblas_float_complex, GEMMUL8_C_32F, s)
OZ2_ROCBLAS_GEMM_SB(rocblas_dgemm_strided_batched, double, GEMMUL8_R_64F, d)
OZ2_ROCBLAS_GEMM_SB(rocblas_zgemm_strided_batched, rocblas_double_complex, GEMMUL8_C_64F, d)
OZ2_ROCBLAS_GEMM_SB(rocblas_sgemm_strided_batched, float, GEMMUL8_R_32F, s)
OZ2_ROCBLAS_GEMM_SB(rocblas_cgemm_strided_batched, rocblas_float_complex, GEMMUL8_C_32F, s)

// D = alpha op(A) op(B) + beta C: emulated in place (d == c, ldd == ldc) only
rocblas_status rocblas_gemm_ex(rocblas_handle handle, rocblas_operation transA, rocblas_operation transB, rocblas_int m,
                               rocblas_int n, rocblas_int k, const void *alpha, const void *a, rocblas_datatype a_type,
                               rocblas_int lda, const void *b, rocblas_datatype b_type, rocblas_int ldb,
                               const void *beta, const void *c, rocblas_datatype c_type, rocblas_int ldc, void *d,
                               rocblas_datatype d_type, rocblas_int ldd, rocblas_datatype compute_type,
                               rocblas_gemm_algo algo, int32_t solution_index, uint32_t flags) {
    static auto real = next_symbol<decltype(&rocblas_gemm_ex)>("rocblas_gemm_ex");
    const int t = ex_type(a_type, b_type, c_type, d_type, compute_type);
    hipStream_t st = nullptr;
    if (t >= 0 && c == d && ldc == ldd && host_stream(handle, &st)) {
        const Outcome o = emulate("rocblas_gemm_ex", mode_of(t), st, (int)transA, (int)transB, m, n, k, t, alpha, a,
                                  lda, b, ldb, beta, d, ldd);
        if (o == Outcome::emulated) return rocblas_status_success;
        if (o == Outcome::failed) return rocblas_status_internal_error;
    }
    return real ? real(handle, transA, transB, m, n, k, alpha, a, a_type, lda, b, b_type, ldb, beta, c, c_type, ldc, d,
                       d_type, ldd, compute_type, algo, solution_index, flags)
                : rocblas_status_not_implemented;
}

rocblas_status rocblas_gemm_strided_batched_ex(rocblas_handle handle, rocblas_operation transA, rocblas_operation transB,
                                               rocblas_int m, rocblas_int n, rocblas_int k, const void *alpha,
                                               const void *a, rocblas_datatype a_type, rocblas_int lda,
                                               rocblas_stride stride_a, const void *b, rocblas_datatype b_type,
                                               rocblas_int ldb, rocblas_stride stride_b, const void *beta,
                                               const void *c, rocblas_datatype c_type, rocblas_int ldc,
                                               rocblas_stride stride_c, void *d, rocblas_datatype d_type,
                                               rocblas_int ldd, rocblas_stride stride_d, rocblas_int batch_count,
                                               rocblas_datatype compute_type, rocblas_gemm_algo algo,
                                               int32_t solution_index, uint32_t flags) {
    static auto real = next_symbol<decltype(&rocblas_gemm_strided_batched_ex)>("rocblas_gemm_strided_batched_ex");
    const int t = ex_type(a_type, b_type, c_type, d_type, compute_type);
    hipStream_t st = nullptr;
    int bi = 0;
    if (t >= 0 && c == d && ldc == ldd && stride_c == stride_d && batch_count > 0 && host_stream(handle, &st))
        for (; bi < batch_count; ++bi) {
            const Outcome o = emulate("rocblas_gemm_strided_batched_ex", mode_of(t), st, (int)transA, (int)transB, m, n,
                                      k, t, alpha, cbyte(a, bi * stride_a, t), lda, cbyte(b, bi * stride_b, t), ldb,
                                      beta, const_cast<char *>(cbyte(d, bi * stride_d, t)), ldd);
            if (o == Outcome::failed) return rocblas_status_internal_error;
            if (o == Outcome::forward) break;
        }
    if (bi == batch_count && batch_count > 0) return rocblas_status_success;
    if (!real) return rocblas_status_not_implemented;
    const int tt = t >= 0 ? t : GEMMUL8_R_64F;  // (bi = 0 whenever the type is not one of the emulated four)
    return real(handle, transA, transB, m, n, k, alpha, cbyte(a, bi * stride_a, tt), a_type, lda, stride_a,
                cbyte(b, bi * stride_b, tt), b_type, ldb, stride_b, beta, cbyte(c, bi * stride_c, tt), c_type, ldc,
                stride_c, const_cast<char *>(cbyte(d, bi * stride_d, tt)), d_type, ldd, stride_d, batch_count - bi,
                compute_type, algo, solution_index, flags);
}
}
