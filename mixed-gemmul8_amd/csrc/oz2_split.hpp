// oz2_split.hpp -- internal launcher interface of the gfx950 kernels.
#pragma once
#include <hip/hip_ext.h>

#include <atomic>
#include <tuple>

#include "oz2_common.hpp"

namespace oz2 {

// ---- kernel launches and the phase timers ----
// The phase times (gemm()'s returned ns, bench.py's product-kernel duration) need timestamps at the
// phase boundaries.  A hipEventRecord between dependent kernels enqueues a marker packet that costs
// ~3.5 us of stream time on MI355X (tools/probes/event_cost.hip: four kernels with five markers
// +17.5 us per iteration, the same events attached to the dispatches +4.7 us; a 1024^3 call
// 60.5 -> 80.4 us with the markers).  So run() arms the events of one phase for the call's stream
// and every library launch goes through launch(), which attaches them to the dispatches themselves
// (hipExtLaunchKernel): `start` to the phase's first launch on that stream, `stop` to each of its
// launches there (the last one's completion stands).
struct PhaseEvents {
    hipStream_t st;
    hipEvent_t start, stop;
    bool stop_taken;
};
inline thread_local PhaseEvents g_phase_ev{};
// a library launch on this thread failed since the entry point began (set from the launch's own return
// code, so an error the application left pending on the thread is neither reported nor consumed)
inline thread_local bool g_launch_failed = false;

// a stream-ordering call of the library (fork / join event, phase marker): a failure is this call's
inline void hip_ok(hipError_t rc) {
    if (rc != hipSuccess) {
        g_launch_failed = true;
        (void)hipGetLastError();
    }
}

template <typename... KArgs, typename... Args>
inline void launch(void (*kernel)(KArgs...), dim3 grid, dim3 block, hipStream_t st, Args... args) {
    std::tuple<KArgs...> kargs(static_cast<KArgs>(args)...);
    void *ptrs[sizeof...(KArgs) > 0 ? sizeof...(KArgs) : 1] = {};
    std::apply([&](auto &...x) {
        int i = 0;
        ((ptrs[i++] = const_cast<void *>(static_cast<const void *>(&x))), ...);
    }, kargs);
    PhaseEvents &e = g_phase_ev;
    hipError_t rc;
    if (e.st == st && (e.start || e.stop)) {
        rc = hipExtLaunchKernel(reinterpret_cast<const void *>(kernel), grid, block, ptrs, 0, st, e.start, e.stop, 0);
        e.start = nullptr;
        e.stop_taken = e.stop != nullptr;
    } else {
        rc = hipLaunchKernel(reinterpret_cast<const void *>(kernel), grid, block, ptrs, 0, st);
    }
    if (rc != hipSuccess) {
        g_launch_failed = true;
        (void)hipGetLastError();  // our own failure, reported through the return code instead
    }
}

// One operand as the kernels see it: vector v = row of op(A) or column of op(B),
// element e runs along k.  contig: element e of vector v is at ptr[v*ld + e]
// (B op N, A op T); otherwise at ptr[e*ld + v] (A op N, B op T).
struct OperandDesc {
    const void *ptr;
    size_t ld;     // leading dimension in elements (complex: in complex elements)
    bool contig;
    bool dbl;      // real part is f64 (else f32)
    bool cplx;
    bool conj;     // op C of a complex operand
};

// ---- split.hip ----
// VT = threads_scaling of the reference entry point (128 or 512); accurate=true
// writes sft0 = 5 - ilogb(amax) instead of the fast-mode shift.
void split_stats(const OperandDesc &d, size_t len, size_t nvec, int VT, bool accurate, float log2M, int16_t *out,
                 hipStream_t st);
// mode 0: N residue planes from sft (reference convention -shift); mode 1: 6-bit magnitudes from sft0
// btail_quirk: accurate-mode big-matrix B magnitudes with the reference's tail defect (see split.hip)
void split_encode(const OperandDesc &d, bool is_A, size_t nvec, size_t len, const int16_t *sft, int8_t *out,
                  size_t plane, const Layout &L, int mode, const ModParams &MP, hipStream_t st,
                  bool btail_quirk = false);
// accurate mode, real operands: sft0 (as split_stats(accurate)) and the 6-bit magnitude plane (as split_encode
// MODE 1) from one read of the operand; scratch: (kblk / 64) * round_up(vpad, 64) int2 of per-tile exponents
// (false: not applicable -- complex, or scratch too small -- nothing launched)
bool split_magnitudes(const OperandDesc &d, bool is_A, size_t nvec, size_t len, int16_t *sft0, int8_t *out,
                      const Layout &L, void *scratch, size_t scratch_bytes, hipStream_t st);
// fast-mode shifts of A (real f64 rows, strided) and B (real f64 columns, contiguous) in one launch
// (false: not applicable, nothing launched)
bool split_stats_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len, int VT,
                      float log2M, int16_t *sftA, int16_t *sftB, hipStream_t st);
// mode 0 slices of both operands (one element type) in a single launch (false: not applicable,
// nothing launched)
// accurate mode, one stream, real operands of one element type: sft0 and the magnitude planes of both operands in
// two launches (tile pass; fix-up with the vector exponents found in-block), zeroing the bound maxima
// [0, nbound) on the way; false (nothing launched) where the forms or the scratch do not allow it
bool split_magnitudes_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len,
                           int16_t *sft0A, int16_t *sft0B, int8_t *outA, int8_t *outB, const Layout &L,
                           void *scratchA, size_t bytesA, void *scratchB, size_t bytesB, int32_t *bound,
                           size_t nbound, hipStream_t st);
// both operands' accurate-mode shifts in one launch
void split_finalize_accurate_pair(const int16_t *sft0A, const int32_t *boundA, size_t m, const int16_t *sft0B,
                                  const int32_t *boundB, size_t n, float log2M, int16_t *outA, int16_t *outB,
                                  hipStream_t st);
// fast mode, one stream, real f64, VT = 128, k <= 2048: both operands' shifts and slices of the moduli in MP in one
// launch reading each operand once (split_fused_kernel); false (nothing launched) where it does not apply
// (GEMMUL8_FUSED_SPLIT=0: never)
bool split_fused_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len, int VT,
                      float log2M, int16_t *sftA, int16_t *sftB, int8_t *outA, int8_t *outB, const Layout &L,
                      const ModParams &MP, hipStream_t st);
// accurate mode, one stream, real f64, k <= 2048: sft0 and the magnitude plane of both operands in one launch
// that reads each operand once (split_fused_kernel, MAG), zeroing the bound maxima [0, nbound); false (nothing
// launched) where it does not apply (GEMMUL8_FUSED_SPLIT=0: never)
bool split_fused_magnitudes_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len,
                                 int16_t *sft0A, int16_t *sft0B, int8_t *outA, int8_t *outB, const Layout &L,
                                 const ModParams &MP, int32_t *bound, size_t nbound, hipStream_t st);
// accurate mode (real operands): the encode computes the final shifts itself from sft0 and the bound maxima and
// stores them to sftA / sftB (finalize_accurate_sft_kernel's arithmetic, one launch fewer)
struct AccurateShifts {
    const int16_t *sft0A, *sft0B;
    const int32_t *boundA, *boundB;
    float log2M;
};
bool split_encode_pair(const OperandDesc &dA, size_t m, const OperandDesc &dB, size_t n, size_t len,
                       const int16_t *sftA, const int16_t *sftB, int8_t *outA, int8_t *outB, const Layout &L,
                       const ModParams &MP, hipStream_t st, const AccurateShifts *accs = nullptr);
// cplx_rows: complex A bound of row v = max(bound[v], bound[v + nvec]) (scaling.hpp:2561-2588)
void split_finalize_accurate(const int16_t *sft0, const int32_t *bound, size_t nvec, float log2M, int16_t *out,
                             hipStream_t st, bool cplx_rows = false);
// p[0, n) = 0 on the stream (graph-capturable)
void zero_i32(int32_t *p, size_t n, hipStream_t st);

// ---- gemm_i8.hip ----
enum class Epi : int { RESIDUE = 0, BOUND = 1, RAW = 2 };
// Products of the N slice planes: residue planes (uint8, [N][n_pad][m_pad]),
// bound (rowmax[m_pad], colmax[n_pad] of |C|, must be zeroed), or raw int32 (plane 0 only).
// queue: the workspace's tile-queue area (Layout::offQueue) for the persistent residue kernel
// (nullptr: one-tile kernel only); queue_zeroed: an earlier launch on st zeroed it (else a zeroing
// launch precedes the persistent kernel).
// tail_small: this launch is the 128 x 128 tail of a residue launch (gemm_i8 splits it off itself)
void gemm_i8(const int8_t *A8, const int8_t *B8, const Layout &L, unsigned nplanes, Epi epi, void *out,
             int32_t *rowmax, int32_t *colmax, const ModParams &MP, hipStream_t st, uint32_t *queue = nullptr,
             bool queue_zeroed = false, bool tail_small = false);
// the residue-product kernel of the last RESIDUE launch: 0 none yet, 1 one-tile (gemm_i8_kernel),
// 2 persistent (gemm_i8_persistent_kernel), 3 k-chunked one-tile launches, 4 128 x 128 (gemm_i8_small_kernel),
// 5 persistent per-group (gemm_i8_persistent_pg_kernel); g_last_tail_small: its last planes ran as 128 x 128 tiles
extern std::atomic<int> g_last_residue_kernel;
extern std::atomic<int> g_last_tail_small;
// exhaustive exactness check of the residue epilogues (0 = biased, 1 = signed): mismatch count
unsigned long long residue_selftest(int path, hipStream_t st);

// ---- crt.hip ----
enum class OutType : int { F64 = 0, F32 = 1, C64 = 2, C32 = 3 };
// ref_epi: 1 = the reference's epilogue kernels including their non-BLAS variants (gemmul8_set_epilogue)
void crt_inverse(const uint8_t *R, const Layout &L, const int16_t *sftA, const int16_t *sftB, const CrtParams &CP,
                 OutType ot, const void *alpha, const void *beta, void *C, size_t ldc, hipStream_t st, int ref_epi);

// partial CRT sums of moduli [j0, j1) into S ([2][n][lds]: C1 then C2) and the CRT finished from summed
// partials (real outputs; gemmul8_crt_partial / gemmul8_crt_finish)
void crt_partial(const uint8_t *R, const Layout &L, unsigned N, bool numM1, unsigned j0, unsigned j1, double *S,
                 size_t lds, hipStream_t st);
void crt_finish(const double *S, size_t lds, const Layout &L, unsigned N, bool numM1, const int16_t *sftA,
                const int16_t *sftB, bool f32, const void *alpha, const void *beta, void *C, size_t ldc,
                hipStream_t st, int ref_epi);

}  // namespace oz2
