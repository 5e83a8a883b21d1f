// gemmul8.hip -- orchestration, the drop-in C++ API (include/gemmul8.hpp) and the C ABI
// (include/gemmul8_c.h) of the MI355X Ozaki-scheme-II emulator.
//
// Per call, on the caller's stream and with no device-wide synchronisation:
//   fast mode      stats(A) -> encode(A)  ||  stats(B) -> encode(B)       split.hip
//   accurate mode  amax(A,B) -> 6-bit magnitudes -> bound product -> shifts -> encode
//   products       one launch, all moduli, fused mod-p epilogue         gemm_i8.hip
//   recombination  CRT + scaling + alpha/beta                           crt.hip
// The reference runs the same phases with 4N+4 hipDeviceSynchronize calls, a
// per-modulus hipblasGemmEx and a separate conversion kernel (gemmul8.cu:149-723).
// Operand B's split runs on a second stream ("lane") forked from and joined back into the
// caller's stream by events, so the two operands' split kernels overlap where either one alone
// leaves the chip idle (small or strided operands); the join precedes everything that reads
// both.  Events only: the call stays asynchronous and graph-capturable.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "../../include/gemmul8.hpp"
#include "../../include/gemmul8_c.h"
#include "oz2_split.hpp"

namespace oz2 {

struct Call {
    OperandDesc A, B;
    int ctype;
    unsigned slice_planes;  // 0: all N resident
    size_t m, n, k;
    unsigned N;
    bool fast;
    bool cplx;
    OutType ot;
    const void *alpha, *beta;
    void *C;
    size_t ldc;
    void *work;
    int VT;
    hipStream_t st;
    hipStream_t stB;  // operand B's split work: the lane's stream, or st without a lane
    struct Lane *lane;
};

// ---------------- operand-B lane: a second stream with fork / join events ----------------
struct Lane {
    hipStream_t s;
    hipEvent_t fork, join;
    int dev;
};
namespace lanes {
static std::mutex mu;
static std::vector<Lane *> free_list;
static bool disabled() {  // GEMMUL8_SINGLE_STREAM=1: everything on the caller's stream (A-B runs)
    static const bool d = [] {
        const char *e = getenv("GEMMUL8_SINGLE_STREAM");
        return e && atoi(e) != 0;
    }();
    return d;
}
static bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone;
}
static Lane *acquire(hipStream_t st) {
    if (disabled()) return nullptr;
    // a call captured into a graph runs on the caller's stream alone: a lane forked into the capture
    // would stay part of it until the origin stream ends the capture, long after this call returns
    // it to the pool, and an eager call of another thread taking it meanwhile would be recorded into
    // the foreign graph.  So capture is tested before the pool is looked at.
    if (capturing(st)) return nullptr;
    int dev = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess) return nullptr;
    {
        std::lock_guard<std::mutex> g(mu);
        for (size_t i = 0; i < free_list.size(); ++i)
            // a pooled lane still joined to somebody's capture is skipped (left in the pool)
            if (free_list[i]->dev == dev && !capturing(free_list[i]->s)) {
                Lane *l = free_list[i];
                free_list[i] = free_list.back();
                free_list.pop_back();
                return l;
            }
    }
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    Lane *l = new Lane{nullptr, nullptr, nullptr, dev};
    const bool ok = hipStreamCreateWithFlags(&l->s, hipStreamNonBlocking) == hipSuccess &&
                    hipEventCreateWithFlags(&l->fork, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&l->join, hipEventDisableTiming) == hipSuccess;
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) {  // no lane: the call runs on one stream
        (void)hipGetLastError();
        delete l;
        return nullptr;
    }
    return l;
}
static void release(Lane *l) {
    if (!l) return;
    std::lock_guard<std::mutex> g(mu);
    free_list.push_back(l);
}
}  // namespace lanes

// holds a lane for the enqueue of one call (released once the join is enqueued: a later call
// on the same lane queues behind this one's B work, which only orders, never races)
struct LaneGuard {
    Call &c;
    explicit LaneGuard(Call &call) : c(call) {
        // the fork / join costs ~10 us of stream latency: worth it from (m + n) k = 2^25 up
        // (4096^3: split 0.228 -> 0.206 ms; 1024^3: 39 -> 50 us with the lane, so none there)
        const bool big = (c.m + c.n) * c.k >= ((size_t)1 << 25);
        // real f64 A (op N) x B (op N) in fast mode runs both operands in each split launch instead (the
        // pair kernels, phase_split): at 8192^3 split 0.757 -> 0.735 ms, at 4096^3 the same.  Other forms
        // keep the two streams (their shift passes stay per operand).
        const bool pairs = c.fast && !c.A.cplx && !c.B.cplx && c.A.dbl && c.B.dbl && !c.A.contig && c.B.contig &&
                           c.VT == 128 && (c.slice_planes == 0 || c.slice_planes >= c.N);
        c.lane = big && !pairs ? lanes::acquire(c.st) : nullptr;
        c.stB = c.lane ? c.lane->s : c.st;
    }
    ~LaneGuard() {
        lanes::release(c.lane);
        c.lane = nullptr;
        c.stB = c.st;
    }
};
// a failed fork / join would leave the operand lanes unordered: it fails the call (GEMMUL8_E_HIP)
static void fork(const Call &c) {
    if (!c.lane) return;
    hip_ok(hipEventRecord(c.lane->fork, c.st));
    hip_ok(hipStreamWaitEvent(c.stB, c.lane->fork, 0));
}
static void join(const Call &c) {
    if (!c.lane) return;
    hip_ok(hipEventRecord(c.lane->join, c.stB));
    hip_ok(hipStreamWaitEvent(c.st, c.lane->join, 0));
}

// ---------------- phase timing (HIP events on the call's stream) ----------------

namespace timing {
static std::mutex mu;
static bool enabled = false;
struct Rec {
    // split start (its first launch), products start / end, CRT end; prod_only: gemmul8_products
    hipEvent_t start, prod0, prod1, crt1;
    bool prod_only;
};
static std::vector<Rec> pending;
static std::vector<Rec> pool;
static double acc_ms[4] = {0, 0, 0, 0};
static int calls = 0;

static Rec acquire() {
    Rec r{};
    if (!pool.empty()) {
        r = pool.back();
        pool.pop_back();
        r.prod_only = false;
        return r;
    }
    (void)hipEventCreate(&r.start);
    (void)hipEventCreate(&r.prod0);
    (void)hipEventCreate(&r.prod1);
    (void)hipEventCreate(&r.crt1);
    return r;
}
static float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}
// phase times of one call in ms: split, products, (conversion: fused), CRT
static void read(const Rec &r, float out[4]) {
    (void)hipEventSynchronize(r.prod_only ? r.prod1 : r.crt1);
    out[0] = r.prod_only ? 0.f : elapsed(r.start, r.prod0);
    out[1] = elapsed(r.prod0, r.prod1);
    out[2] = 0.f;
    out[3] = r.prod_only ? 0.f : elapsed(r.prod1, r.crt1);
}
static void resolve_all() {
    for (auto &r : pending) {
        float t[4];
        read(r, t);
        for (int i = 0; i < 4; ++i) acc_ms[i] += t[i];
        ++calls;
        pool.push_back(r);
    }
    pending.clear();
}

// arms the events of one phase for launch() on stream st; end() records, as markers, whichever of
// them no launch took (a phase with no kernel on that stream), so every event of a call is recorded
struct Phase {
    bool on;
    Phase(bool record, hipStream_t st, hipEvent_t start, hipEvent_t stop) : on(record) {
        if (on) g_phase_ev = PhaseEvents{st, start, stop, false};
    }
    void end() {
        if (!on) return;
        PhaseEvents &e = g_phase_ev;
        if (e.start) hip_ok(hipEventRecord(e.start, e.st));
        if (e.stop && !e.stop_taken) hip_ok(hipEventRecord(e.stop, e.st));
        g_phase_ev = PhaseEvents{};
        on = false;
    }
    ~Phase() { g_phase_ev = PhaseEvents{}; }  // failure paths: nothing left armed
};
}  // namespace timing

// Launch errors: every library launch checks its own return code (launch(), oz2_split.hpp); an entry
// point resets the thread's failure flag first and checks it after each phase, so GEMMUL8_E_HIP always
// means a launch of THIS call failed and no later phase was enqueued.  An error the application left
// pending on the thread (hipGetLastError) is neither reported as ours nor cleared.
static inline void clear_stale_error() { g_launch_failed = false; }
static inline bool launch_ok() { return !g_launch_failed; }
static bool is_capturing(hipStream_t st) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
}

// Workspace views of one call (layout: oz2_common.hpp make_layout)
struct Views {
    Layout L;
    int8_t *A8, *B8;
    uint8_t *R;
    int16_t *sftA, *sftB, *sft0;
    int32_t *bound;
    uint32_t *queue;
};
static Views views(void *work, size_t m, size_t n, size_t k, unsigned N, bool cplx, unsigned slice_planes = 0) {
    Views v;
    v.L = make_layout(m, n, k, N, cplx, slice_planes);
    int8_t *base = static_cast<int8_t *>(work);
    v.A8 = base + v.L.offA;
    v.B8 = base + v.L.offB;
    v.R = reinterpret_cast<uint8_t *>(base + v.L.offR);
    v.sftA = reinterpret_cast<int16_t *>(base + v.L.offSftA);
    v.sftB = reinterpret_cast<int16_t *>(base + v.L.offSftB);
    v.bound = reinterpret_cast<int32_t *>(base + v.L.offBound);
    v.sft0 = reinterpret_cast<int16_t *>(base + v.L.offSft0);
    v.queue = reinterpret_cast<uint32_t *>(base + v.L.offQueue);
    return v;
}

// tile-queue heads of a products launch whose first modulus is j0 (oz2_common.hpp make_layout)
static inline uint32_t *queue_of(const Views &v, unsigned j0) { return v.queue + QUEUE_HEADS * j0; }

// moduli [j0, j1) of an N-moduli call, renumbered from 0 (plane pointers are offset by the caller)
static ModParams sub_mod_params(unsigned N, unsigned j0, unsigned j1) {
    const ModParams full = make_mod_params(N);
    ModParams P{};
    for (unsigned i = 0; i < j1 - j0; ++i) {
        P.p[i] = full.p[j0 + i];
        P.barrett[i] = full.barrett[j0 + i];
        P.rinv_d[i] = full.rinv_d[j0 + i];
        P.rinv_f[i] = full.rinv_f[j0 + i];
    }
    P.N = j1 - j0;
    return P;
}

static bool one_read_magnitudes() {
    static const bool on = [] {
        const char *e = getenv("GEMMUL8_ONE_READ_MAGNITUDES");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// accurate mode, first half of phase 1: sft0 = 5 - ilogb(amax), the 6-bit magnitude planes and the
// bound product's row / column maxima (scaling.hpp:3053-3100).  A on the call's stream, B on the lane.
// Sharded form (gemmul8_shard_bound): sft0 already assembled in the workspace (sft0_ready) and the
// bound product restricted to the columns [c0, c1) of op(B) (c0 a multiple of TILE): the column maxima
// outside the range stay 0 and the row maxima cover those columns only, so a MAX all-reduce of the
// bound area over ranks holding complementary ranges gives the whole product's maxima.
static void phase_bound(const Call &c, const Views &v, size_t c0 = 0, size_t c1 = SIZE_MAX, bool sft0_ready = false) {
    // always the big-matrix geometry (Karatsuba layouts size their slice regions to hold it)
    const Layout L = v.L.kara ? make_layout(c.m, c.n, c.k, c.N, c.cplx, v.L.S, 0) : v.L;
    const ModParams MP = make_mod_params(c.N);
    fork(c);
    // real operands: sft0 and the magnitudes from one read of each operand (split_magnitudes), with the
    // per-tile exponents in slice plane 1, unused until the final encode (GEMMUL8_ONE_READ_MAGNITUDES=0: the
    // reference's two reads, for A/B runs)
    const size_t s1A = v.L.S >= 2 ? L.planeA : 0, s1B = v.L.S >= 2 ? L.planeB : 0;
    // one stream (small problems): both operands' magnitudes in two launches, the bound maxima zeroed by the second
    const bool pair = !c.lane && !sft0_ready && one_read_magnitudes() &&
                      (split_fused_magnitudes_pair(c.A, c.m, c.B, c.n, c.k, v.sft0, v.sft0 + L.m_pad, v.A8, v.B8, L,
                                                   MP, v.bound, L.m_pad + L.n_pad, c.st) ||
                       split_magnitudes_pair(c.A, c.m, c.B, c.n, c.k, v.sft0, v.sft0 + L.m_pad, v.A8, v.B8, L,
                                            v.A8 + L.planeA, s1A, v.B8 + L.planeB, s1B, v.bound, L.m_pad + L.n_pad,
                                            c.st));
    if (pair) {
    } else if (sft0_ready || !one_read_magnitudes() ||
        !split_magnitudes(c.A, true, c.m, c.k, v.sft0, v.A8, L, v.A8 + L.planeA, s1A, c.st)) {
        if (!sft0_ready) split_stats(c.A, c.k, c.m, c.VT, true, 0.f, v.sft0, c.st);
        split_encode(c.A, true, c.m, c.k, v.sft0, v.A8, L.planeA, L, 1, MP, c.st);
    }
    if (pair) {
    } else if (sft0_ready || !one_read_magnitudes() ||
        !split_magnitudes(c.B, false, c.n, c.k, v.sft0 + L.m_pad, v.B8, L, v.B8 + L.planeB, s1B, c.stB)) {
        if (!sft0_ready) split_stats(c.B, c.k, c.n, c.VT, true, 0.f, v.sft0 + L.m_pad, c.stB);
        // big-matrix B magnitudes carry the reference's tail defect; classic / Karatsuba do not
        // the B tail defect lives in the op-N big-matrix extraction only (scaling.hpp:2312-2323, 3201-3203)
        split_encode(c.B, false, c.n, c.k, v.sft0 + L.m_pad, v.B8, L.planeB, L, 1, MP, c.stB,
                     c.cplx && c.ctype == GEMMUL8_COMPLEX_BIG_MATRIX_ENCODE && c.B.contig);
    }
    join(c);
    if (!pair) zero_i32(v.bound, L.m_pad + L.n_pad, c.st);
    if (c1 > c.n) c1 = c.n;
    if (c0 == 0 && c1 == c.n) {
        gemm_i8(v.A8, v.B8, L, 1, Epi::BOUND, nullptr, v.bound, v.bound + L.m_pad, MP, c.st);
    } else if (c0 < c1) {
        const size_t t0 = c0 / TILE, t1 = (c1 + TILE - 1) / TILE;
        gemm_i8(v.A8, v.B8 + t0 * L.ksteps * PANEL, col_tiles(L, t0, t1), 1, Epi::BOUND, nullptr, v.bound,
                v.bound + L.m_pad + t0 * TILE, MP, c.st);
    }
}

// phase 1a: shifts of every row of op(A) (is_A) or column of op(B), shared by all moduli
// (scaling.hpp:3680-3734 fast, :3053-3136 accurate: from the bound maxima already in the workspace)
static void operand_shifts(const Call &c, const Views &v, bool is_A, hipStream_t st) {
    const Layout &L = v.L;
    if (c.fast) {
        const float log2M = oz2_log2M_fast[c.N - 2];
        if (is_A) split_stats(c.A, c.k, c.m, c.VT, false, log2M, v.sftA, st);
        else split_stats(c.B, c.k, c.n, c.VT, false, log2M, v.sftB, st);
    } else {
        const float log2M = oz2_log2M_accu[c.N - 2];
        if (is_A) split_finalize_accurate(v.sft0, v.bound, c.m, log2M, v.sftA, st, c.cplx);
        else split_finalize_accurate(v.sft0 + L.bm_pad, v.bound + L.bm_pad, c.n, log2M, v.sftB, st);
    }
}

// phase 1b: slices of moduli [j0, j1) of one operand into the slice planes starting at `slot`
static void operand_encode(const Call &c, const Views &v, bool is_A, unsigned j0, unsigned j1, unsigned slot,
                           hipStream_t st) {
    const Layout &L = v.L;
    ModParams SP = sub_mod_params(c.N, j0, j1);
    SP.zero_queue = is_A ? queue_of(v, j0) : nullptr;  // the products that follow find their tile queue zeroed
    if (is_A) split_encode(c.A, true, c.m, c.k, v.sftA, v.A8 + slot * L.planeA, L.planeA, L, 0, SP, st);
    else split_encode(c.B, false, c.n, c.k, v.sftB, v.B8 + slot * L.planeB, L.planeB, L, 0, SP, st);
}

// phase 1 (shifts + slices of moduli [j0, j1) into their own planes); bound_ready: accurate mode
// takes the row / column maxima already in the workspace (phase_bound, possibly combined across
// row blocks); shifts_ready: sftA / sftB are already in the workspace (assembled from the shards
// of gemmul8_shard_stats), only the slices are encoded
static void phase_split(const Call &c, const Views &v, unsigned j0, unsigned j1, bool bound_ready,
                        bool shifts_ready = false) {
    if (!c.fast && !bound_ready && !shifts_ready) phase_bound(c, v);
    if (!c.lane) {
        // one stream (small problems): fast mode, k <= 2048: shifts and slices in one launch; otherwise both
        // operands' shifts, then both operands' slices, one launch each where the operand forms allow it
        if (c.fast && !shifts_ready && j1 > j0) {
            const Layout &L = v.L;
            ModParams SP = sub_mod_params(c.N, j0, j1);
            SP.zero_queue = queue_of(v, j0);
            if (split_fused_pair(c.A, c.m, c.B, c.n, c.k, c.VT, oz2_log2M_fast[c.N - 2], v.sftA, v.sftB,
                                 v.A8 + j0 * L.planeA, v.B8 + j0 * L.planeB, L, SP, c.st))
                return;
        }
        if (!c.fast && !c.cplx && !shifts_ready && j1 > j0) {
            // accurate mode: the final shifts inside the pair encode
            const Layout &L = v.L;
            const size_t bm = L.bm_pad;
            ModParams SP = sub_mod_params(c.N, j0, j1);
            SP.zero_queue = queue_of(v, j0);
            const AccurateShifts accs{v.sft0, v.sft0 + bm, v.bound, v.bound + bm, oz2_log2M_accu[c.N - 2]};
            if (split_encode_pair(c.A, c.m, c.B, c.n, c.k, v.sftA, v.sftB, v.A8 + j0 * L.planeA, v.B8 + j0 * L.planeB,
                                  L, SP, c.st, &accs))
                return;
        }
        if (shifts_ready) {
        } else if (!c.fast && !c.cplx) {
            const size_t bm = v.L.bm_pad;
            split_finalize_accurate_pair(v.sft0, v.bound, c.m, v.sft0 + bm, v.bound + bm, c.n,
                                         oz2_log2M_accu[c.N - 2], v.sftA, v.sftB, c.st);
        } else if (!(c.fast && split_stats_pair(c.A, c.m, c.B, c.n, c.k, c.VT, oz2_log2M_fast[c.N - 2], v.sftA,
                                                v.sftB, c.st))) {
            operand_shifts(c, v, true, c.st);
            operand_shifts(c, v, false, c.st);
        }
        if (j1 == j0) return;  // shifts only (a shard that multiplies no modulus but recombines columns)
        const Layout &L = v.L;
        ModParams SP = sub_mod_params(c.N, j0, j1);
        SP.zero_queue = queue_of(v, j0);
        if (split_encode_pair(c.A, c.m, c.B, c.n, c.k, v.sftA, v.sftB, v.A8 + j0 * L.planeA, v.B8 + j0 * L.planeB, L,
                              SP, c.st))
            return;
        operand_encode(c, v, true, j0, j1, j0, c.st);
        operand_encode(c, v, false, j0, j1, j0, c.st);
        return;
    }
    fork(c);
    if (!shifts_ready) operand_shifts(c, v, true, c.st);
    if (j1 > j0) operand_encode(c, v, true, j0, j1, j0, c.st);
    if (!shifts_ready) operand_shifts(c, v, false, c.stB);
    if (j1 > j0) operand_encode(c, v, false, j0, j1, j0, c.stB);
    join(c);
}

// phase 2: residue planes j0..j1-1 from the slice planes starting at `slot` (one launch;
// conv_32i_2_8u fused into the epilogue).  queue_zeroed: the A encode just before on this stream
// zeroed the tile queue (phase_split, operand_encode); otherwise the products zero it themselves.
static void phase_products(const Views &v, unsigned N, unsigned j0, unsigned j1, unsigned slot, hipStream_t st,
                           bool queue_zeroed) {
    const Layout &L = v.L;
    gemm_i8(v.A8 + slot * L.planeA, v.B8 + slot * L.planeB, L, j1 - j0, Epi::RESIDUE, v.R + j0 * L.planeR, nullptr,
            nullptr, sub_mod_params(N, j0, j1), st, queue_of(v, j0), queue_zeroed);
}

// epilogue mode of the process (gemmul8_set_epilogue): 0 BLAS semantics (default), 1 the reference's
// epilogue kernels including their non-BLAS variants; GEMMUL8_EPILOGUE=reference sets 1 at load time
static std::atomic<int> g_epilogue_mode{[] {
    const char *e = getenv("GEMMUL8_EPILOGUE");
    return (e && (e[0] == 'r' || e[0] == '1')) ? 1 : 0;
}()};

// phase 3: CRT + scaling + BLAS epilogue over all N residue planes; columns [c0, c1) of the output only
// when given (C then points at column c0): the residue planes are column-major, so a column range is
// the same kernel over an offset plane base, sftB + c0 and n = c1 - c0
static void phase_crt(const Views &v, unsigned N, OutType ot, const void *alpha, const void *beta, void *C, size_t ldc,
                      hipStream_t st, size_t c0 = 0, size_t c1 = SIZE_MAX) {
    const CrtParams CP = make_crt_params(N, ot == OutType::F32 || ot == OutType::C32);
    const int ref_epi = g_epilogue_mode.load(std::memory_order_relaxed);
    if (c0 == 0 && c1 >= v.L.n) {
        crt_inverse(v.R, v.L, v.sftA, v.sftB, CP, ot, alpha, beta, C, ldc, st, ref_epi);
        return;
    }
    Layout L = v.L;
    L.n = c1 - c0;
    crt_inverse(v.R + c0 * L.ldr, L, v.sftA, v.sftB + c0, CP, ot, alpha, beta, C, ldc, st, ref_epi);
}

// phase 2 over the columns [c0, c1) of the residue planes only (c0 a multiple of TILE, c1 one too or n):
// the B slice tiles and the residue columns of that range, every row
static void phase_products_cols(const Views &v, unsigned N, unsigned j0, unsigned j1, size_t c0, size_t c1,
                                hipStream_t st) {
    const Layout &L = v.L;
    const size_t t0 = c0 / TILE, t1 = (c1 + TILE - 1) / TILE;
    gemm_i8(v.A8 + j0 * L.planeA, v.B8 + j0 * L.planeB + t0 * L.ksteps * PANEL, col_tiles(L, t0, t1), j1 - j0,
            Epi::RESIDUE, v.R + j0 * L.planeR + t0 * TILE * L.ldr, nullptr, nullptr, sub_mod_params(N, j0, j1), st,
            queue_of(v, j0), false);
}

// operand descriptor of the vectors [v0, ...) of d (rows of op(A) / columns of op(B))
static OperandDesc sub_operand(const OperandDesc &d, size_t v0) {
    OperandDesc s = d;
    const size_t es = (d.dbl ? 8 : 4) * (d.cplx ? 2 : 1);
    s.ptr = static_cast<const char *>(d.ptr) + (d.contig ? v0 * d.ld : v0) * es;
    return s;
}

static int run(Call &c, double *phase_ns) {
    const Views v = views(c.work, c.m, c.n, c.k, c.N, c.cplx, c.slice_planes);
    LaneGuard lane(c);

    // a call being captured into a graph records no timing events and returns zero phase times
    // (reading them back would synchronise inside the capture)
    const bool capturing = is_capturing(c.st);
    if (phase_ns && capturing)
        for (int i = 0; i < 4; ++i) phase_ns[i] = 0.0;
    const bool want_events = phase_ns != nullptr && !capturing;
    bool record;
    timing::Rec rec{};
    {
        std::lock_guard<std::mutex> g(timing::mu);
        record = want_events || (timing::enabled && !capturing);
        if (record) rec = timing::acquire();
    }

    // a failed launch ends the call before the next phase is enqueued (the events recorded so far
    // go back to the pool unread)
    auto fail = [&]() {
        if (record) {
            std::lock_guard<std::mutex> g(timing::mu);
            timing::pool.push_back(rec);
        }
        return GEMMUL8_E_HIP;
    };
    const unsigned S = v.L.S;
    if (S >= c.N) {
        timing::Phase split(record, c.st, rec.start, nullptr);
        phase_split(c, v, 0, c.N, false);
        split.end();
        if (!launch_ok()) return fail();
        timing::Phase prod(record, c.st, rec.prod0, rec.prod1);
        phase_products(v, c.N, 0, c.N, 0, c.st, true);
        prod.end();
        if (!launch_ok()) return fail();
    } else {
        // low-memory mode: the moduli in groups of S through the same S slice planes (each group
        // re-reads A and B); the product phase timer then includes the re-encoding
        timing::Phase split(record, c.st, rec.start, nullptr);
        if (!c.fast) phase_bound(c, v);
        fork(c);
        operand_shifts(c, v, true, c.st);
        operand_shifts(c, v, false, c.stB);
        join(c);
        split.end();
        if (!launch_ok()) return fail();
        timing::Phase prod(record, c.st, rec.prod0, rec.prod1);
        for (unsigned j0 = 0; j0 < c.N; j0 += S) {
            const unsigned j1 = j0 + S < c.N ? j0 + S : c.N;
            fork(c);
            operand_encode(c, v, true, j0, j1, 0, c.st);
            operand_encode(c, v, false, j0, j1, 0, c.stB);
            join(c);
            if (!launch_ok()) return fail();
            phase_products(v, c.N, j0, j1, 0, c.st, true);
            if (!launch_ok()) return fail();
        }
        prod.end();
    }

    {
        timing::Phase crt(record, c.st, nullptr, rec.crt1);
        phase_crt(v, c.N, c.ot, c.alpha, c.beta, c.C, c.ldc, c.st);
        crt.end();
    }
    if (!launch_ok()) return fail();

    if (want_events) {
        float t[4];
        timing::read(rec, t);
        for (int i = 0; i < 4; ++i) phase_ns[i] = t[i] * 1e6;
    }
    if (record) {
        std::lock_guard<std::mutex> g(timing::mu);
        if (timing::enabled) timing::pending.push_back(rec);
        else timing::pool.push_back(rec);
    }
    return GEMMUL8_OK;
}

// dtype helpers
static bool dt_dbl(int t) { return t == GEMMUL8_R_64F || t == GEMMUL8_C_64F; }
static bool dt_cplx(int t) { return t == GEMMUL8_C_64F || t == GEMMUL8_C_32F; }

static int prepare(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int ta, int tb, int tc,
                   const void *alpha, const void *A, size_t lda, const void *B, size_t ldb, const void *beta, void *C,
                   size_t ldc, unsigned N, int fast, void *work, int ctype, Call &c) {
    if (N < 2 || N > 20) return GEMMUL8_E_MODULI;
    if (ta < 0 || ta > 3 || tb < 0 || tb > 3 || tc < 0 || tc > 3) return GEMMUL8_E_TYPES;
    const bool cp = dt_cplx(ta);
    if (dt_cplx(tb) != cp || dt_cplx(tc) != cp) return GEMMUL8_E_TYPES;
    // the three complex compute types compute the same residues of Re(AB) and Im(AB): one engine
    // (big-matrix products) serves all of them; only the accurate-mode bound differs (see phase_bound)
    if (cp && !(ctype == GEMMUL8_COMPLEX_BIG_MATRIX_ENCODE || ctype == GEMMUL8_COMPLEX_CLASSIC_MULT ||
                ctype == GEMMUL8_COMPLEX_KARATSUBA_MULT))
        return GEMMUL8_E_TYPES;
    if (!cp && ctype != GEMMUL8_REAL_DEFAULT) return GEMMUL8_E_TYPES;
    // output precision is the higher of the inputs' in every reference specialization (gemmul8.hpp:49-287)
    if (!cp && !(tc == GEMMUL8_R_64F || tc == GEMMUL8_R_32F)) return GEMMUL8_E_TYPES;
    if (op_a < 0 || op_a > 2 || op_b < 0 || op_b > 2) return GEMMUL8_E_OP;
    const size_t kr = cp ? 2 * round_up(k, KSTEP) : round_up(k, KSTEP);
    // fast mode: any k the encode grid spans (the residue product is k-chunked beyond 2^17, gemm_i8);
    // accurate mode: the bound product of 6-bit magnitudes (|x| <= 2^12 k) must stay int32-exact
    if (kr > (fast ? ((size_t)1 << 22) : (((size_t)1 << 19) - KSTEP))) return GEMMUL8_E_SIZE;
    const bool ta_t = op_a != GEMMUL8_OP_N, tb_t = op_b != GEMMUL8_OP_N;
    if (lda < (ta_t ? k : m) || ldb < (tb_t ? n : k) || ldc < m) return GEMMUL8_E_SIZE;
    c.A = OperandDesc{A, lda, ta_t, dt_dbl(ta), cp, cp && op_a == GEMMUL8_OP_C};
    c.B = OperandDesc{B, ldb, !tb_t, dt_dbl(tb), cp, cp && op_b == GEMMUL8_OP_C};
    c.ctype = ctype;
    c.m = m; c.n = n; c.k = k; c.N = N;
    c.fast = fast != 0;
    c.cplx = cp;
    c.ot = static_cast<OutType>(tc);
    c.alpha = alpha; c.beta = beta; c.C = C; c.ldc = ldc; c.work = work;
    // threads_scaling of the matching reference entry point (gemmul8.cu:218-222, 361-365, 502-506, 648-652):
    // 512 for gemm<float>, 128 for gemm<double>, the mixed and the complex paths
    c.VT = (ta == GEMMUL8_R_32F && tb == GEMMUL8_R_32F && tc == GEMMUL8_R_32F) ? 512 : 128;
    c.st = static_cast<hipStream_t>(stream);
    c.stB = c.st;
    c.lane = nullptr;
    return GEMMUL8_OK;
}

}  // namespace oz2

// =============================== C ABI ===================================
extern "C" {

size_t gemmul8_work_size(size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type) {
    if (compute_type < 0 || compute_type > 3) return 0;
    const bool cp = compute_type != GEMMUL8_REAL_DEFAULT;
    return oz2::make_layout(m, n, k, num_moduli, cp).total;
}

int gemmul8_gemm(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b, int type_c,
                 const void *alpha, const void *A, size_t lda, const void *B, size_t ldb, const void *beta, void *C,
                 size_t ldc, unsigned num_moduli, int fastmode, void *work, int compute_type, double *phase_ns) {
    oz2::Call c{};
    const int rc = oz2::prepare(stream, op_a, op_b, m, n, k, type_a, type_b, type_c, alpha, A, lda, B, ldb, beta, C,
                                ldc, num_moduli, fastmode, work, compute_type, c);
    if (rc != GEMMUL8_OK) return rc;
    if (m == 0 || n == 0) return GEMMUL8_OK;
    oz2::clear_stale_error();
    return oz2::run(c, phase_ns);
}

size_t gemmul8_work_size_lowmem(size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type,
                                unsigned slice_planes) {
    if (compute_type < 0 || compute_type > 3) return 0;
    return oz2::make_layout(m, n, k, num_moduli, compute_type != GEMMUL8_REAL_DEFAULT, slice_planes).total;
}

int gemmul8_gemm_lowmem(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *alpha, const void *A, size_t lda, const void *B, size_t ldb,
                        const void *beta, void *C, size_t ldc, unsigned num_moduli, int fastmode, void *work,
                        int compute_type, unsigned slice_planes, double *phase_ns) {
    oz2::Call c{};
    const int rc = oz2::prepare(stream, op_a, op_b, m, n, k, type_a, type_b, type_c, alpha, A, lda, B, ldb, beta, C,
                                ldc, num_moduli, fastmode, work, compute_type, c);
    if (rc != GEMMUL8_OK) return rc;
    c.slice_planes = slice_planes;
    if (m == 0 || n == 0) return GEMMUL8_OK;
    oz2::clear_stale_error();
    return oz2::run(c, phase_ns);
}

int gemmul8_split_bound(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli,
                        void *work, int compute_type) {
    oz2::Call c{};
    const int rc = oz2::prepare(stream, op_a, op_b, m, n, k, type_a, type_b, type_c, nullptr, A, lda, B, ldb, nullptr,
                                nullptr, m, num_moduli, 0, work, compute_type, c);
    if (rc != GEMMUL8_OK) return rc;
    if (m == 0 && n == 0) return GEMMUL8_OK;
    oz2::clear_stale_error();
    const oz2::Views v = oz2::views(work, m, n, k, num_moduli, c.cplx);
    if (m == 0 || n == 0) {  // an empty block contributes nothing to the other operand's maxima
        oz2::zero_i32(v.bound, v.L.bm_pad + v.L.bn_pad, c.st);
        return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
    }
    oz2::LaneGuard lane(c);
    oz2::phase_bound(c, v);
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_split(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b, int type_c,
                  const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli, int fastmode, void *work,
                  int compute_type, unsigned mod_begin, unsigned mod_end, int flags) {
    oz2::Call c{};
    const int rc = oz2::prepare(stream, op_a, op_b, m, n, k, type_a, type_b, type_c, nullptr, A, lda, B, ldb, nullptr,
                                nullptr, m, num_moduli, fastmode, work, compute_type, c);
    if (rc != GEMMUL8_OK) return rc;
    // mod_begin == mod_end: the shifts only (no slices)
    if (mod_begin > mod_end || mod_end > num_moduli) return GEMMUL8_E_MODULI;
    if (m == 0 || n == 0) return GEMMUL8_OK;
    if (mod_begin == mod_end && (flags & GEMMUL8_SPLIT_SHIFTS_READY)) return GEMMUL8_OK;
    oz2::clear_stale_error();
    oz2::LaneGuard lane(c);
    oz2::phase_split(c, oz2::views(work, m, n, k, num_moduli, c.cplx), mod_begin, mod_end,
                     (flags & GEMMUL8_SPLIT_BOUND_READY) != 0, (flags & GEMMUL8_SPLIT_SHIFTS_READY) != 0);
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_products(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type, void *work,
                     unsigned mod_begin, unsigned mod_end) {
    return gemmul8_products_cols(stream, m, n, k, num_moduli, compute_type, work, mod_begin, mod_end, 0, n);
}

int gemmul8_products_cols(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type,
                          void *work, unsigned mod_begin, unsigned mod_end, size_t col_begin, size_t col_end) {
    if (num_moduli < 2 || num_moduli > 20 || mod_begin >= mod_end || mod_end > num_moduli) return GEMMUL8_E_MODULI;
    if (compute_type < GEMMUL8_REAL_DEFAULT || compute_type > GEMMUL8_COMPLEX_KARATSUBA_MULT) return GEMMUL8_E_TYPES;
    if (col_begin > col_end || col_end > n) return GEMMUL8_E_SIZE;
    if (m == 0 || col_begin == col_end) return GEMMUL8_OK;
    if (col_begin % oz2::TILE || (col_end != n && col_end % oz2::TILE)) return GEMMUL8_E_SIZE;
    oz2::clear_stale_error();
    const oz2::Views v = oz2::views(work, m, n, k, num_moduli, compute_type != GEMMUL8_REAL_DEFAULT);
    hipStream_t st = static_cast<hipStream_t>(stream);
    // with timing enabled the launch is timed like gemmul8_gemm's product phase (phases 0/3 read 0)
    bool record;
    oz2::timing::Rec rec{};
    {
        std::lock_guard<std::mutex> g(oz2::timing::mu);
        record = oz2::timing::enabled && !oz2::is_capturing(st);
        if (record) {
            rec = oz2::timing::acquire();
            rec.prod_only = true;
        }
    }
    oz2::timing::Phase prod(record, st, rec.prod0, rec.prod1);
    if (col_begin == 0 && col_end == n) oz2::phase_products(v, num_moduli, mod_begin, mod_end, mod_begin, st, false);
    else oz2::phase_products_cols(v, num_moduli, mod_begin, mod_end, col_begin, col_end, st);
    prod.end();
    if (record) {
        std::lock_guard<std::mutex> g(oz2::timing::mu);
        oz2::timing::pending.push_back(rec);
    }
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_recombine(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c, int compute_type,
                      const void *alpha, const void *beta, void *C, size_t ldc, void *work) {
    return gemmul8_recombine_cols(stream, m, n, k, num_moduli, type_c, compute_type, alpha, beta, C, ldc, work, 0, n);
}

int gemmul8_recombine_cols(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c,
                           int compute_type, const void *alpha, const void *beta, void *C, size_t ldc, void *work,
                           size_t col_begin, size_t col_end) {
    if (num_moduli < 2 || num_moduli > 20) return GEMMUL8_E_MODULI;
    if (col_begin > col_end || col_end > n) return GEMMUL8_E_SIZE;
    if (type_c < 0 || type_c > 3) return GEMMUL8_E_TYPES;
    const bool cp = compute_type != GEMMUL8_REAL_DEFAULT;
    if (cp != oz2::dt_cplx(type_c)) return GEMMUL8_E_TYPES;
    if (compute_type < GEMMUL8_REAL_DEFAULT || compute_type > GEMMUL8_COMPLEX_KARATSUBA_MULT) return GEMMUL8_E_TYPES;
    if (ldc < m) return GEMMUL8_E_SIZE;
    if (m == 0 || col_begin == col_end) return GEMMUL8_OK;
    oz2::clear_stale_error();
    const oz2::Views v = oz2::views(work, m, n, k, num_moduli, cp);
    oz2::phase_crt(v, num_moduli, static_cast<oz2::OutType>(type_c), alpha, beta, C, ldc,
                   static_cast<hipStream_t>(stream), col_begin, col_end);
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

// partial CRT sums / finish (the north star's reduce of FP64 partial accumulators; include/gemmul8_c.h)
static int crt_parts_check(size_t m, size_t n, unsigned num_moduli, int type_c, int compute_type, size_t lds) {
    if (num_moduli < 2 || num_moduli > 20) return GEMMUL8_E_MODULI;
    if (compute_type != GEMMUL8_REAL_DEFAULT) return GEMMUL8_E_UNSUPPORTED;
    if (type_c != GEMMUL8_R_64F && type_c != GEMMUL8_R_32F) return GEMMUL8_E_TYPES;
    if (lds < m) return GEMMUL8_E_SIZE;
    (void)n;
    return GEMMUL8_OK;
}

int gemmul8_crt_partial(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c,
                        int compute_type, const void *work, unsigned mod_begin, unsigned mod_end, double *sums,
                        size_t lds) {
    const int rc = crt_parts_check(m, n, num_moduli, type_c, compute_type, lds);
    if (rc != GEMMUL8_OK) return rc;
    if (mod_begin > mod_end || mod_end > num_moduli) return GEMMUL8_E_MODULI;
    if (m == 0 || n == 0) return GEMMUL8_OK;
    oz2::clear_stale_error();
    const oz2::Views v = oz2::views(const_cast<void *>(work), m, n, k, num_moduli, false);
    const oz2::CrtParams CP = oz2::make_crt_params(num_moduli, type_c == GEMMUL8_R_32F);
    oz2::crt_partial(v.R, v.L, num_moduli, CP.numM1 != 0, mod_begin, mod_end, sums, lds,
                     static_cast<hipStream_t>(stream));
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_crt_finish(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c,
                       int compute_type, const void *alpha, const void *beta, void *C, size_t ldc, const void *work,
                       const double *sums, size_t lds) {
    const int rc = crt_parts_check(m, n, num_moduli, type_c, compute_type, lds);
    if (rc != GEMMUL8_OK) return rc;
    if (ldc < m) return GEMMUL8_E_SIZE;
    if (m == 0 || n == 0) return GEMMUL8_OK;
    oz2::clear_stale_error();
    const oz2::Views v = oz2::views(const_cast<void *>(work), m, n, k, num_moduli, false);
    const oz2::CrtParams CP = oz2::make_crt_params(num_moduli, type_c == GEMMUL8_R_32F);
    oz2::crt_finish(sums, lds, v.L, num_moduli, CP.numM1 != 0, v.sftA, v.sftB, type_c == GEMMUL8_R_32F, alpha, beta,
                    C, ldc, static_cast<hipStream_t>(stream), oz2::g_epilogue_mode.load(std::memory_order_relaxed));
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_shard_stats(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli,
                        int fastmode, void *work, int compute_type, size_t row_begin, size_t row_end,
                        size_t col_begin, size_t col_end) {
    oz2::Call c{};
    const int rc = oz2::prepare(stream, op_a, op_b, m, n, k, type_a, type_b, type_c, nullptr, A, lda, B, ldb, nullptr,
                                nullptr, m, num_moduli, fastmode, work, compute_type, c);
    if (rc != GEMMUL8_OK) return rc;
    if (row_begin > row_end || row_end > m || col_begin > col_end || col_end > n) return GEMMUL8_E_SIZE;
    const size_t rows = row_end - row_begin, cols = col_end - col_begin;
    if (rows == 0 && cols == 0) return GEMMUL8_OK;
    oz2::clear_stale_error();
    const oz2::Views v = oz2::views(work, m, n, k, num_moduli, c.cplx);
    const oz2::OperandDesc a = oz2::sub_operand(c.A, row_begin), b = oz2::sub_operand(c.B, col_begin);
    if (c.fast) {
        const float log2M = oz2_log2M_fast[num_moduli - 2];
        int16_t *sa = v.sftA + row_begin, *sb = v.sftB + col_begin;
        if (!(rows && cols && oz2::split_stats_pair(a, rows, b, cols, k, c.VT, log2M, sa, sb, c.st))) {
            if (rows) oz2::split_stats(a, k, rows, c.VT, false, log2M, sa, c.st);
            if (cols) oz2::split_stats(b, k, cols, c.VT, false, log2M, sb, c.st);
        }
    } else {  // sft0 = 5 - ilogb(amax): A's rows at sft0[0, bm_pad), B's columns after them (phase_bound)
        if (rows) oz2::split_stats(a, k, rows, c.VT, true, 0.f, v.sft0 + row_begin, c.st);
        if (cols) oz2::split_stats(b, k, cols, c.VT, true, 0.f, v.sft0 + v.L.bm_pad + col_begin, c.st);
    }
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_shard_bound(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli,
                        void *work, int compute_type, size_t col_begin, size_t col_end) {
    oz2::Call c{};
    const int rc = oz2::prepare(stream, op_a, op_b, m, n, k, type_a, type_b, type_c, nullptr, A, lda, B, ldb, nullptr,
                                nullptr, m, num_moduli, 0, work, compute_type, c);
    if (rc != GEMMUL8_OK) return rc;
    if (col_begin > col_end || col_end > n) return GEMMUL8_E_SIZE;
    if (col_begin != col_end && (col_begin % oz2::TILE || (col_end != n && col_end % oz2::TILE))) return GEMMUL8_E_SIZE;
    if (m == 0 || n == 0) return GEMMUL8_OK;
    oz2::clear_stale_error();
    const oz2::Views v = oz2::views(work, m, n, k, num_moduli, c.cplx);
    oz2::LaneGuard lane(c);
    oz2::phase_bound(c, v, col_begin, col_end, true);
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

void gemmul8_timing_enable(int on) {
    std::lock_guard<std::mutex> g(oz2::timing::mu);
    oz2::timing::enabled = on != 0;
}

int gemmul8_timing_read(double *phase_ms, int *calls) {
    std::lock_guard<std::mutex> g(oz2::timing::mu);
    oz2::timing::resolve_all();
    for (int i = 0; i < 4; ++i) {
        phase_ms[i] = oz2::timing::acc_ms[i];
        oz2::timing::acc_ms[i] = 0;
    }
    *calls = oz2::timing::calls;
    oz2::timing::calls = 0;
    return GEMMUL8_OK;
}

int gemmul8_layout(size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type, size_t *out) {
    const oz2::Layout L = oz2::make_layout(m, n, k, num_moduli, compute_type != GEMMUL8_REAL_DEFAULT);
    const size_t v[24] = {L.m_pad, L.n_pad, L.k_pad,  L.ksteps, L.planeA, L.planeB, L.planeR, L.offA,
                          L.offB,  L.offR,  L.offSftA, L.offSftB, L.offBound, L.offSft0, L.total, L.kblk,
                          L.ldr,   L.nsub,  L.subA,  L.subB,   L.subR,   L.vsA,    L.vsB,    L.bm_pad};
    for (int i = 0; i < 24; ++i) out[i] = v[i];
    return GEMMUL8_OK;
}

int gemmul8_i8_product_raw(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type,
                           void *work, int32_t *C32) {
    const oz2::Layout L = oz2::make_layout(m, n, k, num_moduli, compute_type != GEMMUL8_REAL_DEFAULT);
    int8_t *base = static_cast<int8_t *>(work);
    const oz2::ModParams MP = oz2::make_mod_params(num_moduli);
    oz2::clear_stale_error();
    oz2::gemm_i8(base + L.offA, base + L.offB, L, 1, oz2::Epi::RAW, C32, nullptr, nullptr, MP,
                 static_cast<hipStream_t>(stream));
    return oz2::launch_ok() ? GEMMUL8_OK : GEMMUL8_E_HIP;
}

int gemmul8_set_epilogue(int mode) {
    if (mode != GEMMUL8_EPILOGUE_BLAS && mode != GEMMUL8_EPILOGUE_REFERENCE) return GEMMUL8_E_UNSUPPORTED;
    oz2::g_epilogue_mode.store(mode, std::memory_order_relaxed);
    return GEMMUL8_OK;
}

int gemmul8_get_epilogue(void) { return oz2::g_epilogue_mode.load(std::memory_order_relaxed); }

const char *gemmul8_last_products_kernel(void) {
    const bool tail = oz2::g_last_tail_small.load(std::memory_order_relaxed) != 0;
    switch (oz2::g_last_residue_kernel.load(std::memory_order_relaxed)) {
    case 1: return tail ? "gemm_i8_kernel+gemm_i8_small_kernel" : "gemm_i8_kernel";
    case 2: return tail ? "gemm_i8_persistent_kernel+gemm_i8_small_kernel" : "gemm_i8_persistent_kernel";
    case 3: return "gemm_i8_kernel (k-chunked)";
    case 4: return "gemm_i8_small_kernel";
    case 5: return tail ? "gemm_i8_persistent_pg_kernel+gemm_i8_small_kernel" : "gemm_i8_persistent_pg_kernel";
    default: return "none";
    }
}

unsigned long long gemmul8_residue_selftest(void *stream, int path) {
    return oz2::residue_selftest(path, static_cast<hipStream_t>(stream));
}

}  // extern "C"

// =========================== drop-in C++ API ===============================
namespace gemmul8 {

// the reference's own per-encoding size functions are exported symbols (gemmul8.cu:27-127)
size_t workSize_real(const size_t m, const size_t n, const size_t k, const unsigned num_moduli) {
    return oz2::make_layout(m, n, k, num_moduli, false).total;
}
size_t workSize_bigmatrix(const size_t m, const size_t n, const size_t k, const unsigned num_moduli) {
    return oz2::make_layout(m, n, k, num_moduli, true).total;
}
size_t workSize_kara(const size_t m, const size_t n, const size_t k, const unsigned num_moduli) {
    return oz2::make_layout(m, n, k, num_moduli, true).total;
}

size_t workSize(const size_t m, const size_t n, const size_t k, const unsigned num_moduli,
                const computeType_t computeType) {
    switch (computeType) {
    case REAL_DEFAULT: return workSize_real(m, n, k, num_moduli);
    case COMPLEX_BIG_MATRIX_ENCODE: return workSize_bigmatrix(m, n, k, num_moduli);
    case COMPLEX_CLASSIC_MULT:
    case COMPLEX_KARATSUBA_MULT: return workSize_kara(m, n, k, num_moduli);
    default: fprintf(stderr, "Unknown compute type\n"); return 0;
    }
}

template <typename T> struct dtype_of;
template <> struct dtype_of<double> { static constexpr int v = GEMMUL8_R_64F; };
template <> struct dtype_of<float> { static constexpr int v = GEMMUL8_R_32F; };
template <> struct dtype_of<hipDoubleComplex> { static constexpr int v = GEMMUL8_C_64F; };
template <> struct dtype_of<hipFloatComplex> { static constexpr int v = GEMMUL8_C_32F; };

static int op_code(hipblasOperation_t op) {
    return op == HIPBLAS_OP_N ? GEMMUL8_OP_N : (op == HIPBLAS_OP_T ? GEMMUL8_OP_T : GEMMUL8_OP_C);
}

// GEMMUL8_TIMERS=0: gemmul8::gemm returns {0,0,0,0} without waiting for its kernels (the call is then as
// asynchronous as gemmul8_gemm with phase_ns = NULL: everything is enqueued on the handle's stream); unset or
// any other value: the reference's contract, phase times in ns, the call returning after its own completion
// (gemmul8.hpp:24-28).  Read once per process.
static bool cxx_timers() {
    static const bool on = [] {
        const char *e = getenv("GEMMUL8_TIMERS");
        return !(e && e[0] == '0' && e[1] == 0);
    }();
    return on;
}

template <typename TA, typename TB, typename TC>
static std::vector<double> gemm_impl(hipblasHandle_t handle, hipblasOperation_t op_A, hipblasOperation_t op_B,
                                     size_t m, size_t n, size_t k, const TC *alpha, const TA *A, size_t lda,
                                     const TB *B, size_t ldb, const TC *beta, TC *C, size_t ldc, unsigned num_moduli,
                                     bool fastmode, void *work, computeType_t computeType) {
    std::vector<double> timer(4, 0.0);
    hipStream_t st = nullptr;
    if (handle) (void)hipblasGetStream(handle, &st);
    const int rc = gemmul8_gemm(st, op_code(op_A), op_code(op_B), m, n, k, dtype_of<TA>::v, dtype_of<TB>::v,
                                dtype_of<TC>::v, alpha, A, lda, B, ldb, beta, C, ldc, num_moduli, fastmode ? 1 : 0,
                                work, (int)computeType, cxx_timers() ? timer.data() : nullptr);
    if (rc == GEMMUL8_E_TYPES) fprintf(stderr, "Unsupported compute type for the argument types.\n");
    else if (rc != GEMMUL8_OK) fprintf(stderr, "gemmul8::gemm: invalid arguments or unsupported mode (code %d)\n", rc);
    if (rc != GEMMUL8_OK) return std::vector<double>(4, 0.0);
    return timer;
}

#define GEMMUL8_DEFINE(TA_, TB_, TC_)                                                                              \
    template <>                                                                                                    \
    std::vector<double> gemm<TA_, TB_, TC_>(hipblasHandle_t handle, const hipblasOperation_t op_A,                  \
                                            const hipblasOperation_t op_B, const size_t m, const size_t n,          \
                                            const size_t k, const TC_ *alpha, const TA_ *const A, const size_t lda, \
                                            const TB_ *const B, const size_t ldb, const TC_ *beta, TC_ *const C,    \
                                            const size_t ldc, const unsigned num_moduli, const bool fastmode,      \
                                            void *const work, const computeType_t computeType) {                  \
        return gemm_impl<TA_, TB_, TC_>(handle, op_A, op_B, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc,          \
                                        num_moduli, fastmode, work, computeType);                                  \
    }

GEMMUL8_DEFINE(double, double, double)
GEMMUL8_DEFINE(float, float, float)
GEMMUL8_DEFINE(double, float, double)
GEMMUL8_DEFINE(float, double, double)
GEMMUL8_DEFINE(double, float, float)
GEMMUL8_DEFINE(float, double, float)
GEMMUL8_DEFINE(hipFloatComplex, hipFloatComplex, hipFloatComplex)
GEMMUL8_DEFINE(hipDoubleComplex, hipDoubleComplex, hipDoubleComplex)
GEMMUL8_DEFINE(hipFloatComplex, hipDoubleComplex, hipDoubleComplex)
GEMMUL8_DEFINE(hipDoubleComplex, hipFloatComplex, hipDoubleComplex)
GEMMUL8_DEFINE(hipDoubleComplex, hipFloatComplex, hipFloatComplex)
GEMMUL8_DEFINE(hipFloatComplex, hipDoubleComplex, hipFloatComplex)
#undef GEMMUL8_DEFINE

}  // namespace gemmul8
