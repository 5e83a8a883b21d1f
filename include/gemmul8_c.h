/* gemmul8_c.h -- C ABI of the MI355X-native Ozaki-scheme-II GEMM emulator.
 *
 * Plain pointers and sizes only (no C++ / torch types), for ctypes, cgo, JNI or
 * any FFI.  The reference has no C ABI; each entry below replaces one C++ entry
 * point of GEMMul8/include/gemmul8.hpp:
 *
 *   gemmul8_work_size  <- gemmul8::workSize            (gemmul8.hpp:18-22, gemmul8.cu:129-147)
 *   gemmul8_gemm       <- gemmul8::gemm<TA,TB,TC>      (gemmul8.hpp:29-287, gemmul8.cu:149-1316)
 *                         stream instead of hipblasHandle_t, dtype codes instead of template args
 *
 * All device pointers are column-major HIP device memory; alpha/beta are host
 * pointers to one TC value; the work buffer is caller-owned (>= work size).
 * Return codes: 0 ok, GEMMUL8_E_* < 0 on invalid arguments (nothing enqueued).
 * GEMMUL8_E_HIP: a kernel launch of THIS call failed; the phases after it were not enqueued
 * (C is written only by the last phase).  An error left pending on the calling thread by
 * earlier HIP calls is neither reported as the call's own nor cleared (hipGetLastError still
 * returns it to the application).
 */
#ifndef GEMMUL8_C_H
#define GEMMUL8_C_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { GEMMUL8_OP_N = 0, GEMMUL8_OP_T = 1, GEMMUL8_OP_C = 2 };
enum { GEMMUL8_R_64F = 0, GEMMUL8_R_32F = 1, GEMMUL8_C_64F = 2, GEMMUL8_C_32F = 3 };
enum { GEMMUL8_REAL_DEFAULT = 0, GEMMUL8_COMPLEX_BIG_MATRIX_ENCODE = 1, GEMMUL8_COMPLEX_CLASSIC_MULT = 2,
       GEMMUL8_COMPLEX_KARATSUBA_MULT = 3 };
enum {
    GEMMUL8_OK = 0,
    GEMMUL8_E_MODULI = -1,       /* num_moduli outside [2, 20] */
    GEMMUL8_E_TYPES = -2,        /* unsupported dtype combination for compute_type */
    GEMMUL8_E_OP = -3,           /* unsupported transpose op */
    GEMMUL8_E_SIZE = -4,         /* padded k beyond 2^22 (fast) / 2^19 - 64 (accurate), or a leading dimension too small */
    GEMMUL8_E_UNSUPPORTED = -5,  /* compute type / mode not implemented on this build */
    GEMMUL8_E_HIP = -6           /* a HIP launch or runtime call failed */
};

/* bytes of workspace required by gemmul8_gemm for this shape (0 for an unknown compute_type) */
size_t gemmul8_work_size(size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type);

/* C = alpha * op(A) * op(B) + beta * C, emulated with num_moduli int8 products.
 * stream: hipStream_t (NULL = null stream).  fastmode: 1 = vecnorm shifts, 0 = accurate (int8 bound product).
 * phase_ns: optional double[4]; when non-NULL the call waits for its own completion and stores the
 * phase times {scaling, int8 products, conversion (fused: 0), inverse scaling} in nanoseconds. */
int gemmul8_gemm(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b, int type_c,
                 const void *alpha, const void *A, size_t lda, const void *B, size_t ldb, const void *beta, void *C,
                 size_t ldc, unsigned num_moduli, int fastmode, void *work, int compute_type, double *phase_ns);

/* --- low-memory mode ------------------------------------------------------
 * The same product with only `slice_planes` planes of A / B slices resident: the moduli are
 * encoded and multiplied in groups of that size (A and B are re-read once per group).  The
 * result is bit-identical to gemmul8_gemm.  At 8192^3 with 14 moduli the workspace drops from
 * 2.63 GiB to 1.13 GiB with slice_planes = 2.  slice_planes = 0 or >= num_moduli: all resident. */
size_t gemmul8_work_size_lowmem(size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type,
                                unsigned slice_planes);
int gemmul8_gemm_lowmem(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *alpha, const void *A, size_t lda, const void *B, size_t ldb,
                        const void *beta, void *C, size_t ldc, unsigned num_moduli, int fastmode, void *work,
                        int compute_type, unsigned slice_planes, double *phase_ns);

/* --- phase entry points (multi-GPU sharding, gemmul8/dist.py) ------------------------------------
 * gemmul8_gemm == gemmul8_split(0, N) + gemmul8_products(0, N) + gemmul8_recombine, on one stream.
 * Splitting the moduli range lets a rank produce only the residue planes [mod_begin, mod_end)
 * (plane j at work + offR + j * planeR, see gemmul8_layout), e.g. to send them to a root that runs
 * gemmul8_recombine (gemm_moduli_planes_to_root); the sharded entry points further below split the
 * columns too, and the CRT with them (gemm_moduli).
 *
 * Accurate mode couples the shifts of op(B)'s columns to every row of op(A) (the int8 bound
 * product's column maxima).  A row-block shard therefore runs gemmul8_split_bound, combines the
 * column maxima (int32 [n] at work + offBound + 4 * m_pad) with a MAX all-reduce, and calls
 * gemmul8_split with GEMMUL8_SPLIT_BOUND_READY.
 *
 * One workspace may serve several gemmul8_products / _products_cols launches in flight on
 * different streams only when their mod_begin differ (each first modulus has its own tile-queue
 * heads); launches ordered on one stream may share anything. */
enum { GEMMUL8_SPLIT_BOUND_READY = 1, GEMMUL8_SPLIT_SHIFTS_READY = 2 };
int gemmul8_split_bound(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli,
                        void *work, int compute_type);
/* flags: GEMMUL8_SPLIT_BOUND_READY (accurate: bound maxima in the workspace, derive the shifts from
 * them), GEMMUL8_SPLIT_SHIFTS_READY (sftA / sftB already in the workspace: encode the slices only).
 * mod_begin == mod_end: the shifts only, no slices (e.g. an accurate-mode shard that multiplies no
 * modulus but recombines columns). */
int gemmul8_split(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b, int type_c,
                  const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli, int fastmode, void *work,
                  int compute_type, unsigned mod_begin, unsigned mod_end, int flags);
int gemmul8_products(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type, void *work,
                     unsigned mod_begin, unsigned mod_end);
int gemmul8_recombine(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c, int compute_type,
                      const void *alpha, const void *beta, void *C, size_t ldc, void *work);

/* --- sharded entry points (the moduli x column-block partition of gemmul8/dist.py) ---------------
 * Every output element's CRT needs all N residues, and every residue plane is column-major
 * (plane j, column c at work + offR + j * planeR + c * ldr), so a column range of a plane is one
 * contiguous run of bytes.  A job over W ranks: (1) each rank computes the shifts of its own
 * rows / columns (gemmul8_shard_stats), the ranks all-gather the int16 shift vectors into every
 * workspace (offSftA / offSftB; accurate mode: sft0 at offSft0, A's rows then B's columns from
 * bm_pad), accurate mode then runs gemmul8_shard_bound over its column range and MAX-all-reduces
 * the bound area (int32 [bm_pad + n_pad] at offBound); (2) gemmul8_split(..., SHIFTS_READY or
 * BOUND_READY) encodes its moduli; (3) gemmul8_products_cols produces its (modulus, column-range)
 * units; (4) the ranks exchange the residue column runs so each holds all N planes of its own
 * output columns; (5) gemmul8_recombine_cols.  Row / column range starts are multiples of 256
 * (the product tile) for products_cols / shard_bound; range ends are multiples of 256 or n.
 * The result is bit-identical to gemmul8_gemm on the same operands. */
/* fast mode: sftA[row_begin, row_end) and sftB[col_begin, col_end); accurate mode: the sft0 of the same ranges */
int gemmul8_shard_stats(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli,
                        int fastmode, void *work, int compute_type, size_t row_begin, size_t row_end,
                        size_t col_begin, size_t col_end);
/* accurate mode, sft0 assembled: magnitude planes + the bound product over columns [col_begin, col_end)
 * (the bound area is zeroed first; the other columns' maxima stay 0) */
int gemmul8_shard_bound(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                        int type_c, const void *A, size_t lda, const void *B, size_t ldb, unsigned num_moduli,
                        void *work, int compute_type, size_t col_begin, size_t col_end);
/* residue planes [mod_begin, mod_end), columns [col_begin, col_end) only (one launch) */
int gemmul8_products_cols(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type,
                          void *work, unsigned mod_begin, unsigned mod_end, size_t col_begin, size_t col_end);
/* CRT + scaling + epilogue of the output columns [col_begin, col_end); C points at column col_begin */
int gemmul8_recombine_cols(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c,
                           int compute_type, const void *alpha, const void *beta, void *C, size_t ldc, void *work,
                           size_t col_begin, size_t col_end);

/* --- partial CRT sums (the north star's "single RCCL reduce of partial FP64 accumulators") ------
 * A rank holding the residue planes of moduli [mod_begin, mod_end) (gemmul8_split + gemmul8_products of that
 * range, every shift in its workspace) writes per output element the partial CRT sums of its range into
 * sums = column-major double [2][n][lds] (plane 0: C1 = sum hi_i r_i, plane 1: C2 = sum lo_i r_i; one-level
 * moduli, N <= 7 or float output: C1 = sum NMi_i r_i, C2 = 0) -- inverse_scaling.hpp:35-62, 138-172
 * restricted to the range.  The element-wise sums of all ranks' planes (an RCCL sum reduce) finish into C with
 * gemmul8_crt_finish (sftA / sftB from `work`).  Not bit-identical to gemmul8_gemm; how close depends on the
 * moduli level:
 *   two-level (f64 output, N >= 8): C1 is exact in any order, only C2's rounded sum is reordered: C within a
 *     few ulp, max |C - C_gemm| <= 2^-40 max |C_gemm| in the tests;
 *   one-level, N <= 5 (f64): every partial sum stays below 2^53, so C1 is exact: the same few-ulp bound;
 *   one-level, N = 6, 7 (f64): C1 = sum NMi_i r_i exceeds 2^53 and is rounded in whatever order the reduce
 *     takes (the single call's own C carries an error of that size): max |C - C_gemm| <= 2^-26 max |C_gemm|;
 *   float output (one-level at every N): the same reordering, then the rounding to float:
 *     max |C - C_gemm| <= 2^-19 max |C_gemm|.
 * Real outputs only (GEMMUL8_E_UNSUPPORTED for complex compute types). */
int gemmul8_crt_partial(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c,
                        int compute_type, const void *work, unsigned mod_begin, unsigned mod_end, double *sums,
                        size_t lds);
int gemmul8_crt_finish(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int type_c,
                       int compute_type, const void *alpha, const void *beta, void *C, size_t ldc, const void *work,
                       const double *sums, size_t lds);

/* --- instrumentation (used by bench.py / tests) --------------------------------------------- */
/* When enabled, every gemmul8_gemm records HIP events between its phases on its stream; the
 * accumulated per-phase milliseconds and the call count are read (and reset) with
 * gemmul8_timing_read, which synchronises on the recorded events. */
void gemmul8_timing_enable(int on);
int gemmul8_timing_read(double *phase_ms /* [4] */, int *calls);

/* Workspace layout for a shape: fills out[0..23] = {m_pad, n_pad, k_pad, ksteps, planeA, planeB,
 * planeR, offA, offB, offR, offSftA, offSftB, offBound, offSft0, total, kblk, ldr, nsub, subA, subB,
 * subR, vsA, vsB, bm_pad}.  Complex compute types run Karatsuba products: per modulus the slice planes
 * hold the sub-blocks [re | im | re + im] (vsA rows / vsB columns each, subA / subB bytes apart) and the
 * residue plane the three products Ar Br, Ai Bi, (Ar + Ai)(Br + Bi) (subR bytes apart, ld = ldr);
 * nsub = 1 otherwise.  The accurate-mode bound maxima are rows [0, bm_pad) then columns. */
int gemmul8_layout(size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type, size_t *out);

/* Validation hook: int32 product of plane 0 of the tiled int8 operands already in `work`
 * (layout of gemmul8_layout) into C32 (column-major, ld = m_pad).  Used by the MFMA tests. */
int gemmul8_i8_product_raw(void *stream, size_t m, size_t n, size_t k, unsigned num_moduli, int compute_type,
                           void *work, int32_t *C32);

/* Validation hook: exhaustive exactness check of the product kernel's residue epilogue against exact
 * arithmetic, for all 20 moduli -- path 0: the biased reduction (integer Barrett) over every x in
 * [-2^30, 2^30]; path 3: the same range through the f64 form the product kernels use; path 1: the
 * reference's signed Barrett step (conv_32i_2_8u.hpp:7-56) over every int32.  Returns the number of
 * mismatching (input, modulus) pairs (0 expected; path 2 is a negative control that compares path 0
 * with a wrong expectation, so every pair mismatches). */
unsigned long long gemmul8_residue_selftest(void *stream, int path);

/* Epilogue semantics of C = alpha * AB + beta * C, process-wide (default GEMMUL8_EPILOGUE_BLAS; the
 * environment variable GEMMUL8_EPILOGUE=reference selects the other at load time).
 *   GEMMUL8_EPILOGUE_BLAS       BLAS: beta = 0 never reads C; alpha = 1 with another beta is
 *                               beta * C + AB; beta = 1 is alpha * AB + C at every moduli count.
 *   GEMMUL8_EPILOGUE_REFERENCE  the reference's kernels bit for bit, its non-BLAS variants included
 *                               (inverse_scaling.hpp): alpha = 1 with beta off {0, 1} computes beta * AB + C
 *                               (_1b, :417, :682), alpha != 1 with beta = 1 at num_moduli >= 8 (two-level
 *                               moduli, real and complex double output) computes alpha * C + AB (_2_a1,
 *                               :736, :763), and alpha != 1 with beta = 0 reads C as fma(0, C, alpha * AB)
 *                               (_ab, :522, :549, :791, :819: NaN / Inf in C propagate).
 * Returns GEMMUL8_E_UNSUPPORTED for an unknown mode.  Takes effect for calls enqueued afterwards. */
enum { GEMMUL8_EPILOGUE_BLAS = 0, GEMMUL8_EPILOGUE_REFERENCE = 1 };
int gemmul8_set_epilogue(int mode);
int gemmul8_get_epilogue(void);

/* Name of the residue-product kernel the last products launch of this process took
 * ("gemm_i8_persistent_pg_kernel", "gemm_i8_persistent_kernel", "gemm_i8_kernel", "gemm_i8_small_kernel",
 * "gemm_i8_kernel (k-chunked)" or "none"). */
const char *gemmul8_last_products_kernel(void);

/* --- bench / test harness (not part of the emulation path) ------------------------------------ */
/* The reference's input generator (testing/make_matrix.hpp:8-71): x = (U(0,1] - 0.5) * exp(phi * N(0,1))
 * from hiprand XORWOW, init(seed, idx, 0); complex draws (u_re, n_re, u_im, n_im). dtype: GEMMUL8_*. */
int gemmul8_randmat(void *stream, int dtype, size_t m, size_t n, void *A, double phi, unsigned long long seed);
/* Double-double reference product C1 + C2 = A * B (testing/eval.hpp:265-308); A m x k, B k x n, col-major. */
int gemmul8_dd_gemm(void *stream, size_t m, size_t n, size_t k, const double *A, const double *B, double *C1,
                    double *C2);
/* err[i] = |C[i] - (C1[i] + C2[i])| / |C1[i] + C2[i]| evaluated in double-double (eval.hpp:317-338). */
int gemmul8_relerr_dd(void *stream, size_t count, const double *C, const double *C1, const double *C2, double *err);
/* the reference drivers' timing loop (GEMMul8/testing/test_double.cu:422-431) in native code: `iters` calls of
 * gemmul8_gemm, each bracketed by hipDeviceSynchronize and the host clock; *sec = mean seconds per call (calls
 * without phase events), phase_ns[4] = mean phase times from a second loop of `iters` calls (NULL: not run) */
int gemmul8_time_gemm(void *stream, int op_a, int op_b, size_t m, size_t n, size_t k, int type_a, int type_b,
                      int type_c, const void *alpha, const void *A, size_t lda, const void *B, size_t ldb,
                      const void *beta, void *C, size_t ldc, unsigned num_moduli, int fastmode, void *work,
                      int compute_type, int iters, double *sec, double *phase_ns);
/* the same loop around the vendor GEMM of the drivers (test_double.cu:318-331): hipblasGemmEx op N / N, alpha 1,
 * beta 0, every operand of `type`, lda = m, ldb = k, ldc = m */
int gemmul8_time_vendor_gemm(void *stream, int type, size_t m, size_t n, size_t k, const void *A, const void *B,
                             void *C, int iters, double *sec);
/* Data-bound ceiling of the int8 products: TOPS of the better of v_mfma_i32_32x32x32_i8 and
 * v_mfma_i32_16x16x64_i8 alone on uniformly random operand bytes held in registers (2 waves per
 * SIMD, the ops of `iters` x 64 32x32x32 MFMAs per wave); synchronises. */
double gemmul8_mfma_ceiling(void *stream, int iters);

#ifdef __cplusplus
}
#endif
#endif /* GEMMUL8_C_H */
