/*
 * vgposp.h — C-ABI of libvgposp.so, the MI355X (gfx950) hot path of DL-WG/VGPosp:
 * GP kernel assembly -> fp64 Cholesky (+ fused inverse) -> GP log-marginal-likelihood / gradient
 * -> greedy mutual-information sensor placement.
 *
 * The reference exposes this path as Python (TF1 graph + TFP + numpy).  Each entry point below
 * names the reference interface it replaces (file:line under the reference checkout).  Bindings:
 * vgposp_amd/_lib.py (ctypes); a maintainer-side ctypes stub for the reference is in
 * INTEGRATION.md.
 *
 * Conventions
 *   - Every array argument is a caller-owned DEVICE pointer (e.g. a torch tensor's data_ptr());
 *     the library never allocates device memory.  Scratch is passed in as `ws`/`ws_bytes`, sized
 *     by the matching *_workspace_bytes() query.
 *   - Matrices are row-major fp64 with an explicit leading dimension (elements).  Batched
 *     operands are `batch` matrices `stride` elements apart.
 *   - `stream` is a hipStream_t (may be NULL = default stream).  Calls only enqueue work: no host
 *     synchronisation happens inside the library, so device-side status (`info`) must be read by
 *     the caller after synchronising.
 *   - Return: 0 = enqueued; -i = argument i (1-based) invalid; VGPOSP_E_HIP = HIP runtime error;
 *     VGPOSP_E_WS = workspace too small.  vgposp_last_error() returns a thread-local message.
 *   - Device `info` (int32 per batch entry): 0 = success, k > 0 = the leading minor of order k
 *     is not positive definite (LAPACK potrf convention).  The Python layer maps k > 0 to the
 *     TF error "Cholesky decomposition was not successful".
 *   - Stateless and re-entrant; concurrent calls on different streams with disjoint buffers are
 *     safe.
 */
#ifndef VGPOSP_H_
#define VGPOSP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VGPOSP_ABI_VERSION 2

#define VGPOSP_E_HIP (-100)
#define VGPOSP_E_WS (-101)

/* PSD kernel families (tfp.positive_semidefinite_kernels). */
#define VGPOSP_KERNEL_EQ 0       /* ExponentiatedQuadratic: 3D_sin_wave.py:158-159, main_tests.py:617 */
#define VGPOSP_KERNEL_MATERN12 1 /* MaternOneHalf: gp_functions.py:160-163, main.py:94 */
#define VGPOSP_KERNEL_MATERN32 2 /* MaternThreeHalves */
#define VGPOSP_KERNEL_MATERN52 3 /* MaternFiveHalves: main_architecture_2_sampledistribution.py:211 */

/* Output triangle selectors. */
#define VGPOSP_FULL 0
#define VGPOSP_LOWER 1

int vgposp_abi_version(void);
const char* vgposp_last_error(void);

/* ---------------------------------------------------------------------------------------------
 * Kernel assembly.  Replaces `kernel.matrix(x1, x2)` of the TFP PSD kernels built by
 * gp_functions.create_cov_kernel (gp_functions.py:160-163) and consumed by tfd.GaussianProcess
 * (gp_functions.py:166-172), GPRM (:283-297) and the VGP (variational_Gaussian_process_example.py
 * :55-89):
 *     K[b][i][j] = exp(2*log(amp[b]) + log k(|X1_i - X2_j| / ls[b])) + (i==j ? diag_shift[b] : 0)
 * X1: n1 x d, X2: n2 x d (row-major, d <= 8).  amp, ls: [batch] device arrays.  diag_shift:
 * [batch] device array or NULL (added on i == j, used for noise + jitter of a symmetric K).
 * uplo = VGPOSP_LOWER writes only j <= i (the upper triangle is left untouched).
 * --------------------------------------------------------------------------------------------- */
int vgposp_kernel_matrix(int kind, const double* X1, int64_t n1, const double* X2, int64_t n2,
                         int d, const double* amp, const double* ls, const double* diag_shift,
                         int batch, int uplo, double* K, int64_t ldk, int64_t stride_k,
                         void* stream);

/* Kernel assembly fused with its product by a vector (the VGP's optimal posterior,
 * variational_Gaussian_process_example.py:68-74, needs Kzx and c = Kzx y over all N observations):
 * writes the full K (batch 1, no diagonal shift) and out[n1] = K v[n2] without re-reading K.
 * Deterministic (per-tile partials in ws, summed in a fixed order); ws is
 * vgposp_kernel_matrix_matvec_workspace_bytes(n1, n2) bytes. */
size_t vgposp_kernel_matrix_matvec_workspace_bytes(int64_t n1, int64_t n2);
int vgposp_kernel_matrix_matvec(int kind, const double* X1, int64_t n1, const double* X2,
                                int64_t n2, int d, const double* amp, const double* ls, double* K,
                                int64_t ldk, const double* v, double* out, void* ws,
                                size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * fp64 GEMM on MFMA (v_mfma_f64_16x16x4f64):  C = alpha * op(A) * op(B) + beta * C
 * op(A) = A (m x k, transa=0) or A^T (A stored k x m, transa=1);
 * op(B) = B (k x n, transb=0) or B^T (B stored n x k, transb=1).
 * uplo_c = VGPOSP_LOWER updates only the lower triangle of C (j <= i).  tri_a / tri_b = 1 treat
 * the STORED A / B as lower triangular (entries above their diagonal read as 0).
 * The building block of the Cholesky trailing update / TRMM / C^-1 formation below.
 * --------------------------------------------------------------------------------------------- */
int vgposp_gemm(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, void* stream);

/* Batched vgposp_gemm: element b (< batch) computes C + b sC from A + b sA and B + b sB, all in
 * one launch (e.g. the VGP's four M x M inverse factors' L^-T L^-1).  Split-K over the workspace
 * as vgposp_gemm_splitk when ws holds vgposp_gemm_batched_workspace_bytes, else unsplit. */
size_t vgposp_gemm_batched_workspace_bytes(int64_t m, int64_t n, int64_t k, int uplo_c, int batch);
int vgposp_gemm_batched(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                        const double* A, int64_t lda, int64_t sA, const double* B, int64_t ldb,
                        int64_t sB, double beta, double* C, int64_t ldc, int64_t sC, int uplo_c,
                        int tri_a, int tri_b, int batch, void* ws, size_t ws_bytes, void* stream);

/* Split-K form of vgposp_gemm for few output tiles and a long K (e.g. the VGP's
 * Kzx Kzx^T with M = 512 inducing points and K = N = 262,144 observations: 10 lower tiles).  Each
 * of `splits` K-ranges writes alpha * partial into ws ([splits][m][n]); a second kernel sums them
 * in a fixed order and adds beta * C, so results are deterministic.  splits <= 0 chooses a count
 * (about 512 workgroups, >= 512-deep ranges).  Falls back to vgposp_gemm's kernels (no split) for
 * operands the MFMA path does not take. */
size_t vgposp_gemm_splitk_workspace_bytes(int64_t m, int64_t n, int64_t k, int uplo_c, int splits);
/* Process-wide tuning of the automatic split-K: a short-K split (few output tiles, K < 4096) is at
 * least min_k deep (a multiple of 16 in [16, 4096]; default 16, measured: profiles/
 * r4_vgp_ab_splitk_*.jsonl).  Change it only while no work that was sized under the old value
 * is being enqueued: workspace queries (vgposp_*_workspace_bytes) and the launches that use the
 * workspace must see the same value.  Not read from the environment. */
int vgposp_gemm_set_split_depth(int min_k);
int vgposp_gemm_split_depth(void);
int vgposp_gemm_splitk(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                       const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                       double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, int splits,
                       void* ws, size_t ws_bytes, void* stream);

/* Grouped vgposp_gemm: `count` independent products, problem g with flags[5g..5g+4] = (transa,
 * transb, uplo_c, tri_a, tri_b), dims[3g..3g+2] = (m, n, k), alpha[g], beta[g], A[g] (lda[g]),
 * B[g] (ldb[g]), C[g] (ldc[g]), all in ONE launch (problem on blockIdx.y) plus one grouped split-K
 * reduction; problems the MFMA tile kernel does not take (n == 1, odd or unaligned operands) run
 * one by one.  For the VGP step's latency-bound M x M products.  ws holds
 * vgposp_gemm_group_workspace_bytes(count, flags, dims) bytes of split-K partials. */
size_t vgposp_gemm_group_workspace_bytes(int count, const int* flags, const int64_t* dims);
int vgposp_gemm_group(int count, const int* flags, const int64_t* dims, const double* alpha,
                      const double* beta, const double* const* A, const int64_t* lda,
                      const double* const* B, const int64_t* ldb, double* const* C,
                      const int64_t* ldc, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * VGP training-step glue (vgposp_amd/vgp_training.py): the non-GEMM element-wise and reduction
 * parts of variational_loss and of the gradient TF autodiff takes through it
 * (variational_Gaussian_process_example.py:51-102, AdamOptimizer.minimize).  Row-major fp64; s
 * (the observation noise variance) and amp are device scalars, so the step has no host sync.
 *   vgposp_vgp_sinv:       P0 (lower, from the SYRK) -> symmetric in place;
 *                          F[0] = Sinv = Kzz + P0 / s + pj I  (n x n, ld n); nf = 4 also
 *                          writes F[1] = Kzz + jitter I, F[2] = Kzz + (s + 1e-6) I, F[3] = Kzz
 *                          (the step's four M x M factorizations, done as one batch)
 *   vgposp_sym_from_lower: A's strict upper triangle <- its lower triangle
 *   vgposp_lincomb:        out = sum_k coef[k] (s + shift)^spow[k] X[k], on i == j times
 *                          diag_scale plus diag_coef (s + shift)^diag_spow; k <= 4, all
 *                          rows x cols with ld
 *   vgposp_vgp_kzz_bar:    KzzS = Kbar + Kbar^T of Kzz and G = (2 / s) Sinv_bar, from
 *                          vecs = {u, v, qv, m_bar, t, c_bar} and mats = {HHt, P HHt, Kp^-1,
 *                          QA QA^T, Kzz^-1, Li^T Li, Sc, Li^T A_bar} (n x n, ld n)
 *   vgposp_dots:           out[p] = sum_i x_p[i incx_p] y_p[i incy_p] (y_p NULL: sum x) for
 *                          op 0, sum_i log x_p[i incx_p] for op 1; p < 16, deterministic
 *   vgposp_vgp_scalars:    out = (-E, -dE/damp, -dE/dls, -dE/dnoise) from the sums below, the
 *                          three kernel-VJP gradients g1 (Kzz, halved inside), g2 (Kzx), g3 (Kzb)
 * --------------------------------------------------------------------------------------------- */
enum {
  VGPOSP_S_RR = 0,       /* r . r, r = y_b - Kzb^T Kzj^-1 m            */
  VGPOSP_S_KZB_H = 1,    /* <Kzb, H>, H = Kzj^-1 Kzb                   */
  VGPOSP_S_Q_HHT = 2,    /* <Q, H H^T>                                 */
  VGPOSP_S_PA2 = 3,      /* <Lp^-1 A, Lp^-1 A>                         */
  VGPOSP_S_QM2 = 4,      /* |Lp^-1 m|^2                                */
  VGPOSP_S_LOGDET_S = 5, /* sum log diag chol(Sinv)                    */
  VGPOSP_S_LOGDET_P = 6, /* sum log diag chol(Kzz + (s + 1e-6) I)      */
  VGPOSP_S_LOGDET_K = 7, /* sum log diag chol(Kzz)                     */
  VGPOSP_S_TR_KPINV = 8, /* tr Kp^-1                                   */
  VGPOSP_S_QV2 = 9,      /* |Kp^-1 m|^2                                */
  VGPOSP_S_TR_QAQA = 10, /* tr (Kp^-1 A)(Kp^-1 A)^T                    */
  VGPOSP_S_MB_M = 11,    /* m_bar . m                                  */
  VGPOSP_S_G_P0 = 12,    /* <G, P0>                                    */
  VGPOSP_S_COUNT = 13
};
int vgposp_vgp_sinv(double* P0, int64_t n, int64_t ldp, const double* Kzz, const double* s,
                    double pj, double jitter, double* F, int nf, void* stream);
int vgposp_sym_from_lower(double* A, int64_t n, int64_t lda, void* stream);
int vgposp_lincomb(int64_t rows, int64_t cols, int64_t ld, int nterms, const double* const* X,
                   const double* coef, const int* spow, double diag_scale, double diag_coef,
                   int diag_spow, const double* s, double shift, double* out, void* stream);
int vgposp_vgp_kzz_bar(int64_t n, const double* const* vecs, const double* const* mats,
                       const double* s, double w, double* KzzS, double* G, void* stream);
size_t vgposp_dots_workspace_bytes(int ndots);
int vgposp_dots(int ndots, const double* const* x, const int64_t* incx, const double* const* y,
                const int64_t* incy, const int64_t* len, const int* op, double* out, void* ws,
                size_t ws_bytes, void* stream);
int vgposp_vgp_scalars(const double* sums, const double* s, const double* amp, const double* g1,
                       const double* g2, const double* g3, double nb, double m, double w,
                       double jitter, double* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Vector-Jacobian product of kernel assembly: the reverse pass TF autodiff runs through
 * kernel.matrix when the reference trains a VGP (variational_Gaussian_process_example.py:95-102,
 * AdamOptimizer.minimize over amplitude, length_scale, inducing_index_points).  For one kernel
 * (amp, ls: device [1]) and Kbar [n1 x n2] (ld ldk) plus an optional rank-1 term u w^T
 * (u: [n1], w: [n2], both NULL or both set):
 *     grad[0] = sum_ij Kbar_ij dK_ij/damp,   grad[1] = sum_ij Kbar_ij dK_ij/dls,
 *     X1bar[i][:] = sum_j Kbar_ij dK_ij/dX1[i][:]    (X1bar [n1 x d] or NULL)
 * K is recomputed on the fly (one HBM pass over Kbar).  Deterministic (fixed-order reduction).
 * For a symmetric use (K(Z, Z)) pass Kbar + Kbar^T and halve grad.
 * --------------------------------------------------------------------------------------------- */
size_t vgposp_kernel_vjp_workspace_bytes(int64_t n1, int64_t n2, int d);
int vgposp_kernel_vjp(int kind, const double* X1, int64_t n1, const double* X2, int64_t n2, int d,
                      const double* amp, const double* ls, const double* Kbar, int64_t ldk,
                      const double* u, const double* w, double* grad, double* X1bar, void* ws,
                      size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Covariance builders (cov_vv on device).
 * vgposp_kernel_matvec: out[i] = sum_j K(X1_i, X2_j) v[j] + beta * out[i] for one kernel (amp, ls:
 *   device [1]), without materialising K: the VGP / GPRM predictive mean at many points, e.g. the
 *   tracer value at every (location, T/P sample) 5-D point that main_architecture_2_
 *   sampledistribution.py:432-458 evaluates one vgp.mean() at a time.
 * vgposp_center_rows: T[i][0:s] <- (T[i][:] - mean(T[i][:])) * scale.  A SYRK of the result
 *   (vgposp_gemm, alpha = 1/s) is tfp.stats.covariance(t_i, t_j, sample_axis=0) for every pair
 *   (main.py:190-199, main_architecture_2_sampledistribution.py:470-479).
 * vgposp_index_taper: C[i][j] *= g(|idx_i - idx_j|), g(d) = exp(-(beta d)^2 / (2 pi)), 0 where
 *   g < threshold, over an I0 x I1 x I2 C-order grid (the beta-decay local kernel filter,
 *   main_architecture_2_sampledistribution.py:361-421; threshold 0.01 there).  uplo as elsewhere.
 * --------------------------------------------------------------------------------------------- */
int vgposp_kernel_matvec(int kind, const double* X1, int64_t n1, const double* X2, int64_t n2,
                         int d, const double* amp, const double* ls, const double* v, double beta,
                         double* out, void* stream);
int vgposp_center_rows(double* T, int64_t n, int64_t s, int64_t ld, double scale, void* stream);
int vgposp_index_taper(double* C, int64_t n, int64_t ldc, int64_t I0, int64_t I1, int64_t I2,
                       double beta, double threshold, int uplo, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Recursive Cholesky, lower, in place (128x128 leaves in LDS, everything else fp64 MFMA GEMMs).
 * Replaces tf.linalg.cholesky inside tfd.GaussianProcess.log_prob / GPRM / VGP
 * (gp_functions.py:166-172, main.py:105, 3D_sin_wave.py:172) and is the O(N^3) core of the dense
 * greedy placement.
 *   invert = 0: lower triangle of A <- L with A = L L^T.
 *   invert = 1: lower triangle of A <- L^-1 (recursive triangular inverse after the factor).
 * The strictly upper triangle of A is never read or written (it keeps Sigma for the greedy
 * nominators).  diag_out ([batch][n], or NULL) receives diag(L) (log-det).  info: [batch] int32.
 * ws must hold vgposp_potrf_workspace_bytes(n).
 * --------------------------------------------------------------------------------------------- */
/* Workspace for factoring a batch of n > 128 matrices in ONE recursion (every launch covers the
 * whole batch): pass at least this many bytes to vgposp_potrf_lower with batch > 1 (a smaller
 * workspace of vgposp_potrf_workspace_bytes(n) factors them one after another). */
size_t vgposp_potrf_batched_workspace_bytes(int64_t n, int batch);
size_t vgposp_potrf_workspace_bytes(int64_t n);
int vgposp_potrf_lower(double* A, int64_t n, int64_t lda, int64_t stride, int batch, int invert,
                       double* diag_out, int* info, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Mixed-precision Cholesky (config C5, "fp32 mixed-prec Cholesky": the VGP's M x M factorizations,
 * tf.linalg.cholesky inside tfd.VariationalGaussianProcess, main_architecture_2_sampledistribution
 * .py:223-265): fp32 factor of A on the f32 matrix cores (v_mfma_f32_16x16x4_f32), then `iters`
 * fp64 refinement steps X <- (I - Phi(X A X^T - I)) X of X0 = L32^-1 (Phi: lower part, diagonal
 * halved), which converge quadratically to the fp64 inverse Cholesky factor.
 *   A: full symmetric n x n (lda), not modified.  Linv (ldl, != A) <- L^-1, zeros above the
 *   diagonal (what vgposp_potrf_lower(invert = 1) leaves in the lower triangle).  diag_out [n] (or
 *   NULL) <- diag(L) = 1 / diag(L^-1).  resid (device double or NULL) <- max|X A X^T - I| of the
 *   last step.  info: k > 0 = fp32 pivot k not positive; n + 1 = not converged (resid > 1e-6).
 * --------------------------------------------------------------------------------------------- */
size_t vgposp_potrf_mixed_workspace_bytes(int64_t n);
int vgposp_potrf_mixed(const double* A, int64_t n, int64_t lda, double* Linv, int64_t ldl,
                       double* diag_out, int iters, double* resid, int* info, void* ws,
                       size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * The Cholesky of ONE matrix distributed over R ranks (one process per GPU) that each hold the
 * whole matrix: the O(N^3) factorization behind placement_algorithm2.py:151-219's pinv calls,
 * which the candidate-sharded placement would otherwise replicate on every rank.
 * The host (vgposp_amd/dist_cholesky.py) walks vgposp_potrf_lower's recursion: a node of size nsub
 * at column col0 splits at n1 = vgposp_potrf_split(nsub); nodes below a size threshold are factored
 * whole on every rank (vgposp_potrf_block); above it every rank computes a share of the node's
 * panel TRSM (vgposp_potrf_panel: rows [r0, r1) of L21 = A21 L11^-T, rows counted from col0 + n1)
 * and of its SYRK (vgposp_potrf_trailing: rows [b0, b1) of the lower triangle of A22 -= L21 L21^T),
 * and the ranks all-gather the shares (vgposp_pack_rows / unpack into contiguous buffers, RCCL
 * all-gather).  ws: a vgposp_potrf_workspace_bytes(n) workspace for the whole n (the leaf and
 * 512-block inverses are kept at their global columns, as vgposp_potrf_lower leaves them, e.g.
 * vgposp_greedy_fact_ws's).  col0 is a multiple of 128.
 * vgposp_pack_rows: rows [r0, r1) x columns [c0, c1) of A (lower = 0) or the lower trapezoid
 * (columns [c0, r] of row r; lower = 1 needs c0 <= r0, c1 >= r1) <-> buf, packed row after row
 * (unpack = 1 writes A); vgposp_pack_elems gives the element count.
 * --------------------------------------------------------------------------------------------- */
int64_t vgposp_potrf_split(int64_t n);
int vgposp_potrf_block(double* A, int64_t n, int64_t lda, int64_t col0, int64_t nb, int* info,
                       void* ws, size_t ws_bytes, void* stream);
int vgposp_potrf_panel(double* A, int64_t n, int64_t lda, int64_t col0, int64_t nsub, int64_t r0,
                       int64_t r1, void* ws, size_t ws_bytes, void* stream);
int vgposp_potrf_trailing(double* A, int64_t n, int64_t lda, int64_t col0, int64_t nsub,
                          int64_t b0, int64_t b1, void* ws, size_t ws_bytes, void* stream);
int64_t vgposp_pack_elems(int64_t r0, int64_t r1, int64_t c0, int64_t c1, int lower);
int vgposp_pack_rows(double* A, int64_t lda, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                     int lower, double* buf, int unpack, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Left-side triangular solve with a factor from vgposp_potrf_lower(invert = 0), in place on B:
 *   trans = 0:  B (n x nrhs, ldb) <- L^-1 B        trans = 1:  B <- L^-T B
 * Replaces tf.linalg.triangular_solve(L, ...) inside tfd.GaussianProcess.log_prob and the
 * GPRM posterior (gp_functions.py:166-172, 283-297; SURVEY §8(b) vgposp_trsm_lower).  The
 * strictly upper triangle of L is never read.  ws: vgposp_trsm_workspace_bytes(n, nrhs).
 * --------------------------------------------------------------------------------------------- */
size_t vgposp_trsm_workspace_bytes(int64_t n, int64_t nrhs);
int vgposp_trsm_lower(const double* L, int64_t n, int64_t ldl, int trans, double* B, int64_t nrhs,
                      int64_t ldb, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * GP log marginal likelihood from the inverted factor.  Replaces
 * tfd.GaussianProcess(...).log_prob(y) (gp_functions.py:166-172, main.py:105):
 *     z = Minv y,   out[b] = -0.5 |z|^2 - sum_i log Ldiag[b][i] - n/2 log(2 pi)
 * Minv: output of vgposp_potrf_lower(invert=1); Ldiag: its diag_out; y: [n] (shared over batch).
 * alpha ([batch][n] or NULL) <- C^-1 y = Minv^T z.  ws: vgposp_lml_workspace_bytes(n, batch).
 * --------------------------------------------------------------------------------------------- */
size_t vgposp_lml_workspace_bytes(int64_t n, int batch);
int vgposp_lml(const double* Minv, int64_t n, int64_t lda, int64_t stride, int batch,
               const double* Ldiag, const double* y, double* alpha, double* out, void* ws,
               size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Gradient of the LML w.r.t. (amp[b], ls[b], noise) for the kernel family `kind`:
 *     dLML/dtheta = 0.5 * sum_ij (alpha alpha^T - C^-1)_ij dC_ij/dtheta
 * Cinv: the full C^-1 (lower triangle suffices; formed by vgposp_gemm(transa=1, tri) from Minv).
 * grad: [batch][3] = (d/damp, d/dls, d/dnoise).  Replaces TF autodiff of
 * tf_train_gp_adam's loss (gp_functions.py:179-182).
 * --------------------------------------------------------------------------------------------- */
size_t vgposp_lml_grad_workspace_bytes(int64_t n, int batch);
int vgposp_lml_grad(int kind, const double* X, int64_t n, int d, const double* amp,
                    const double* ls, const double* Cinv, int64_t ldc, int64_t stride_c,
                    const double* alpha, int batch, double* grad, void* ws, size_t ws_bytes,
                    void* stream);

/* ---------------------------------------------------------------------------------------------
 * Greedy mutual-information placement (Krause, Singh & Guestrin Alg. 2 as implemented by
 * placement_algorithm2.placement_algorithm_2, placement_algorithm2.py:151-219; lazy = 0 gives
 * placement_algorithm_1, :128-145).  Same selections: delta_y = nom/denom with
 *   nom   = sigma_yy - Sigma_yA Sigma_AA^-1 Sigma_Ay                    (nominator, :371-388)
 *   denom = conditional variance of y given V \ (A u {y})               (denominator, :408-413)
 * zeroed when |nom| < 1e-8 or |denom| < 1e-8 (:198); the lazy cache starts at +inf and every
 * round re-scores the stale arg-max until the arg-max is fresh (:173-208); ties -> lowest index.
 *
 * Sigma: n x n row-major covariance (cov_vv) on device, lda >= n.  vgposp_greedy_init factors it
 * IN PLACE (lower triangle <- L^-1, diagonal saved in ws; the strictly upper triangle must hold
 * Sigma and is kept).  vgposp_greedy_step performs one selection round (round = 0, 1, ...).
 * selected: int64 [kmax] device; sel_delta: f64 [kmax] device (delta of each pick) or NULL;
 * info: int32 device (Cholesky status of init).  evals: int64 [kmax] device or NULL (number of
 * delta evaluations the reference would have made in each round).
 * --------------------------------------------------------------------------------------------- */
size_t vgposp_greedy_workspace_bytes(int64_t n, int kmax);
int vgposp_greedy_init(double* Sigma, int64_t n, int64_t lda, int kmax, int* info, void* ws,
                       size_t ws_bytes, void* stream);
int vgposp_greedy_step(const double* Sigma, int64_t n, int64_t lda, int kmax, int round, int lazy,
                       int64_t* selected, double* sel_delta, int64_t* evals, void* ws,
                       size_t ws_bytes, void* stream);

/* The TF-graph variant snippets_a2.sparse_placement_algorithm_2 (snippets_a2.py:679-822, with
 * tf_nominator :138-213 and placement_algorithm2.sparse_argmax_cache_linear :24-50) differs only in
 * three constants, which vgposp_greedy_init_ex stores in the workspace for the later rounds:
 *   jitter      eps added to the diagonal of Sigma_AA and of Sigma_AbarAbar (snippets_a2.py:161-163:
 *               1e-6; 0 for placement_algorithm_2).  The factorization is of Sigma + eps I and
 *               denom_y = 1 / [(Sigma_SS + eps I)^-1]_yy - eps.
 *   threshold   |nom| or |denom| < threshold -> delta = 0 (:480: 1e-7; 1e-8 for alg. 2)
 *   cache_init  initial lazy-cache value (:690: INF = 1e8; +inf for alg. 2)
 * vgposp_greedy_init(...) == vgposp_greedy_init_ex(..., 0, 1e-8, +inf, ...).
 * After a failed pivot every later launch of init's factorization and inverse reads `info` on
 * the device and exits: a singular Sigma costs the factorization up to the failed pivot, not a
 * whole factor + inverse, before the caller's jitter retry (placement_algorithm2.py:399-413's
 * pinv has no failure mode) — without any host synchronisation, so init can be captured into a
 * graph.  Sigma and the workspace are then undefined, as after any failed factorization.
 * vgposp_greedy_cache returns the device pointer of the lazy cache [n] (delta_cached): the
 * per-round snapshot delta_cached_iters[:, r] of the TF variant is a copy of it after round r. */
int vgposp_greedy_init_ex(double* Sigma, int64_t n, int64_t lda, int kmax, double jitter,
                          double threshold, double cache_init, int* info, void* ws,
                          size_t ws_bytes, void* stream);
int vgposp_greedy_cache(void* ws, int64_t n, int kmax, double** cache);
/* Mark candidate idx as never selectable (after init: it is never scored, never an arg-max,
 * never counted in evals).  placement_algorithm2 factors an odd-order cov_vv as
 * [Sigma 0; 0 s] at the even order n + 1 (the fast GEMM needs even leading dimensions; the leading
 * block's factor and inverse are unchanged and the padding couples to nothing) and excludes the
 * padding candidate with this. */
int vgposp_greedy_exclude(void* ws, int64_t n, int kmax, int64_t idx, void* stream);

/* Placement algorithm 3, the local-kernel greedy (snippets_a3.sparse_placement_algorithm_3,
 * snippets_a3.py:43-330; with vgposp_greedy_init_ex(..., 1e-6, 1e-7, 1e8, ...) as its tf_nominator
 * constants).  Per round, after vgposp_greedy_update(round): round 0 scores every candidate into
 * the cache; round r >= 1 refreshes the cache only for candidates in the index window
 * [i_d - cutoff, i_d + cutoff) (per grid axis d, clipped, upper bound exclusive) around the
 * previous pick y* = selected[r-1] of the I0 x I1 x I2 C-order grid (candidates in A -> 0,
 * cache[y*] = 0); entries outside the window keep their stale values.  Then selects the arg-max of
 * the cache over the unselected candidates (lowest index on ties).  sel_delta[r] = cache[y];
 * evals[r] = entries scored this round. */
int vgposp_greedy_select_window(int64_t n, int kmax, int round, int64_t I0, int64_t I1, int64_t I2,
                                int cutoff, int64_t c0, int64_t c1, int64_t* selected,
                                double* sel_delta, int64_t* evals, void* ws, size_t ws_bytes,
                                void* stream);

/* The two phases of vgposp_greedy_step, for candidate-sharded multi-GPU placement:
 * every rank holds the factored Sigma (replicated init) and owns the candidate slab [c0, c1).
 *   vgposp_greedy_update: rank-1 updates of nom / P_yy and fresh deltas for y in [c0, c1) only
 *                         (the triangular mat-vec reads only the slab's columns of L^-1).
 *   -> caller all-gathers the delta slabs into the full delta vector (vgposp_greedy_buffers)
 *   vgposp_greedy_select: lazy-cache emulation over ALL candidates (identical on every rank) and
 *                         the pivot row of the pick, written only by the rank whose slab owns it
 *                         (zeros elsewhere)
 *   -> caller sum-all-reduces the pivot buffer (2 + 2*kmax doubles) before the next update.
 * With c0 = 0, c1 = n and no collectives this is exactly vgposp_greedy_step. */
int vgposp_greedy_update(const double* Sigma, int64_t n, int64_t lda, int kmax, int round,
                         int64_t c0, int64_t c1, const int64_t* selected, void* ws,
                         size_t ws_bytes, void* stream);
int vgposp_greedy_select(int64_t n, int kmax, int round, int lazy, int64_t c0, int64_t c1,
                         int64_t* selected, double* sel_delta, int64_t* evals, void* ws,
                         size_t ws_bytes, void* stream);
/* Partitioned inverse for one problem sharded over R ranks (the O(N^3) factorization is replicated,
 * the inverse is not): vgposp_greedy_init_slab factors Sigma like vgposp_greedy_init_ex but forms
 * L^-1 only in columns [c0, c1) (the rank's candidate slab; c0 and c1 multiples of 128 or c1 = n),
 * about 1/R of the inverse's flops; tmp: vgposp_greedy_slab_tmp_bytes(n, c0, c1) bytes.  Per round
 * the owner of the last pick's column then provides it: vgposp_greedy_extract writes xcol = that
 * column of L^-1 if the pick is in [own0, own1) and zeros otherwise, the caller sum-all-reduces
 * xcol (vgposp_greedy_xcol gives its device address) and runs vgposp_greedy_update_ex with
 * extract = 0.  vgposp_greedy_update(...) == vgposp_greedy_update_ex(..., extract = 1, ...). */
size_t vgposp_greedy_slab_tmp_bytes(int64_t n, int64_t c0, int64_t c1);
int vgposp_greedy_init_slab(double* Sigma, int64_t n, int64_t lda, int kmax, double jitter,
                            double threshold, double cache_init, int64_t c0, int64_t c1,
                            double* tmp, size_t tmp_bytes, int* info, void* ws, size_t ws_bytes,
                            void* stream);
/* vgposp_greedy_init_slab in phases, for a factorization the caller runs itself (the distributed
 * Cholesky above): vgposp_greedy_prepare (saves diag(Sigma), jitter, cache init, info = 0), then the
 * lower factor of Sigma in place with the potrf workspace vgposp_greedy_fact_ws returns, then
 * vgposp_greedy_finish_slab (L^-1 in columns [c0, c1) and their column norms). */
int vgposp_greedy_prepare(double* Sigma, int64_t n, int64_t lda, int kmax, double jitter,
                          double threshold, double cache_init, int* info, void* ws,
                          size_t ws_bytes, void* stream);
int vgposp_greedy_fact_ws(void* ws, int64_t n, int kmax, void** fws, size_t* fws_bytes);
int vgposp_greedy_finish_slab(double* Sigma, int64_t n, int64_t lda, int kmax, int64_t c0,
                              int64_t c1, double* tmp, size_t tmp_bytes, void* ws,
                              size_t ws_bytes, void* stream);
int vgposp_greedy_extract(const double* Sigma, int64_t n, int64_t lda, int kmax, int round,
                          int64_t own0, int64_t own1, const int64_t* selected, void* ws,
                          size_t ws_bytes, void* stream);
int vgposp_greedy_update_ex(const double* Sigma, int64_t n, int64_t lda, int kmax, int round,
                            int64_t c0, int64_t c1, const int64_t* selected, int extract, void* ws,
                            size_t ws_bytes, void* stream);
int vgposp_greedy_xcol(void* ws, int64_t n, int kmax, double** xcol);
/* Device pointers into the workspace: the full delta vector [n] and the pivot buffer. */
int vgposp_greedy_buffers(void* ws, int64_t n, int kmax, double** delta, double** piv,
                          int64_t* piv_len);

/* ---------------------------------------------------------------------------------------------
 * Exact algorithm 3 at grid sizes where cov_vv cannot be dense (config C4, 128^3): the beta-decay
 * tapered covariance (main_architecture_2_sampledistribution.py:355-421) is a sparse SPD stencil
 * matrix, and snippets_a3.sparse_placement_algorithm_3 (snippets_a3.py:43-364) with tf_nominator /
 * tf_denominator (snippets_a2.py:138-218) over the FULL sets A and V \ (A u {y}) needs
 *   round 0:  denom_y = 1 / Q_yy - eps,  Q = (Sigma + eps I)^-1   (every candidate)
 *   round t:  denom_y = 1 / (Q_yy - Q_yA Q_AA^-1 Q_Ay) - eps,
 *             nom_y   = s_yy - s_yA (Sigma_AA + eps I)^-1 s_Ay        (the window re-score)
 * diag(Q) comes from a nested-dissection multifrontal Cholesky and its selected inverse (the
 * symbolic plan is host-side, vgposp_amd/nested_dissection.py).  A front = pivots P + boundary U,
 * stored as row-major blocks PP [p][p] (lower), UP [u][p], UU [u][u]; a group of nf fronts of one
 * tree level is a strided batch (strides p*p, u*p, u*u).  p and u even (padded by the plan).
 *   vgposp_front_assemble:   original entries of the pivot columns into zeroed PP / UP:
 *       s(i, j) = tau[|i - j|^2] (K(x_i, x_j) + diag_shift [i == j]) + jitter [i == j]
 *     (the taper arguments as VGPOSP_LOCAL_ARGS); owner_ord / owner_pos [N]: post-order id of the
 *     front eliminating each node and its pivot position; piv [nf][p] (-1 = padding: identity);
 *     U [nf][u] ascending, ulen [nf]; order [nf]: the fronts' post-order ids.
 *   vgposp_front_extend_add: parent front += the lower triangle of each child's update UUc
 *     ([nfc][uc][uc]) at positions pmap [nfc][uc] (-1 = padding) of its parent front, which sits
 *     at element offsets par_off [nfc][3] of the parent level's PP / UP / UU buffers with padded
 *     sizes par_dim [nfc][2] = (p, u); only children with sibling[c] == sib (call once per
 *     sibling index: siblings share a parent).
 *   vgposp_front_factor:     per front, PP <- M = L^-1 (F_PP = L L^T), UU -= L_UP L_UP^T with
 *     L_UP = F_UP M^T, UP <- W = L_UP M.  info [nf] (potrf convention).  ws:
 *     vgposp_front_factor_workspace_bytes(p, u, nf).
 *   vgposp_front_gather:     child's full Q_UU [nfc][uc][uc] <- its parent's Q front (QPP lower,
 *     QUP, QUU full; the parent level's buffers, par_off / par_dim as above) at
 *     (pmap[a], pmap[b]); 0 on padding.
 *   vgposp_front_selinv:     QPP <- M^T M - W^T T (lower), QUP <- T = -QUU W (out of place).
 *   vgposp_front_diag:       out[piv[f][k]] <- QPP[f][k][k] for piv >= 0.
 * --------------------------------------------------------------------------------------------- */
size_t vgposp_front_factor_workspace_bytes(int64_t p, int64_t u, int nf);
int vgposp_front_assemble(int kind, const double* X, int64_t I0, int64_t I1, int64_t I2,
                          double amp, double ls, double diag_shift, double jitter,
                          const int* offsets, int m, const double* tau, int ntau,
                          const int* owner_ord, const int* owner_pos, const int* piv, int64_t p,
                          const int* U, int64_t u, const int* ulen, const int* order, int nf,
                          double* PP, double* UP, void* stream);
int vgposp_front_extend_add(const double* UUc, int64_t uc, int nfc, const int* pmap,
                            const int64_t* par_off, const int* par_dim, const int* sibling, int sib,
                            double* PP, double* UP, double* UU, void* stream);
int vgposp_front_factor(double* PP, double* UP, double* UU, int64_t p, int64_t u, int nf,
                        int* info, void* ws, size_t ws_bytes, void* stream);
int vgposp_front_gather(const double* QPP, const double* QUP, const double* QUU,
                        const int* pmap, const int64_t* par_off, const int* par_dim, int nfc,
                        int64_t uc, double* QUUc, void* stream);
int vgposp_front_selinv(const double* M, const double* W, const double* QUU, int64_t p, int64_t u,
                        int nf, double* QPP, double* QUP, void* stream);
int vgposp_front_diag(const double* QPP, int64_t p, int nf, const int* piv, double* out,
                      void* stream);

/* The rounds of exact algorithm 3 on the tapered covariance (taper arguments as above; kmax <= 128;
 * cutoff: the window [i_d - cutoff, i_d + cutoff) of snippets_a3.py:190-303; threshold: |nom| or
 * |denom| below -> delta 0, snippets_a2.py:480; radius: the stencil radius (largest offset
 * component); cg_iters: conjugate-gradient iterations per column).  qdiag [N]:
 * diag((Sigma + jitter I)^-1) from the front_* calls, or upper bounds of it from
 * vgposp_exact_bounds; cache [N] f64 (delta_cached), selected [N] uint8, both caller-owned.
 *
 * Selected-inverse form (qdiag exact):
 *   vgposp_exact_prepare(flags = 0): the stencil coefficients, round 0 (every candidate:
 *     nom = s_yy, denom = 1 / Q_yy - jitter) and the arg-max keys; clears `selected`.
 *   vgposp_exact_round:   pick `round` = the arg-max of the cache over V \ A (lowest index on ties),
 *     picks[round] / pick_delta[round]; unless `last`: q = Q e_pick by cg_iters CG iterations on
 *     Sigma + jitter I (stopping early once |r| <= cg_tol) on the box of half-width
 *     radius * cg_iters around the pick (the Krylov vectors are exactly zero beyond it), the next
 *     rows of chol(Q_AA) and chol(Sigma_AA + jitter I), and the window re-score
 *       nom = s_yy - |LS^-1 s_Ay|^2,  denom = 1 / (Q_yy - |LQ^-1 q_Ay|^2) - jitter.
 *
 * Bounded-lazy form (no selected inverse; same picks):
 *   vgposp_exact_coef:    the stencil coefficients and Gershgorin bounds [lambda_min, lambda_max]
 *     of Sigma + jitter I (device doubles, vgposp_exact_buffers' `gersh`).
 *   vgposp_exact_bounds:  qdiag[y] for y in [c0, c1) <- an upper bound of e_y^T (Sigma + jitter I)^-1
 *     e_y from K CG steps from x = 0: with mu = 0, hi_scale * g_K (g_K = the CG estimate, a
 *     lower bound; hi_scale = (1 + margin) / (1 - 4 rho^2K)); with 0 < mu <= lambda_min, the
 *     Gauss-Radau bound hi_scale * (g_K + gamma^mu_K |r_K|^2) (hi_scale = 1 + margin; the
 *     recurrence is in exact_greedy.hip).  tab_off int [T][3]: the offsets
 *     within K stencil steps, sorted by step count (offset 0 first); tab_cnt int [K + 1]: offsets
 *     within d steps; tab_nb int [T][m - 1]: row of (offset + offsets[o]) in the table or -1.
 *     T <= 1024, T (m - 1) <= 8192.
 *   vgposp_exact_prepare(flags = 1): round 0 from those bounds (cache = upper bounds); flags = 3:
 *     the same, the bounds being the first of two levels (vgposp_exact_tighten_pending).
 *   vgposp_exact_steps_reset: clears the rounds' control block (after prepare, before the rounds).
 *   vgposp_exact_steps:   rounds [round0, round1) of a run of k picks, decided on the device.
 *     Each round is two kernels: the first refreshes the arg-max keys of the previous round's
 *     window, takes the arg-max of the cache over V \ A (lowest index on ties) and either picks
 *     it (its Q_yy exact, its column in a slot: picks[round] / pick_delta[round], the pick's rows
 *     of chol(Q_AA) and chol(Sigma_AA + jitter I)) or STALLS: the control block records the round
 *     and the refinement
 *     batch: every later kernel of the issued rounds then does nothing.  The second re-scores the
 *     window of the pick (upper bounds where Q_yy is still only bounded).  After the rounds one
 *     kernel chooses the batch of a stalled round: of the `batch` <= 32 best entries without a
 *     column, those still on their first (K_lo-step) bound go to the TIGHTENING list, the others
 *     and the arg-max to the CG batch, each given a free column slot or the oldest unpinned one.
 *   vgposp_exact_tighten_pending: the tightening list's bounds again with the K_hi-step table
 *     (arguments as vgposp_exact_bounds; the smaller of the two bounds is kept), the candidates'
 *     cache entries re-scored; clears the stall when the CG batch is empty.  m = 7 only.
 *   vgposp_exact_pretighten: after prepare(flags = 3) and steps_reset, before the rounds: the
 *     M <= 32,768 candidates with the largest round-0 entries (a radix select of the M-th largest
 *     key; ties at the threshold included; if that lists more than 65,536, none) get the K_hi-step
 *     bounds at once
 *     (arguments as vgposp_exact_bounds), their entries re-scored and the arg-max keys rebuilt;
 *     the count is added to the control block's tightened total.  m = 7 only.
 *   vgposp_exact_refine_pending: Q e_c for the pending CG batch by one batched CG (columns into
 *     their slots); each Q_cc becomes exact and the candidate's cache entry the reference's value
 *     (scored with the A of its last re-score); clears the stall.  After the tightening when both
 *     are pending.
 *   vgposp_exact_ctl:     device address of the control block, int32 [8]: stalled round (-1:
 *     none), CG batch size, refined-not-picked count, refinement batches, candidates refined,
 *     refinement counter, tightening list size, candidates tightened.
 *   vgposp_exact_update:  after pick `round`: the factor rows and the window re-score (upper
 *     bounds where Q_yy is still only bounded); vgposp_exact_steps issues it per round.
 *   The caller issues rounds, reads the control block, and on a stall refines the pending batch
 *   and re-issues the rounds from the stalled one: one host read per refinement batch (the B best
 *   entries are refined together, one batched CG, the launches of one column; the next rounds'
 *   picks are mostly among them).
 *
 *   vgposp_exact_buffers: device addresses of the column slots [2 kmax][b0 b1 b2] (box-local, C
 *     order, box dims b_d = min(2 radius cg_iters + 1, I_d)), their box origins int64
 *     [2 kmax][3], the CG state (int [2]: converged flag, iterations of the last solve), the
 *     column slot of every pick (int [kmax]), the arg-max candidate (int64) and the Gershgorin
 *     bounds (double [2]). */
#define VGPOSP_EXACT_ARGS                                                                         \
  int kind, const double *X, int64_t I0, int64_t I1, int64_t I2, double amp, double ls,          \
      double diag_shift, double jitter, double threshold, const int *offsets, int m,             \
      const double *tau, int ntau, int kmax, int cutoff, int radius, int cg_iters,               \
      const double *qdiag, double *cache, uint8_t *selected, void *ws, size_t ws_bytes
size_t vgposp_exact_workspace_bytes(int64_t I0, int64_t I1, int64_t I2, int m, int kmax, int radius,
                                    int cg_iters);
int vgposp_exact_prepare(VGPOSP_EXACT_ARGS, int flags, void* stream);
int vgposp_exact_round(VGPOSP_EXACT_ARGS, int round, int last, int64_t* picks, double* pick_delta,
                       double cg_tol, void* stream);
int vgposp_exact_coef(VGPOSP_EXACT_ARGS, void* stream);
int vgposp_exact_bounds(VGPOSP_EXACT_ARGS, const int* tab_off, const int* tab_nb,
                        const int* tab_cnt, int T, int K, double hi_scale, double mu, int64_t c0,
                        int64_t c1, void* stream);
int vgposp_exact_steps_reset(VGPOSP_EXACT_ARGS, void* stream);
int vgposp_exact_steps(VGPOSP_EXACT_ARGS, int round0, int round1, int k, int batch,
                       int64_t* picks, double* pick_delta, void* stream);
int vgposp_exact_refine_pending(VGPOSP_EXACT_ARGS, int batch, const int64_t* picks, double cg_tol,
                                void* stream);
int vgposp_exact_tighten_pending(VGPOSP_EXACT_ARGS, const int* tab_off, const int* tab_nb,
                                 const int* tab_cnt, int T, int K, double hi_scale, double mu,
                                 const int64_t* picks, void* stream);
int vgposp_exact_pretighten(VGPOSP_EXACT_ARGS, const int* tab_off, const int* tab_nb,
                            const int* tab_cnt, int T, int K, double hi_scale, double mu,
                            int64_t M, void* stream);
int vgposp_exact_ctl(void* ws, int64_t I0, int64_t I1, int64_t I2, int m, int kmax, int radius,
                     int cg_iters, int** ctl);
int vgposp_exact_update(VGPOSP_EXACT_ARGS, int round, const int64_t* picks, void* stream);
int vgposp_exact_buffers(void* ws, int64_t I0, int64_t I1, int64_t I2, int m, int kmax, int radius,
                         int cg_iters, double** qcols, int64_t** boxlo, int** cgstate,
                         int** slot_of_round, int64_t** cand, double** gersh);

/* ---------------------------------------------------------------------------------------------
 * TF1 AdamOptimizer step on a device parameter vector (tf.train.AdamOptimizer in
 * gp_functions.tf_train_gp_adam, gp_functions.py:179-182; variational_Gaussian_process_example.py
 * :101-102).  g = grad_scale * grad (grad_scale = -1 maximises);  t = *step + 1 (device int64,
 * incremented):  lr_t = lr sqrt(1 - b2^t) / (1 - b1^t);  m = b1 m + (1-b1) g;
 * v = b2 v + (1-b2) g^2;  theta -= lr_t m / (sqrt(v) + eps).
 * --------------------------------------------------------------------------------------------- */
int vgposp_adam_update(double* theta, const double* grad, double* m, double* v, int64_t n,
                       double lr, double beta1, double beta2, double eps, int64_t* step,
                       double grad_scale, void* stream);

/* Softplus-constrained parameters (the reference's `softplus(var)` / `1e-5 + softplus(var)`
 * kernel amplitude, length scale and noise, variational_Gaussian_process_example.py:47-61;
 * gp_functions.py:131-134) whose unconstrained vars live in theta:
 *   vgposp_softplus_values:       out[k] = offsets[k] + softplus(theta[slots[k]]), nparam <= 4;
 *   vgposp_adam_update_softplus:  vgposp_adam_update where the gradient of theta[slots[k]] is
 *                                 *gsrc[k] * sigmoid(theta[slots[k]]) (gsrc: nparam device
 *                                 pointers; the chain rule through the softplus; grad[slots[k]]
 *                                 is not read).
 * One launch each instead of a few elementwise launches per parameter. */
int vgposp_softplus_values(const double* theta, int64_t n, int nparam, const int* slots,
                           const double* offsets, double* out, void* stream);
int vgposp_adam_update_softplus(double* theta, const double* grad, double* m, double* v,
                                int64_t n, double lr, double beta1, double beta2, double eps,
                                int64_t* step, double grad_scale, int nparam, const int* slots,
                                const double* const* gsrc, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Optional per-launch timing (no reference counterpart; the reference times with wall clocks,
 * placement_algorithm2.py:416-430).  When enabled, every launch of the library's named kernels
 * ("gemm_f64", "potrf_diag", "kernel_matrix", "greedy_trmv", "greedy_update", "greedy_select",
 * ...) is bracketed by a hipEvent pair on its stream together with its algorithmic flops and
 * bytes.  vgposp_prof_query synchronises on the recorded events and sums them per kernel name.
 * Enabling (or re-enabling) clears the records.  Host-side state, guarded by a mutex.
 * --------------------------------------------------------------------------------------------- */
int vgposp_prof_enable(int on);
int vgposp_prof_query(const char* name, double* total_ms, int64_t* launches, double* flops,
                      double* bytes);
/* Text summary of all records: one "name<TAB>ms<TAB>launches<TAB>flops<TAB>bytes" line per
 * distinct kernel name.  Returns the size needed (with the NUL); buf may be NULL. */
int64_t vgposp_prof_dump(char* buf, size_t len);

#ifdef __cplusplus
}
#endif

#endif /* VGPOSP_H_ */
