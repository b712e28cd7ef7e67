// Blocked right-looking Cholesky (lower, in place) with an optional fused block Gauss-Jordan
// inversion, so that one sweep leaves L^-1 in the lower triangle:
//
//   for each 128-wide block column j:
//     (a) diag kernel: L_jj = chol(A_jj) and Linv_jj = L_jj^-1 in LDS (one workgroup)
//     (b) panel       L_21 = A_21 Linv_jj^T                 [MFMA GEMM, in place]
//     (c) trailing    A_22 -= L_21 L_21^T  (lower)          [MFMA GEMM]
//   and, when inverting (R = the rows of L^-1 built so far):
//     (d) row scale   R_j,<j = Linv_jj R_j,<j               [MFMA GEMM, in place]
//     (e) GJ update   R_>j,<j -= L_21 R_j,<j                [MFMA GEMM]
//     (f) GJ column   R_>j,j = -L_21 Linv_jj                [MFMA GEMM, in place]
//
// Replaces the Eigen LLT that tf.linalg.cholesky runs inside tfd.GaussianProcess.log_prob
// (gp_functions.py:166-172, main.py:105) and the per-candidate SVD pinv of
// placement_algorithm2.denominator (placement_algorithm2.py:399-413).
// The strictly upper triangle is never read or written.
#include "common.h"

namespace vgposp {

int gemm_launch(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, hipStream_t stream);

constexpr int NB = 128;        // block column width (== GEMM tile, so (b),(d),(f) are in place)
constexpr int DP = NB + 1;     // LDS pitch of the diagonal block (conflict-free column walks)
constexpr int DIAG_THREADS = 1024;

// Factor the jb x jb diagonal block at A (lower), write
//   A_jj lower <- L (invert == 0) or L^-1 (invert == 1),
//   linv (NB x NB, zero above the diagonal) <- L^-1,
//   diag_out[c] <- L[c][c],  info <- first failing global column + 1.
__global__ __launch_bounds__(DIAG_THREADS) void potrf_diag_kernel(double* A, int64_t lda, int jb,
                                                                  int64_t col0, int invert,
                                                                  double* linv, double* diag_out,
                                                                  int* info) {
  extern __shared__ double L[];  // [NB][DP]; X (the inverse) lives transposed in the upper part
  __shared__ double xdiag[NB];
  __shared__ int bad;
  const int t = threadIdx.x;
  if (t == 0) bad = 0;
  for (int e = t; e < jb * jb; e += DIAG_THREADS) {
    const int r = e / jb, c = e % jb;
    if (c <= r) L[r * DP + c] = A[(int64_t)r * lda + c];
  }
  __syncthreads();

  // Unblocked right-looking Cholesky in LDS.
  for (int c = 0; c < jb; ++c) {
    const double d = L[c * DP + c];
    if (!(d > 0.0)) {
      if (t == 0 && bad == 0) {
        bad = 1;
        if (*info == 0) *info = (int)(col0 + c + 1);
      }
    }
    const double piv = sqrt(d);
    const double inv = 1.0 / piv;
    __syncthreads();
    for (int r = c + 1 + t; r < jb; r += DIAG_THREADS) L[r * DP + c] *= inv;
    if (t == 0) L[c * DP + c] = piv;
    __syncthreads();
    const int m = jb - c - 1;
    // rank-1 update of the trailing lower triangle, (r, s) with c < s <= r
    for (int e = t; e < m * m; e += DIAG_THREADS) {
      const int r = c + 1 + e / m, s = c + 1 + e % m;
      if (s <= r) L[r * DP + s] -= L[r * DP + c] * L[s * DP + c];
    }
    __syncthreads();
  }

  // Triangular inverse X = L^-1, column c by a group of 8 lanes:
  //   X[c][c] = 1/L[c][c];  X[r][c] = -(sum_{t=c}^{r-1} L[r][t] X[t][c]) / L[r][r]
  // X[r][c] (r > c) is kept at L[c][r] (upper part), X[c][c] in xdiag.
  {
    const int c = t >> 3, g = t & 7;
    if (c < jb) {
      const double xcc = 1.0 / L[c * DP + c];
      if (g == 0) xdiag[c] = xcc;
      for (int r = c + 1; r < jb; ++r) {
        double s = 0.0;
        for (int tt = c + g; tt < r; tt += 8) {
          const double x = (tt == c) ? xcc : L[c * DP + tt];
          s += L[r * DP + tt] * x;
        }
        s += __shfl_xor(s, 1, 8);
        s += __shfl_xor(s, 2, 8);
        s += __shfl_xor(s, 4, 8);
        const double xr = -s / L[r * DP + r];
        if (g == 0) L[c * DP + r] = xr;
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  __syncthreads();

  for (int e = t; e < NB * NB; e += DIAG_THREADS) {
    const int r = e / NB, c = e % NB;
    double x = 0.0;
    if (r < jb && c < jb && c <= r) x = (r == c) ? xdiag[c] : L[c * DP + r];
    linv[e] = x;
    if (r < jb && c <= r) {
      A[(int64_t)r * lda + c] = invert ? x : L[r * DP + c];
    }
  }
  if (diag_out != nullptr) {
    for (int c = t; c < jb; c += DIAG_THREADS) diag_out[c] = L[c * DP + c];
  }
}

int potrf_one(double* A, int64_t n, int64_t lda, int invert, double* diag_out, int* info,
              double* linv, hipStream_t stream) {
  const size_t shmem = (size_t)NB * DP * sizeof(double);
  static bool attr_set = false;
  if (!attr_set) {
    VG_HIP(hipFuncSetAttribute((const void*)potrf_diag_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
    attr_set = true;
  }
  for (int64_t j0 = 0; j0 < n; j0 += NB) {
    const int jb = (int)(n - j0 < NB ? n - j0 : NB);
    const int64_t j1 = j0 + jb, m = n - j1;
    double* Ajj = A + j0 * lda + j0;
    {
      ProfScope ps("potrf_diag", stream, 2.0 * jb * (double)jb * jb / 3.0, 8.0 * jb * (double)jb * 2);
      hipLaunchKernelGGL(potrf_diag_kernel, dim3(1), dim3(DIAG_THREADS), shmem, stream, Ajj, lda,
                         jb, j0, invert, linv, diag_out ? diag_out + j0 : nullptr, info);
      VG_LAUNCH_CHECK();
    }
    double* A21 = A + j1 * lda + j0;
    int rc;
    if (m > 0) {
      // (b) L21 = A21 Linv^T   (in place: one 128-wide column tile)
      if ((rc = gemm_launch(0, 1, m, jb, jb, 1.0, A21, lda, linv, NB, 0.0, A21, lda, VGPOSP_FULL, 0,
                            0, stream)))
        return rc;
      // (c) A22 -= L21 L21^T  (lower)
      if ((rc = gemm_launch(0, 1, m, m, jb, -1.0, A21, lda, A21, lda, 1.0, A + j1 * lda + j1, lda,
                            VGPOSP_LOWER, 0, 0, stream)))
        return rc;
    }
    if (invert) {
      double* Rj = A + j0 * lda;  // row block j, columns [0, j0)
      if (j0 > 0) {
        // (d) R_j,<j = Linv R_j,<j  (in place: one 128-high row tile)
        if ((rc = gemm_launch(0, 0, jb, j0, jb, 1.0, linv, NB, Rj, lda, 0.0, Rj, lda, VGPOSP_FULL,
                              0, 0, stream)))
          return rc;
      }
      if (m > 0) {
        if (j0 > 0) {
          // (e) R_>j,<j -= L21 R_j,<j
          if ((rc = gemm_launch(0, 0, m, j0, jb, -1.0, A21, lda, Rj, lda, 1.0, A + j1 * lda, lda,
                                VGPOSP_FULL, 0, 0, stream)))
            return rc;
        }
        // (f) R_>j,j = -L21 Linv  (in place)
        if ((rc = gemm_launch(0, 0, m, jb, jb, -1.0, A21, lda, linv, NB, 0.0, A21, lda, VGPOSP_FULL,
                              0, 0, stream)))
          return rc;
      }
    }
  }
  return 0;
}

size_t potrf_ws_bytes() { return (size_t)NB * NB * sizeof(double); }

}  // namespace vgposp

extern "C" size_t vgposp_potrf_workspace_bytes(int64_t n) {
  (void)n;
  return vgposp::potrf_ws_bytes();
}

extern "C" int vgposp_potrf_lower(double* A, int64_t n, int64_t lda, int64_t stride, int batch,
                                  int invert, double* diag_out, int* info, void* ws,
                                  size_t ws_bytes, void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(A != nullptr || n == 0, 1);
  VG_CHECK_ARG(n >= 0, 2);
  VG_CHECK_ARG(lda >= (n > 0 ? n : 1), 3);
  VG_CHECK_ARG(batch >= 1, 5);
  VG_CHECK_ARG(batch == 1 || stride >= lda * n, 4);
  VG_CHECK_ARG(info != nullptr, 8);
  VG_CHECK_ARG(ws != nullptr, 9);
  if (ws_bytes < potrf_ws_bytes()) {
    set_error("vgposp_potrf_lower: workspace %zu < %zu bytes", ws_bytes, potrf_ws_bytes());
    return VGPOSP_E_WS;
  }
  hipStream_t s = as_stream(stream);
  VG_HIP(hipMemsetAsync(info, 0, sizeof(int) * batch, s));
  for (int b = 0; b < batch; ++b) {
    int rc = potrf_one(A + b * stride, n, lda, invert, diag_out ? diag_out + (int64_t)b * n : nullptr,
                       info + b, static_cast<double*>(ws), s);
    if (rc) return rc;
  }
  return 0;
}
