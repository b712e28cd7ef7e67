// Recursive Cholesky (lower, in place) and recursive triangular inverse, built so that nearly all
// flops land in large-K fp64 MFMA GEMMs (gemm.hip):
//
//   potrf_rec(A):  L11 = potrf_rec(A11)
//                  A21 <- A21 L11^-T           trsm_rec: leaves multiply by the saved 128x128
//                                              diagonal-block inverses, inner steps are GEMMs
//                  A22 -= A21 A21^T (lower)    SYRK with K = n1 ~ n/2
//                  L22 = potrf_rec(A22)
//   trtri_rec(L):  X11 = trtri_rec(L11), X22 = trtri_rec(L22)
//                  W   = L21 X11               TRMM (X11 lower)        K = n1
//                  X21 = -X22 W                TRMM (X22 lower)        K = n2
// Leaves (<= 128) are factored and inverted in LDS by one workgroup (potrf_diag_kernel); their
// inverses are kept in the workspace for the trsm leaves and the trtri leaves.
//
// Replaces the Eigen LLT that tf.linalg.cholesky runs inside tfd.GaussianProcess.log_prob
// (gp_functions.py:166-172, main.py:105) and, through L^-1, the per-candidate SVD pinv of
// placement_algorithm2.denominator (placement_algorithm2.py:399-413).
// The strictly upper triangle is never read or written.
#include "common.h"

namespace vgposp {

int gemm_launch(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, hipStream_t stream);

constexpr int NB = 128;        // leaf size (== GEMM tile, so trsm leaves are in place)

#ifdef VGPOSP_STAMPS
__device__ long long g_stamps[8];
#define STAMP(i) \
  if (threadIdx.x == 0) g_stamps[i] = (long long)__builtin_amdgcn_s_memtime()
#else
#define STAMP(i)
#endif

// Factor and invert the jb x jb diagonal block at A (lower) in LDS, one workgroup:
//   A_jj lower <- L (invert == 0) or L^-1 (invert == 1),
//   linv (NB x NB, zero above the diagonal) <- L^-1,
//   diag_out[c] <- L[c][c],  info <- first failing global column + 1.
constexpr int DP = NB + 1;  // LDS pitch (conflict-free column walks)
constexpr int DIAG_THREADS = 1024;

// Batched use (small matrices): workgroup b handles A + b * stride_a, info + b, diag_out + b * n
// (linv must then be null).
__global__ __launch_bounds__(DIAG_THREADS) void potrf_diag_kernel(double* A, int64_t lda, int jb,
                                                                  int64_t col0, int invert,
                                                                  double* linv, double* diag_out,
                                                                  int* info, int64_t stride_a = 0) {
  extern __shared__ double L[];  // [NB][DP]; X (the inverse) lives transposed in the upper part
  __shared__ double rdiag[NB];   // 1 / L[r][r]
  const int t = threadIdx.x;
  A += blockIdx.x * stride_a;
  info += blockIdx.x;
  if (diag_out) diag_out += (int64_t)blockIdx.x * jb;
  const int tx = t & 31, ty = t >> 5;
  for (int e = t; e < jb * jb; e += DIAG_THREADS) {
    const int r = e / jb, c = e % jb;
    if (c <= r) L[r * DP + c] = A[(int64_t)r * lda + c];
  }
  __syncthreads();
  STAMP(0);

  // Unblocked right-looking Cholesky; the trailing update walks a 32x32 thread grid (no integer
  // division), each thread keeping its column multiplier of the step in a register.
  for (int c = 0; c < jb; ++c) {
    const double d = L[c * DP + c];
    const double piv = sqrt(d);
    const double inv = 1.0 / piv;
    if (t == 0) {
      if (!(d > 0.0)) atomicCAS(info, 0, (int)(col0 + c + 1));  // first failure
      rdiag[c] = inv;
    }
    __syncthreads();
    for (int r = c + 1 + t; r < jb; r += DIAG_THREADS) L[r * DP + c] *= inv;
    if (t == 0) L[c * DP + c] = piv;
    __syncthreads();
    for (int r = c + 1 + ty; r < jb; r += 32) {
      const double lr = L[r * DP + c];
      for (int s2 = c + 1 + tx; s2 <= r; s2 += 32) L[r * DP + s2] -= lr * L[s2 * DP + c];
    }
    __syncthreads();
  }
  STAMP(1);

  // Triangular inverse X = L^-1, column c by a group of 8 lanes:
  //   X[c][c] = 1/L[c][c];  X[r][c] = -(sum_{k=c}^{r-1} L[r][k] X[k][c]) / L[r][r]
  // X[r][c] (r > c) is kept at L[c][r] (upper part), X[c][c] at L[c][c] after the copy-out of L
  // (diag(L) is saved first).  Four independent partial sums keep the LDS reads in flight.
  {
    const int c = t >> 3, g = t & 7;
    if (c < jb) {
      const double xcc = rdiag[c];
      for (int r = c + 1; r < jb; ++r) {
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int k = c + g;
        for (; k + 24 < r; k += 32) {
          s0 += L[r * DP + k] * (k == c ? xcc : L[c * DP + k]);
          s1 += L[r * DP + k + 8] * L[c * DP + k + 8];
          s2 += L[r * DP + k + 16] * L[c * DP + k + 16];
          s3 += L[r * DP + k + 24] * L[c * DP + k + 24];
        }
        for (; k < r; k += 8) s0 += L[r * DP + k] * (k == c ? xcc : L[c * DP + k]);
        double s = (s0 + s1) + (s2 + s3);
        s += __shfl_xor(s, 1, 8);
        s += __shfl_xor(s, 2, 8);
        s += __shfl_xor(s, 4, 8);
        if (g == 0) L[c * DP + r] = -s * rdiag[r];
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  __syncthreads();
  STAMP(2);

  for (int e = t; e < NB * NB; e += DIAG_THREADS) {
    const int r = e / NB, c = e % NB;
    double x = 0.0;
    if (r < jb && c < jb && c <= r) x = (r == c) ? rdiag[c] : L[c * DP + r];
    if (linv) linv[e] = x;
    if (r < jb && c <= r) {
      A[(int64_t)r * lda + c] = invert ? x : L[r * DP + c];
    }
  }
  if (diag_out != nullptr) {
    for (int c = t; c < jb; c += DIAG_THREADS) diag_out[c] = L[c * DP + c];
  }
  STAMP(3);
}

// A (jb x jb lower) <- linv (the saved leaf inverse)
__global__ void copy_leaf_kernel(double* A, int64_t lda, int jb, const double* linv) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = e / NB, c = e % NB;
  if (r < jb && c <= r) A[(int64_t)r * lda + c] = linv[e];
}

static int64_t split_point(int64_t n) {
  const int64_t nb = (n + NB - 1) / NB;
  return NB * (nb / 2);  // >= NB for n > NB
}

struct Fact {
  int64_t lda;
  double* linv_all;  // ceil(n/NB) leaf inverses, NB*NB each, indexed by global column / NB
  double* work;      // trtri scratch, >= n1 * n2 doubles of the top split
  double* diag_out;  // [n] or null
  int* info;
  hipStream_t s;
  double* leaf(int64_t col0) const { return linv_all + (col0 / NB) * NB * NB; }
};

static size_t diag_shmem() { return (size_t)NB * DP * sizeof(double); }

static int leaf_factor(const Fact& f, double* A, int jb, int64_t col0, int invert) {
  ProfScope ps("potrf_diag", f.s, 2.0 * jb * (double)jb * jb / 3.0, 8.0 * jb * (double)jb * 2);
  hipLaunchKernelGGL(potrf_diag_kernel, dim3(1), dim3(DIAG_THREADS), diag_shmem(), f.s, A, f.lda,
                     jb, col0, invert, f.leaf(col0), f.diag_out ? f.diag_out + col0 : nullptr,
                     f.info);
  VG_LAUNCH_CHECK();
  return 0;
}

// B (m x nL, ldb) <- B L^-T, L = the nL x nL lower factor at Lp (already factored), col0 = global
// column of L's first column (locates the leaf inverses).
static int trsm_rec(const Fact& f, double* B, int64_t m, int64_t ldb, const double* Lp, int64_t nL,
                    int64_t col0) {
  int rc;
  if (nL <= NB) {
    // in place: the output is a single 128-wide column tile
    return gemm_launch(0, 1, m, nL, nL, 1.0, B, ldb, f.leaf(col0), NB, 0.0, B, ldb, VGPOSP_FULL, 0,
                       0, f.s);
  }
  const int64_t a = split_point(nL), b = nL - a;
  if ((rc = trsm_rec(f, B, m, ldb, Lp, a, col0))) return rc;
  // B2 -= B1 Lb^T,  Lb = L[a:, :a]
  if ((rc = gemm_launch(0, 1, m, b, a, -1.0, B, ldb, Lp + a * f.lda, f.lda, 1.0, B + a, ldb,
                        VGPOSP_FULL, 0, 0, f.s)))
    return rc;
  return trsm_rec(f, B + a, m, ldb, Lp + a * f.lda + a, b, col0 + a);
}

static int potrf_rec(const Fact& f, double* A, int64_t n, int64_t col0) {
  if (n <= NB) return leaf_factor(f, A, (int)n, col0, 0);
  const int64_t n1 = split_point(n), n2 = n - n1;
  int rc;
  double* A21 = A + n1 * f.lda;
  double* A22 = A21 + n1;
  if ((rc = potrf_rec(f, A, n1, col0))) return rc;
  if ((rc = trsm_rec(f, A21, n2, f.lda, A, n1, col0))) return rc;
  if ((rc = gemm_launch(0, 1, n2, n2, n1, -1.0, A21, f.lda, A21, f.lda, 1.0, A22, f.lda,
                        VGPOSP_LOWER, 0, 0, f.s)))
    return rc;
  return potrf_rec(f, A22, n2, col0 + n1);
}

// Lower triangle of A holds L (leaf inverses saved) -> L^-1.
static int trtri_rec(const Fact& f, double* A, int64_t n, int64_t col0) {
  if (n <= NB) {
    ProfScope ps("trtri_leaf", f.s, 0.0, 8.0 * NB * NB * 2);
    hipLaunchKernelGGL(copy_leaf_kernel, dim3(NB * NB / 256), dim3(256), 0, f.s, A, f.lda, (int)n,
                       f.leaf(col0));
    VG_LAUNCH_CHECK();
    return 0;
  }
  const int64_t n1 = split_point(n), n2 = n - n1;
  int rc;
  double* A21 = A + n1 * f.lda;
  double* A22 = A21 + n1;
  if ((rc = trtri_rec(f, A, n1, col0))) return rc;
  if ((rc = trtri_rec(f, A22, n2, col0 + n1))) return rc;
  // W = L21 X11   (X11 lower, stored [k][j])
  if ((rc = gemm_launch(0, 0, n2, n1, n1, 1.0, A21, f.lda, A, f.lda, 0.0, f.work, n1, VGPOSP_FULL,
                        0, 1, f.s)))
    return rc;
  // X21 = -X22 W  (X22 lower, stored [i][k])
  return gemm_launch(0, 0, n2, n1, n2, -1.0, A22, f.lda, f.work, n1, 0.0, A21, f.lda, VGPOSP_FULL,
                     1, 0, f.s);
}

size_t potrf_ws_bytes(int64_t n) {
  const int64_t leaves = (n + NB - 1) / NB;
  const int64_t n1 = n > NB ? split_point(n) : 0;
  return (size_t)(leaves * NB * NB + n1 * (n - n1) + 64) * sizeof(double);
}

int potrf_one(double* A, int64_t n, int64_t lda, int invert, double* diag_out, int* info,
              void* ws, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    VG_HIP(hipFuncSetAttribute((const void*)potrf_diag_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)diag_shmem()));
    attr_set = true;
  }
  const int64_t leaves = (n + NB - 1) / NB;
  Fact f{lda, static_cast<double*>(ws), static_cast<double*>(ws) + leaves * NB * NB, diag_out,
         info, stream};
  int rc = potrf_rec(f, A, n, 0);
  if (rc || !invert) return rc;
  return trtri_rec(f, A, n, 0);
}

}  // namespace vgposp

extern "C" size_t vgposp_potrf_workspace_bytes(int64_t n) {
  return n > 0 ? vgposp::potrf_ws_bytes(n) : 0;
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
  VG_CHECK_ARG(ws != nullptr || n == 0, 9);
  hipStream_t s = as_stream(stream);
  VG_HIP(hipMemsetAsync(info, 0, sizeof(int) * batch, s));
  if (n == 0) return 0;
  if (ws_bytes < potrf_ws_bytes(n)) {
    set_error("vgposp_potrf_lower: workspace %zu < %zu bytes", ws_bytes, potrf_ws_bytes(n));
    return VGPOSP_E_WS;
  }
  if (n <= NB && batch > 1) {
    // one launch, one workgroup per matrix (e.g. the calc_H likelihood surface)
    static bool attr_set = false;
    if (!attr_set) {
      VG_HIP(hipFuncSetAttribute((const void*)potrf_diag_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)diag_shmem()));
      attr_set = true;
    }
    ProfScope ps("potrf_diag", s, batch * 2.0 * n * (double)n * n / 3.0, batch * 16.0 * n * (double)n);
    hipLaunchKernelGGL(potrf_diag_kernel, dim3(batch), dim3(DIAG_THREADS), diag_shmem(), s, A, lda,
                       (int)n, (int64_t)0, invert, (double*)nullptr, diag_out, info, stride);
    VG_LAUNCH_CHECK();
    return 0;
  }
  for (int b = 0; b < batch; ++b) {
    int rc = potrf_one(A + b * stride, n, lda, invert, diag_out ? diag_out + (int64_t)b * n : nullptr,
                       info + b, ws, s);
    if (rc) return rc;
  }
  return 0;
}
