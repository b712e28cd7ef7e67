// Mixed-precision Cholesky (config C5 of BASELINE.json: "fp32 mixed-prec Cholesky"): the factor is
// computed in fp32 on the f32 matrix cores (v_mfma_f32_16x16x4_f32, 2x the fp64 MFMA rate), then
// refined in fp64 to the inverse Cholesky factor the fp64 path produces.  Replaces the
// tf.linalg.cholesky calls of the reference's VGP graph (main_architecture_2_sampledistribution.py
// :223-265 through tfd.VariationalGaussianProcess) when the caller asks for mixed precision.
//
//   1. A32 = fp32(A);  right-looking blocked Cholesky in fp32 with 64-column leaves (one wave, rows
//      in registers) and NT GEMMs on v_mfma_f32_16x16x4_f32 for the panel (P <- P Linv^T) and trailing update.
//   2. X0 = fp64(L32)^-1 (fp64 TRSM against I).
//   3. k iterations in fp64:  E = X A X^T - I,  X <- (I - Phi(E)) X,  Phi = lower(E), diag halved.
//      X A X^T = I + E  =>  X' A X'^T = I + O(E^2): quadratic convergence from |E0| ~ cond(A) eps32,
//      three iterations reach fp64 rounding from |E0| ~ 1e-2 (-> 1e-4 -> 1e-8 -> 1e-16; C5's
//      unjittered Kzz needs the third).  The converged X is the lower
//      L^-1 of A = L L^T, so diag(L) = 1 / diag(X) gives the log-determinant.
// max|E| of the last iteration is reported (resid); info = n + 1 when it stays above 1e-6 (the
// fp32 factor too poor to refine), k > 0 when fp32 pivot k fails.
#include <algorithm>

#include "common.h"

namespace vgposp {

int trsm_left(const double* L, int64_t n, int64_t ldl, int trans, double* B, int64_t m, int64_t ldb,
              void* ws, hipStream_t s);
size_t trsm_ws_bytes(int64_t n, int64_t m);
int gemm_launch_split(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                      const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                      double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, int nsplit,
                      double* part, hipStream_t stream);
int gemm_auto_splits(int64_t m, int64_t n, int64_t k, int uplo_c, int transa);

constexpr int64_t RPART = 1 << 23;  // split-K partials of the refinement GEMMs (64 MiB)

constexpr int SNB = 64;  // fp32 leaf

typedef float flt4 __attribute__((ext_vector_type(4)));

// fp32 leaf: factor the jb x jb diagonal block at A (lda) and write L back (lower) and its dense
// inverse to linv [SNB][SNB].  One wave: lane i holds row i of the block (rows >= jb padded with
// identity rows) and row i of the inverse in registers; column values move by v_readlane (the
// loops are fully unrolled, so every register index is static).  Right-looking elimination, then
// forward substitution row by row.  info <- col0 + k + 1 at the first non-positive pivot.
__global__ __launch_bounds__(64) void spotrf_leaf_kernel(float* A, int64_t lda, int jb,
                                                         int64_t col0, float* linv, int* info) {
  const int i = threadIdx.x;
  float a[SNB], x[SNB];
#pragma unroll
  for (int j = 0; j < SNB; ++j) {
    a[j] = (i < jb && j <= i) ? A[(int64_t)i * lda + j] : (i == j ? 1.0f : 0.0f);
    x[j] = i == j ? 1.0f : 0.0f;
  }
#pragma unroll
  for (int k = 0; k < SNB; ++k) {
    const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a[k]), k));
    if (i == 0 && k < jb && !(d > 0.0f) && info != nullptr && *info == 0)
      *info = (int)(col0 + k + 1);
    const float piv = sqrtf(d);
    const float lik = i > k ? a[k] / piv : (i == k ? piv : a[k]);
    a[k] = lik;
#pragma unroll
    for (int j = k + 1; j < SNB; ++j)
      a[j] -= lik * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lik), j));
  }
  // X = L^-1: row k final once divided by L_kk, then removed from the rows below
#pragma unroll
  for (int k = 0; k < SNB; ++k) {
    const float rinv = 1.0f / __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a[k]), k));
    if (i == k) {
#pragma unroll
      for (int j = 0; j <= k; ++j) x[j] *= rinv;
    }
    const float lik = i > k ? a[k] : 0.0f;
#pragma unroll
    for (int j = 0; j <= k; ++j)
      x[j] -= lik * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[j]), k));
  }
#pragma unroll
  for (int j = 0; j < SNB; ++j) {
    if (i < jb && j <= i) A[(int64_t)i * lda + j] = a[j];
    linv[i * SNB + j] = j <= i ? x[j] : 0.0f;
  }
}

// C (m x n) = alpha A B^T + beta C in fp32; A [m][k], B [n][k] row-major (k contiguous).  64 x 64
// tiles, 4 waves of 32 x 32 (2 x 2 v_mfma_f32_16x16x4_f32 accumulators), 16-deep K-steps through
// LDS.  lower: only C entries with col <= row (tiles above the diagonal exit at once).
__global__ __launch_bounds__(256) void sgemm_nt_kernel(int64_t m, int64_t n, int64_t k, float alpha,
                                                       const float* A, int64_t lda, const float* B,
                                                       int64_t ldb, float beta, float* C,
                                                       int64_t ldc, int lower) {
  __shared__ float As[64 * 17];
  __shared__ float Bs[64 * 17];
  const int64_t m0 = (int64_t)blockIdx.y * 64, n0 = (int64_t)blockIdx.x * 64;
  if (lower && n0 > m0 + 63) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;
  flt4 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) acc[i][j] = flt4{0.f, 0.f, 0.f, 0.f};
  for (int64_t k0 = 0; k0 < k; k0 += 16) {
    for (int e = tid; e < 64 * 16; e += 256) {
      const int r = e >> 4, kk = e & 15;
      const int64_t gk = k0 + kk;
      As[r * 17 + kk] = (m0 + r < m && gk < k) ? A[(m0 + r) * lda + gk] : 0.0f;
      Bs[r * 17 + kk] = (n0 + r < n && gk < k) ? B[(n0 + r) * ldb + gk] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[(wm * 32 + i * 16 + fr) * 17 + ks * 4 + fk];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[(wn * 32 + j * 16 + fr) * 17 + ks * 4 + fk];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // f32 16x16x4 C/D map: col = lane & 15, row = 4 (lane >> 4) + reg
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 32 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 32 + i * 16 + 4 * fk + r;
        if (row < m && col < n && (!lower || col <= row)) {
          float* c = C + row * ldc + col;
          float v = alpha * acc[i][j][r];
          if (beta != 0.0f) v += beta * *c;
          *c = v;
        }
      }
    }
}

// dst32 (n x n, ld n) <- lower triangle of src64 (lda)
__global__ void cast_lower_kernel(const double* src, int64_t lda, float* dst, int64_t n) {
  const int64_t r = blockIdx.y;
  for (int64_t c = threadIdx.x; c < n; c += blockDim.x)
    dst[r * n + c] = c <= r ? (float)src[r * lda + c] : 0.0f;
}

// dst64 (ldd) <- fp64(lower src32) with zeros above the diagonal; I64 (ldd) <- identity
__global__ void upcast_lower_kernel(const float* src, int64_t n, double* dst, int64_t ldd,
                                    double* eye) {
  const int64_t r = blockIdx.y;
  for (int64_t c = threadIdx.x; c < n; c += blockDim.x) {
    dst[r * ldd + c] = c <= r ? (double)src[r * n + c] : 0.0;
    eye[r * n + c] = r == c ? 1.0 : 0.0;
  }
}

// E <- Phi(E - I) (lower, diagonal halved, zeros above); amax <- max |E - I| (bit pattern of a
// non-negative double: integer max orders it)
__global__ void refine_phi_kernel(double* E, int64_t n, unsigned long long* amax) {
  const int64_t r = blockIdx.y;
  double mx = 0.0;
  for (int64_t c = threadIdx.x; c < n; c += blockDim.x) {
    double e = E[r * n + c] - (r == c ? 1.0 : 0.0);
    mx = fmax(mx, fabs(e));
    E[r * n + c] = c < r ? e : (c == r ? 0.5 * e : 0.0);
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) atomicMax(amax, (unsigned long long)__double_as_longlong(mx));
}

// diag_out[i] = 1 / X_ii (= diag L);  resid <- max|E| of the last iteration;  info <- n + 1 when
// that exceeds tol (and no fp32 pivot failed)
__global__ void refine_finish_kernel(const double* X, int64_t ldx, int64_t n, double* diag_out,
                                     const unsigned long long* amax, double* resid, double tol,
                                     int* info) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && diag_out) diag_out[i] = 1.0 / X[i * ldx + i];
  if (i == 0) {
    const double r = __longlong_as_double((long long)*amax);
    if (resid) *resid = r;
    if (!(r <= tol) && *info == 0) *info = (int)(n + 1);
  }
}

static size_t al(size_t b) { return (b + 255) & ~(size_t)255; }

struct MixedWS {
  float *A32, *linv, *tmp;
  double *T, *E, *Y, *part;
  unsigned long long* amax;
  void* tws;
  size_t bytes;
};

static MixedWS mixed_layout(void* base, int64_t n) {
  MixedWS w{};
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t b) {
    char* r = p ? p + off : nullptr;
    off += al(b);
    return r;
  };
  const int64_t nl = ceil_div(n, SNB);
  w.A32 = (float*)take((size_t)n * n * 4);
  w.linv = (float*)take((size_t)nl * SNB * SNB * 4);
  w.tmp = (float*)take((size_t)n * SNB * 4);
  w.T = (double*)take((size_t)n * n * 8);
  w.E = (double*)take((size_t)n * n * 8);
  w.Y = (double*)take((size_t)n * n * 8);
  w.part = (double*)take((size_t)std::min<int64_t>(RPART, 8 * n * n) * 8);
  w.amax = (unsigned long long*)take(64);
  w.tws = take(trsm_ws_bytes(n, n));
  w.bytes = off;
  return w;
}

// the refinement's n x n x n fp64 products: few 128 x 128 tiles (64 at n = 1024), so split-K
static int rgemm(const MixedWS& w, int transa, int transb, int64_t n, double alpha, const double* A,
                 int64_t lda, const double* B, int64_t ldb, double beta, double* C, int64_t ldc,
                 int uplo_c, int tri_a, int tri_b, hipStream_t s) {
  int sp = gemm_auto_splits(n, n, n, uplo_c, transa);
  while (sp > 1 && (int64_t)sp * n * n > RPART) --sp;
  return gemm_launch_split(transa, transb, n, n, n, alpha, A, lda, B, ldb, beta, C, ldc, uplo_c,
                           tri_a, tri_b, sp, sp > 1 ? w.part : nullptr, s);
}

static int sgemm_nt(int64_t m, int64_t n, int64_t k, float alpha, const float* A, int64_t lda,
                    const float* B, int64_t ldb, float beta, float* C, int64_t ldc, int lower,
                    hipStream_t s) {
  dim3 g((unsigned)ceil_div(n, 64), (unsigned)ceil_div(m, 64));
  ProfScope ps("gemm_f32", s, (lower ? 1.0 : 2.0) * m * n * k, 0.0);
  hipLaunchKernelGGL(sgemm_nt_kernel, g, dim3(256), 0, s, m, n, k, alpha, A, lda, B, ldb, beta, C,
                     ldc, lower);
  VG_LAUNCH_CHECK();
  return 0;
}

// right-looking fp32 Cholesky of A32 (n x n, ld n) in place, leaf inverses kept in w.linv
static int spotrf(const MixedWS& w, int64_t n, int* info, hipStream_t s) {
  float* A = w.A32;
  for (int64_t j0 = 0; j0 < n; j0 += SNB) {
    const int jb = (int)(n - j0 < SNB ? n - j0 : SNB);
    float* Lj = w.linv + (j0 / SNB) * SNB * SNB;
    {
      ProfScope ps("potrf_diag_f32", s, jb * (double)jb * jb / 3.0, 0.0);
      hipLaunchKernelGGL(spotrf_leaf_kernel, dim3(1), dim3(64), 0, s, A + j0 * n + j0, n, jb, j0,
                         Lj, info);
      VG_LAUNCH_CHECK();
    }
    const int64_t rest = n - j0 - jb;
    if (rest <= 0) break;
    float* P = A + (j0 + jb) * n + j0;
    int rc;
    // tmp = P Linv^T  (Linv [jb][jb] at pitch SNB), then back into the panel
    if ((rc = sgemm_nt(rest, jb, jb, 1.0f, P, n, Lj, SNB, 0.0f, w.tmp, jb, 0, s))) return rc;
    VG_HIP(vg_memcpy2d(P, n * sizeof(float), w.tmp, jb * sizeof(float), jb * sizeof(float),
                            rest, hipMemcpyDeviceToDevice, s));
    // trailing A22 -= P P^T (lower)
    if ((rc = sgemm_nt(rest, rest, jb, -1.0f, w.tmp, jb, w.tmp, jb, 1.0f, P + jb, n, 1, s)))
      return rc;
  }
  return 0;
}

}  // namespace vgposp

using namespace vgposp;

extern "C" size_t vgposp_potrf_mixed_workspace_bytes(int64_t n) {
  return n > 0 ? mixed_layout(nullptr, n).bytes : 0;
}

extern "C" int vgposp_potrf_mixed(const double* A, int64_t n, int64_t lda, double* Linv,
                                  int64_t ldl, double* diag_out, int iters, double* resid,
                                  int* info, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(A != nullptr, 1);
  VG_CHECK_ARG(n >= 1 && n <= 16384, 2);
  VG_CHECK_ARG(lda >= n, 3);
  VG_CHECK_ARG(Linv != nullptr && Linv != A, 4);
  VG_CHECK_ARG(ldl >= n, 5);
  VG_CHECK_ARG(iters >= 0 && iters <= 8, 7);
  VG_CHECK_ARG(info != nullptr, 9);
  VG_CHECK_ARG(ws != nullptr, 10);
  MixedWS w = mixed_layout(ws, n);
  if (ws_bytes < w.bytes) {
    set_error("vgposp_potrf_mixed: workspace %zu < %zu bytes", ws_bytes, w.bytes);
    return VGPOSP_E_WS;
  }
  hipStream_t s = as_stream(stream);
  VG_HIP(vg_memset(info, 0, sizeof(int), s));
  VG_HIP(vg_memset(w.amax, 0, sizeof(unsigned long long), s));
  hipLaunchKernelGGL(cast_lower_kernel, dim3(1, (unsigned)n), dim3(256), 0, s, A, lda, w.A32, n);
  VG_LAUNCH_CHECK();
  int rc = spotrf(w, n, info, s);
  if (rc) return rc;
  // X0 = fp64(L32)^-1: L64 in T, I in Linv, TRSM in place on Linv
  double* X = Linv;
  hipLaunchKernelGGL(upcast_lower_kernel, dim3(1, (unsigned)n), dim3(256), 0, s, w.A32, n, w.T, n,
                     w.E);
  VG_LAUNCH_CHECK();
  VG_HIP(vg_memcpy2d(X, ldl * sizeof(double), w.E, n * sizeof(double), n * sizeof(double), n,
                          hipMemcpyDeviceToDevice, s));
  if ((rc = trsm_left(w.T, n, n, 0, X, n, ldl, w.tws, s))) return rc;
  for (int it = 0; it < iters; ++it) {
    // T = A X^T (X lower), E = X T
    if ((rc = rgemm(w, 0, 1, n, 1.0, A, lda, X, ldl, 0.0, w.T, n, VGPOSP_FULL, 0, 1, s))) return rc;
    if ((rc = rgemm(w, 0, 0, n, 1.0, X, ldl, w.T, n, 0.0, w.E, n, VGPOSP_FULL, 1, 0, s))) return rc;
    if (it == iters - 1) VG_HIP(vg_memset(w.amax, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(refine_phi_kernel, dim3(1, (unsigned)n), dim3(256), 0, s, w.E, n, w.amax);
    VG_LAUNCH_CHECK();
    // X <- X - Phi X  (out of place through Y)
    VG_HIP(vg_memcpy2d(w.Y, n * sizeof(double), X, ldl * sizeof(double), n * sizeof(double),
                            n, hipMemcpyDeviceToDevice, s));
    if ((rc = rgemm(w, 0, 0, n, -1.0, w.E, n, w.Y, n, 1.0, X, ldl, VGPOSP_LOWER, 1, 1, s))) return rc;
  }
  hipLaunchKernelGGL(refine_finish_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, X,
                     ldl, n, diag_out, w.amax, resid, iters > 0 ? 1e-6 : 1e300, info);
  VG_LAUNCH_CHECK();
  return 0;
}
