// Exact-GP log marginal likelihood and its gradient from the inverted Cholesky factor.
//
// Replaces, for tfd.GaussianProcess(kernel, X, noise).log_prob(y) (gp_functions.py:166-172,
// main.py:105, 3D_sin_wave.py:172) and the TF autodiff behind tf_train_gp_adam
// (gp_functions.py:179-182):
//     C = K + (noise + jitter) I = L L^T,   M = L^-1   (potrf.hip, invert=1)
//     z = M y,  LML = -0.5 |z|^2 - sum log L_ii - n/2 log(2 pi),  alpha = C^-1 y = M^T z
//     dLML/dtheta = 0.5 sum_ij (alpha alpha^T - C^-1)_ij dC_ij/dtheta
// The gradient pass regenerates dK/dtheta from X on the fly (no dK matrices in HBM) and reads the
// lower triangle of C^-1 once: it is HBM-bound at 4 n(n+1) bytes per batch entry.
#include <cmath>

#include "common.h"

namespace vgposp {

constexpr double LOG_2PI = 1.8378770664093453;

// z[b][r] = sum_{c <= r} M[r][c] y[c]   (one wave per row)
__global__ __launch_bounds__(256) void trmv_rows_kernel(const double* M, int64_t n, int64_t lda,
                                                        int64_t stride, const double* y,
                                                        double* z) {
  const int b = blockIdx.y;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const double* row = M + b * stride + r * lda;
  double s = 0.0;
  for (int64_t c = lane; c <= r; c += 64) s += row[c] * y[c];
  s = wave_sum(s);
  if (lane == 0) z[b * n + r] = s;
}

// alpha[b][i] = sum_{r >= i} M[r][i] z[b][r]   (one thread per column, coalesced rows)
__global__ __launch_bounds__(256) void trmv_cols_kernel(const double* M, int64_t n, int64_t lda,
                                                        int64_t stride, const double* z,
                                                        double* alpha) {
  const int b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double* Mb = M + b * stride;
  const double* zb = z + b * n;
  double s0 = 0.0, s1 = 0.0;
  int64_t r = i;
  for (; r + 1 < n; r += 2) {
    s0 += Mb[r * lda + i] * zb[r];
    s1 += Mb[(r + 1) * lda + i] * zb[r + 1];
  }
  if (r < n) s0 += Mb[r * lda + i] * zb[r];
  alpha[b * n + i] = s0 + s1;
}

__device__ double block_sum_1024(double v) {
  __shared__ double sh[16];
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  v = (l < (int)(blockDim.x >> 6)) ? sh[l] : 0.0;
  return wave_sum(v);
}

__global__ __launch_bounds__(1024) void lml_reduce_kernel(int64_t n, const double* z,
                                                          const double* Ldiag, double* out) {
  const int b = blockIdx.x;
  double q = 0.0, ld = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double zi = z[b * n + i];
    q += zi * zi;
    ld += log(Ldiag[b * n + i]);
  }
  q = block_sum_1024(q);
  ld = block_sum_1024(ld);
  if (threadIdx.x == 0) out[b] = -0.5 * q - ld - 0.5 * (double)n * LOG_2PI;
}

// dK/damp and dK/dls at squared distance d2 (same formulas as kernel_matrix.hip).
__device__ __forceinline__ void kgrad(int kind, double d2, double a, double l, double& dka,
                                      double& dkl) {
  const double tla = 2.0 * log(a);
  double K;
  const double r0 = sqrt(d2);
  const double r = r0 / l;
  if (kind == VGPOSP_KERNEL_EQ) {
    K = exp(tla - 0.5 * d2 / (l * l));
    dkl = K * d2 / (l * l * l);
  } else if (kind == VGPOSP_KERNEL_MATERN12) {
    K = exp(tla - r);
    dkl = K * r / l;
  } else if (kind == VGPOSP_KERNEL_MATERN32) {
    const double s = 1.7320508075688772 * r;
    K = exp(tla + log1p(s) - s);
    dkl = a * a * exp(-s) * s * s / l;
  } else {
    const double s = 2.23606797749979 * r;
    K = exp(tla + log1p(s + s * s / 3.0) - s);
    dkl = a * a * exp(-s) * (s * s / 3.0) * (1.0 + s) / l;
  }
  dka = 2.0 * K / a;
}

constexpr int GR_ROWS = 16;

// Partial sums over 16-row stripes of the lower triangle:
//   part[b][blk] = (sum G dK/damp, sum G dK/dls, sum_i G_ii)   with symmetric weights.
__global__ __launch_bounds__(256) void lml_grad_kernel(int kind, const double* X, int64_t n,
                                                       int d, const double* amp,
                                                       const double* ls, const double* Cinv,
                                                       int64_t ldc, int64_t stride_c,
                                                       const double* alpha, double* part) {
  const int b = blockIdx.y;
  const double a = amp[b], l = ls[b];
  const double* Cb = Cinv + b * stride_c;
  const double* al = alpha + b * n;
  double sa = 0.0, sl = 0.0, sn = 0.0;
  const int64_t r0 = (int64_t)blockIdx.x * GR_ROWS;
  for (int rr = 0; rr < GR_ROWS; ++rr) {
    const int64_t i = r0 + rr;
    if (i >= n) break;
    const double ai = al[i];
    for (int64_t j = threadIdx.x; j <= i; j += 256) {
      double d2 = 0.0;
      for (int k = 0; k < d; ++k) {
        const double e = X[i * d + k] - X[j * d + k];
        d2 += e * e;
      }
      const double g = ai * al[j] - Cb[i * ldc + j];
      double dka, dkl;
      kgrad(kind, d2, a, l, dka, dkl);
      const double wgt = (j == i) ? 1.0 : 2.0;
      sa += wgt * g * dka;
      sl += wgt * g * dkl;
      if (j == i) sn += g;
    }
  }
  sa = wave_sum(sa);
  sl = wave_sum(sl);
  sn = wave_sum(sn);
  __shared__ double sh[3][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = sa;
    sh[1][w] = sl;
    sh[2][w] = sn;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const double v = sh[threadIdx.x][0] + sh[threadIdx.x][1] + sh[threadIdx.x][2] + sh[threadIdx.x][3];
    part[((int64_t)b * gridDim.x + blockIdx.x) * 3 + threadIdx.x] = v;
  }
}

__global__ __launch_bounds__(1024) void lml_grad_reduce_kernel(int64_t nblk, const double* part,
                                                               double* grad) {
  const int b = blockIdx.x;
  double s[3] = {0.0, 0.0, 0.0};
  for (int64_t e = threadIdx.x; e < nblk; e += blockDim.x)
    for (int q = 0; q < 3; ++q) s[q] += part[((int64_t)b * nblk + e) * 3 + q];
  for (int q = 0; q < 3; ++q) {
    const double v = block_sum_1024(s[q]);
    if (threadIdx.x == 0) grad[b * 3 + q] = 0.5 * v;
  }
}

}  // namespace vgposp

using namespace vgposp;

extern "C" size_t vgposp_lml_workspace_bytes(int64_t n, int batch) {
  return (size_t)n * batch * sizeof(double);
}

extern "C" int vgposp_lml(const double* Minv, int64_t n, int64_t lda, int64_t stride, int batch,
                          const double* Ldiag, const double* y, double* alpha, double* out,
                          void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(Minv != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(lda >= n, 3);
  VG_CHECK_ARG(batch >= 1 && batch <= 65535, 5);
  VG_CHECK_ARG(batch == 1 || stride >= lda * n, 4);
  VG_CHECK_ARG(Ldiag != nullptr, 6);
  VG_CHECK_ARG(y != nullptr, 7);
  VG_CHECK_ARG(out != nullptr, 9);
  VG_CHECK_ARG(ws != nullptr, 10);
  if (ws_bytes < vgposp_lml_workspace_bytes(n, batch)) {
    set_error("vgposp_lml: workspace too small");
    return VGPOSP_E_WS;
  }
  hipStream_t s = as_stream(stream);
  double* z = static_cast<double*>(ws);
  hipLaunchKernelGGL(trmv_rows_kernel, dim3((unsigned)ceil_div(n, 4), batch), dim3(256), 0, s,
                     Minv, n, lda, stride, y, z);
  VG_LAUNCH_CHECK();
  hipLaunchKernelGGL(lml_reduce_kernel, dim3(batch), dim3(1024), 0, s, n, z, Ldiag, out);
  VG_LAUNCH_CHECK();
  if (alpha) {
    hipLaunchKernelGGL(trmv_cols_kernel, dim3((unsigned)ceil_div(n, 256), batch), dim3(256), 0, s,
                       Minv, n, lda, stride, z, alpha);
    VG_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" size_t vgposp_lml_grad_workspace_bytes(int64_t n, int batch) {
  return (size_t)ceil_div(n, GR_ROWS) * batch * 3 * sizeof(double);
}

extern "C" int vgposp_lml_grad(int kind, const double* X, int64_t n, int d, const double* amp,
                               const double* ls, const double* Cinv, int64_t ldc,
                               int64_t stride_c, const double* alpha, int batch, double* grad,
                               void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);
  VG_CHECK_ARG(X != nullptr, 2);
  VG_CHECK_ARG(n >= 1, 3);
  VG_CHECK_ARG(d >= 1, 4);
  VG_CHECK_ARG(amp != nullptr, 5);
  VG_CHECK_ARG(ls != nullptr, 6);
  VG_CHECK_ARG(Cinv != nullptr, 7);
  VG_CHECK_ARG(ldc >= n, 8);
  VG_CHECK_ARG(batch == 1 || stride_c >= ldc * n, 9);
  VG_CHECK_ARG(alpha != nullptr, 10);
  VG_CHECK_ARG(batch >= 1 && batch <= 65535, 11);
  VG_CHECK_ARG(grad != nullptr, 12);
  VG_CHECK_ARG(ws != nullptr, 13);
  if (ws_bytes < vgposp_lml_grad_workspace_bytes(n, batch)) {
    set_error("vgposp_lml_grad: workspace too small");
    return VGPOSP_E_WS;
  }
  hipStream_t s = as_stream(stream);
  const int64_t nblk = ceil_div(n, GR_ROWS);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(lml_grad_kernel, dim3((unsigned)nblk, batch), dim3(256), 0, s, kind, X, n, d,
                     amp, ls, Cinv, ldc, stride_c, alpha, part);
  VG_LAUNCH_CHECK();
  hipLaunchKernelGGL(lml_grad_reduce_kernel, dim3(batch), dim3(1024), 0, s, nblk, part, grad);
  VG_LAUNCH_CHECK();
  return 0;
}
