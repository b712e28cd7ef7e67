// Covariance builders producing cov_vv on device:
//
// * vgposp_kernel_matvec: out = K(X1, X2) v without materialising K.  This is the predictive mean
//   K_*z Kzz^-1 m of the trained VGP at every (location, temperature/pressure sample) 5-D point
//   (main_architecture_2_sampledistribution.py:432-458, tfd.VariationalGaussianProcess(...).mean())
//   and the GPRM mean.  X2 / v stream through LDS in 256-point tiles; each thread owns one X1 row.
//   Bound by the fp64 exp / VALU, not by HBM.
// * vgposp_center_rows: T[i][:] <- (T[i][:] - mean_s T[i][s]) * scale, one wave per location.
//   Followed by a SYRK on fp64 MFMA this is tfp.stats.covariance(t_i, t_j, sample_axis=0)
//   (biased, centred by the sample mean) for every pair (i, j) at once (main.py:190-199,
//   main_architecture_2_sampledistribution.py:470-479).  The reference's fixed standardisation
//   (t - tr_mean) / tr_stdev only rescales by 1 / tr_stdev^2.
// * vgposp_index_taper: the beta-decay "local kernel filter"
//   (main_architecture_2_sampledistribution.py:361-421):
//     C[i][j] *= g(delta_ij),  g(d) = exp(-(beta d)^2 / (2 pi)),  0 where g < threshold (0.01),
//   with delta_ij the Euclidean distance between the grid indices of locations i and j.  The
//   flattening is C-order, i = i0 I1 I2 + i1 I2 + i2 (main.py:259-267).  One HBM pass.
#include <algorithm>

#include "psd.h"

namespace vgposp {

constexpr int MV_TILE = 256;

template <int KIND, int D>
__global__ __launch_bounds__(256) void kernel_matvec_kernel(const double* X1, int64_t n1,
                                                            const double* X2, int64_t n2,
                                                            const double* amp, const double* ls,
                                                            const double* v, double beta,
                                                            double* out) {
  __shared__ double xs[MV_TILE * D];
  __shared__ double vs[MV_TILE];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const double tla = 2.0 * log(amp[0]), inv_l = 1.0 / ls[0], inv_l2 = inv_l * inv_l;
  double x1[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x1[k] = i < n1 ? X1[i * D + k] : 0.0;
  double acc0 = 0.0, acc1 = 0.0;
  for (int64_t j0 = 0; j0 < n2; j0 += MV_TILE) {
    const int jn = (int)min((int64_t)MV_TILE, n2 - j0);
    __syncthreads();
    for (int e = threadIdx.x; e < MV_TILE * D; e += 256)
      xs[e] = e < jn * D ? X2[j0 * D + e] : 0.0;
    vs[threadIdx.x] = threadIdx.x < jn ? v[j0 + threadIdx.x] : 0.0;
    __syncthreads();
    int jj = 0;
    for (; jj + 1 < jn; jj += 2) {
      double d2a = 0.0, d2b = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double da = x1[k] - xs[jj * D + k], db = x1[k] - xs[(jj + 1) * D + k];
        d2a += da * da;
        d2b += db * db;
      }
      acc0 += kfun<KIND>(d2a, tla, inv_l, inv_l2) * vs[jj];
      acc1 += kfun<KIND>(d2b, tla, inv_l, inv_l2) * vs[jj + 1];
    }
    if (jj < jn) {
      double d2 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double dd = x1[k] - xs[jj * D + k];
        d2 += dd * dd;
      }
      acc0 += kfun<KIND>(d2, tla, inv_l, inv_l2) * vs[jj];
    }
  }
  if (i < n1) out[i] = (acc0 + acc1) + (beta != 0.0 ? beta * out[i] : 0.0);
}

__global__ __launch_bounds__(256) void center_rows_kernel(double* T, int64_t n, int64_t s,
                                                          int64_t ld, double scale) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  double* row = T + i * ld;
  double acc = 0.0;
  for (int64_t c = lane; c < s; c += 64) acc += row[c];
  const double mean = wave_sum(acc) / (double)s;
  for (int64_t c = lane; c < s; c += 64) row[c] = (row[c] - mean) * scale;
}

__global__ __launch_bounds__(256) void index_taper_kernel(double* C, int64_t n, int64_t ldc,
                                                          int64_t I1, int64_t I2, double beta,
                                                          double threshold, int lower) {
  const int64_t s0 = I1 * I2;
  const double c2 = beta * beta / (2.0 * 3.141592653589793);
  for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t i0 = i / s0, i1 = (i - i0 * s0) / I2, i2 = i - i0 * s0 - i1 * I2;
    const int64_t jend = lower ? i + 1 : n;
    for (int64_t j = threadIdx.x; j < jend; j += 256) {
      const int64_t j0 = j / s0, j1 = (j - j0 * s0) / I2, j2 = j - j0 * s0 - j1 * I2;
      const double d0 = (double)(i0 - j0), d1 = (double)(i1 - j1), d2 = (double)(i2 - j2);
      // exp(-(beta * delta)^2 / (2 pi)) with delta^2 = d0^2 + d1^2 + d2^2 (the sqrt cancels)
      const double g = exp(-c2 * (d0 * d0 + d1 * d1 + d2 * d2));
      double* c = C + i * ldc + j;
      *c = g < threshold ? 0.0 : *c * g;
    }
  }
}

template <int KIND>
static void launch_matvec(unsigned g, hipStream_t s, int d, const double* X1, int64_t n1,
                          const double* X2, int64_t n2, const double* amp, const double* ls,
                          const double* v, double beta, double* out) {
#define MV_CASE(DD)                                                                               \
  case DD:                                                                                        \
    hipLaunchKernelGGL((kernel_matvec_kernel<KIND, DD>), dim3(g), dim3(256), 0, s, X1, n1, X2, n2, \
                       amp, ls, v, beta, out);                                                    \
    break;
  switch (d) { MV_CASE(1) MV_CASE(2) MV_CASE(3) MV_CASE(4) MV_CASE(5) MV_CASE(6) MV_CASE(7) MV_CASE(8) }
#undef MV_CASE
}

}  // namespace vgposp

using namespace vgposp;

extern "C" int vgposp_kernel_matvec(int kind, const double* X1, int64_t n1, const double* X2,
                                    int64_t n2, int d, const double* amp, const double* ls,
                                    const double* v, double beta, double* out, void* stream) {
  clear_error();
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);
  VG_CHECK_ARG(X1 != nullptr || n1 == 0, 2);
  VG_CHECK_ARG(n1 >= 0, 3);
  VG_CHECK_ARG(X2 != nullptr || n2 == 0, 4);
  VG_CHECK_ARG(n2 >= 0, 5);
  VG_CHECK_ARG(d >= 1 && d <= 8, 6);
  VG_CHECK_ARG(amp != nullptr, 7);
  VG_CHECK_ARG(ls != nullptr, 8);
  VG_CHECK_ARG(v != nullptr || n2 == 0, 9);
  VG_CHECK_ARG(out != nullptr || n1 == 0, 11);
  if (n1 == 0) return 0;
  hipStream_t s = as_stream(stream);
  const unsigned g = (unsigned)ceil_div(n1, 256);
  ProfScope ps("kernel_matvec", s, 0.0, 8.0 * ((double)n1 * (d + 1) + (double)n2 * (d + 1)));
  switch (kind) {
    case VGPOSP_KERNEL_EQ: launch_matvec<VGPOSP_KERNEL_EQ>(g, s, d, X1, n1, X2, n2, amp, ls, v, beta, out); break;
    case VGPOSP_KERNEL_MATERN12: launch_matvec<VGPOSP_KERNEL_MATERN12>(g, s, d, X1, n1, X2, n2, amp, ls, v, beta, out); break;
    case VGPOSP_KERNEL_MATERN32: launch_matvec<VGPOSP_KERNEL_MATERN32>(g, s, d, X1, n1, X2, n2, amp, ls, v, beta, out); break;
    default: launch_matvec<VGPOSP_KERNEL_MATERN52>(g, s, d, X1, n1, X2, n2, amp, ls, v, beta, out); break;
  }
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_center_rows(double* T, int64_t n, int64_t s, int64_t ld, double scale,
                                  void* stream) {
  clear_error();
  VG_CHECK_ARG(T != nullptr || n == 0, 1);
  VG_CHECK_ARG(n >= 0, 2);
  VG_CHECK_ARG(s >= 1, 3);
  VG_CHECK_ARG(ld >= s, 4);
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  ProfScope ps("center_rows", st, 0.0, 24.0 * (double)n * s);
  hipLaunchKernelGGL(center_rows_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, st, T, n, s,
                     ld, scale);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_index_taper(double* C, int64_t n, int64_t ldc, int64_t I0, int64_t I1,
                                  int64_t I2, double beta, double threshold, int uplo,
                                  void* stream) {
  clear_error();
  VG_CHECK_ARG(C != nullptr || n == 0, 1);
  VG_CHECK_ARG(n >= 0, 2);
  VG_CHECK_ARG(ldc >= n, 3);
  VG_CHECK_ARG(I0 >= 1 && I1 >= 1 && I2 >= 1 && I0 * I1 * I2 == n, 4);
  VG_CHECK_ARG(beta >= 0.0, 7);
  VG_CHECK_ARG(uplo == VGPOSP_FULL || uplo == VGPOSP_LOWER, 9);
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  ProfScope ps("index_taper", s, 0.0, 16.0 * (double)n * n * (uplo == VGPOSP_LOWER ? 0.5 : 1.0));
  hipLaunchKernelGGL(index_taper_kernel, dim3((unsigned)std::min<int64_t>(n, 16384)), dim3(256), 0,
                     s, C, n, ldc, I1, I2, beta, threshold, uplo == VGPOSP_LOWER);
  VG_LAUNCH_CHECK();
  return 0;
}
