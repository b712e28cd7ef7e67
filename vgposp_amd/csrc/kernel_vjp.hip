// Vector-Jacobian product of the PSD kernel matrix K(X1, X2) — the reverse pass of kernel assembly
// that TF autodiff runs through `kernel.matrix` when the reference trains a VGP
// (variational_Gaussian_process_example.py:95-102: AdamOptimizer.minimize over amplitude,
// length_scale and the inducing_index_points).  Given Kbar (+ an optional rank-1 term u w^T):
//   grad[0] = sum_ij Kbar_ij dK_ij/damp        = sum Kbar 2K/amp
//   grad[1] = sum_ij Kbar_ij dK_ij/dls
//   X1bar_i = sum_j  Kbar_ij dK_ij/dx1_i       = sum_j Kbar_ij c(r_ij) (x1_i - x2_j)
// K is recomputed, never read: one pass over Kbar, HBM-bound (8 B per entry).
//
// Layout: a workgroup owns 16 rows x 1024 columns; its X2 columns sit in LDS, each wave walks whole
// row segments (16 columns per lane, coalesced 512 B per row per wave) and keeps per-row X1bar
// sums in registers, so the cross-lane reduction happens once per 1024 entries.  Partials go to
// the workspace ([col-blocks][n1][d] and [blocks][2]) and a second kernel reduces them in a fixed
// order: results are deterministic.
#include "common.h"
#include "psd.h"

namespace vgposp {

constexpr int VJ_ROWS = 16;
constexpr int VJ_COLS = 1024;
constexpr int VJ_MAXD = 8;

template <int KIND, int D>
__global__ __launch_bounds__(256) void kernel_vjp_kernel(const double* X1, int64_t n1,
                                                         const double* X2, int64_t n2,
                                                         const double* amp, const double* ls,
                                                         const double* Kbar, int64_t ldk,
                                                         const double* u, const double* w,
                                                         double* part_x, double* part_g) {
  __shared__ double x2s[VJ_COLS * D];
  __shared__ double red[2][4];
  const int64_t c0 = (int64_t)blockIdx.x * VJ_COLS;
  const int64_t r0 = (int64_t)blockIdx.y * VJ_ROWS;
  for (int e = threadIdx.x; e < VJ_COLS * D; e += 256) {
    const int64_t col = c0 + e / D;
    x2s[e] = col < n2 ? X2[c0 * D + e] : 0.0;
  }
  __syncthreads();
  const double a = amp[0], l = ls[0];
  const double tla = 2.0 * log(a), inv_l = 1.0 / l, inv_l2 = inv_l * inv_l, two_over_a = 2.0 / a;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double ga = 0.0, gl = 0.0;
  for (int rr = wave; rr < VJ_ROWS; rr += 4) {
    const int64_t i = r0 + rr;
    if (i >= n1) break;
    double x1[D], sx[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      x1[k] = X1[i * D + k];
      sx[k] = 0.0;
    }
    const double ui = u ? u[i] : 0.0;
    const double* krow = Kbar + i * ldk;
    for (int cc = lane; cc < VJ_COLS; cc += 64) {
      const int64_t j = c0 + cc;
      if (j >= n2) break;
      const double kb = krow[j] + (u ? ui * w[j] : 0.0);
      double diff[D], d2 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        diff[k] = x1[k] - x2s[cc * D + k];
        d2 += diff[k] * diff[k];
      }
      double K, dkl, cx;
      kvjp_entry<KIND>(d2, tla, inv_l, inv_l2, K, dkl, cx);
      ga += kb * K * two_over_a;
      gl += kb * dkl;
      const double cf = kb * cx;
#pragma unroll
      for (int k = 0; k < D; ++k) sx[k] += cf * diff[k];
    }
    if (part_x) {
#pragma unroll
      for (int k = 0; k < D; ++k) sx[k] = wave_sum(sx[k]);
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < D; ++k) part_x[((int64_t)blockIdx.x * n1 + i) * D + k] = sx[k];
      }
    }
  }
  ga = wave_sum(ga);
  gl = wave_sum(gl);
  if (lane == 0) {
    red[0][wave] = ga;
    red[1][wave] = gl;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const double v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
    part_g[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 2 + threadIdx.x] = v;
  }
}

// X1bar[i][k] = sum over the column blocks of part_x[cb][i][k]: one wave per output, lanes stride
// over the blocks, fixed order (deterministic).  The last workgroup also reduces the two scalars.
__global__ __launch_bounds__(256) void kernel_vjp_reduce_kernel(int64_t n1, int d, int64_t ncb,
                                                                int64_t nblk, const double* part_x,
                                                                const double* part_g,
                                                                double* grad, double* X1bar) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nout = X1bar ? n1 * d : 0;
  const int64_t nwg_x = (nout + 3) / 4;
  if ((int64_t)blockIdx.x < nwg_x) {
    const int64_t e = (int64_t)blockIdx.x * 4 + wv;
    if (e < nout) {
      double s = 0.0;
      for (int64_t cb = lane; cb < ncb; cb += 64) s += part_x[cb * n1 * d + e];
      s = wave_sum(s);
      if (lane == 0) X1bar[e] = s;
    }
    return;
  }
  __shared__ double sh[2][4];
  double s0 = 0.0, s1 = 0.0;
  for (int64_t b = threadIdx.x; b < nblk; b += 256) {
    s0 += part_g[2 * b];
    s1 += part_g[2 * b + 1];
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (lane == 0) {
    sh[0][wv] = s0;
    sh[1][wv] = s1;
  }
  __syncthreads();
  if (threadIdx.x < 2) grad[threadIdx.x] = sh[threadIdx.x][0] + sh[threadIdx.x][1] + sh[threadIdx.x][2] + sh[threadIdx.x][3];
}

int kernel_vjp_reduce_launch(int64_t n1, int d, int64_t ncb, int64_t nblk, const double* part_x,
                             const double* part_g, double* grad, double* X1bar, hipStream_t s) {
  const int64_t nwg_x = X1bar ? ceil_div(n1 * d, 4) : 0;
  hipLaunchKernelGGL(kernel_vjp_reduce_kernel, dim3((unsigned)(nwg_x + 1)), dim3(256), 0, s, n1, d,
                     ncb, nblk, part_x, part_g, grad, X1bar);
  VG_LAUNCH_CHECK();
  return 0;
}

static void vjp_layout(int64_t n1, int64_t n2, int d, int64_t* ncb, int64_t* nrb, size_t* bytes) {
  *ncb = ceil_div(n2, VJ_COLS);
  *nrb = ceil_div(n1, VJ_ROWS);
  *bytes = 8 * (size_t)((*ncb) * n1 * d + 2 * (*ncb) * (*nrb)) + 256;
}

template <int KIND>
static void launch_vjp(dim3 g, hipStream_t s, int d, const double* X1, int64_t n1,
                       const double* X2, int64_t n2, const double* amp, const double* ls,
                       const double* Kbar, int64_t ldk, const double* u, const double* w,
                       double* px, double* pg) {
#define VJ_CASE(DD)                                                                                \
  case DD:                                                                                         \
    hipLaunchKernelGGL((kernel_vjp_kernel<KIND, DD>), g, dim3(256), 0, s, X1, n1, X2, n2, amp, ls, \
                       Kbar, ldk, u, w, px, pg);                                                   \
    break;
  switch (d) {
    VJ_CASE(1) VJ_CASE(2) VJ_CASE(3) VJ_CASE(4) VJ_CASE(5) VJ_CASE(6) VJ_CASE(7) VJ_CASE(8)
  }
#undef VJ_CASE
}

}  // namespace vgposp

using namespace vgposp;

extern "C" size_t vgposp_kernel_vjp_workspace_bytes(int64_t n1, int64_t n2, int d) {
  if (n1 <= 0 || n2 <= 0 || d <= 0) return 0;
  int64_t ncb, nrb;
  size_t b;
  vjp_layout(n1, n2, d, &ncb, &nrb, &b);
  return b;
}

extern "C" int vgposp_kernel_vjp(int kind, const double* X1, int64_t n1, const double* X2,
                                 int64_t n2, int d, const double* amp, const double* ls,
                                 const double* Kbar, int64_t ldk, const double* u, const double* w,
                                 double* grad, double* X1bar, void* ws, size_t ws_bytes,
                                 void* stream) {
  clear_error();
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);
  VG_CHECK_ARG(X1 != nullptr, 2);
  VG_CHECK_ARG(n1 >= 1, 3);
  VG_CHECK_ARG(X2 != nullptr, 4);
  VG_CHECK_ARG(n2 >= 1, 5);
  VG_CHECK_ARG(d >= 1 && d <= VJ_MAXD, 6);
  VG_CHECK_ARG(amp != nullptr, 7);
  VG_CHECK_ARG(ls != nullptr, 8);
  VG_CHECK_ARG(Kbar != nullptr, 9);
  VG_CHECK_ARG(ldk >= n2, 10);
  VG_CHECK_ARG((u == nullptr) == (w == nullptr), 11);
  VG_CHECK_ARG(grad != nullptr, 13);
  VG_CHECK_ARG(ws != nullptr, 15);
  int64_t ncb, nrb;
  size_t need;
  vjp_layout(n1, n2, d, &ncb, &nrb, &need);
  if (ws_bytes < need) {
    set_error("vgposp_kernel_vjp: workspace %zu < %zu bytes", ws_bytes, need);
    return VGPOSP_E_WS;
  }
  double* px = static_cast<double*>(ws);
  double* pg = px + ncb * n1 * d;
  hipStream_t s = as_stream(stream);
  dim3 g((unsigned)ncb, (unsigned)nrb);
  {
    ProfScope ps("kernel_vjp", s, 0.0, 8.0 * ((double)n1 * n2 + (double)(n1 + n2) * d));
    switch (kind) {
      case VGPOSP_KERNEL_EQ: launch_vjp<VGPOSP_KERNEL_EQ>(g, s, d, X1, n1, X2, n2, amp, ls, Kbar, ldk, u, w, X1bar ? px : nullptr, pg); break;
      case VGPOSP_KERNEL_MATERN12: launch_vjp<VGPOSP_KERNEL_MATERN12>(g, s, d, X1, n1, X2, n2, amp, ls, Kbar, ldk, u, w, X1bar ? px : nullptr, pg); break;
      case VGPOSP_KERNEL_MATERN32: launch_vjp<VGPOSP_KERNEL_MATERN32>(g, s, d, X1, n1, X2, n2, amp, ls, Kbar, ldk, u, w, X1bar ? px : nullptr, pg); break;
      default: launch_vjp<VGPOSP_KERNEL_MATERN52>(g, s, d, X1, n1, X2, n2, amp, ls, Kbar, ldk, u, w, X1bar ? px : nullptr, pg); break;
    }
    VG_LAUNCH_CHECK();
  }
  return kernel_vjp_reduce_launch(n1, d, ncb, ncb * nrb, px, pg, grad, X1bar, s);
}
