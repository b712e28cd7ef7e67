// PSD kernel assembly K(X1, X2) — HBM-write-bound (8 B written per entry, ~20-40 fp64 VALU ops for
// the transcendental).  Replaces TFP's `kernel.matrix` for the kernels the reference builds
// (gp_functions.py:160-163 MaternOneHalf, 3D_sin_wave.py:158-159 / main_tests.py:617
// ExponentiatedQuadratic, main_architecture_2_sampledistribution.py:211 MaternFiveHalves), which
// TF evaluates by materialising an [n, m, d] squared-difference tensor.
//
// Layout: each 256-thread workgroup writes a 128-row x 128-column tile; lane pairs of columns are
// stored as one 16-byte write per row so a wave stores 1 KiB contiguous per row.  The X2 columns
// of the tile are held in registers; the tile's X1 rows are staged in LDS once and read back as
// broadcasts (a global load per row put its latency in front of every row's exp and store).
// Formula, as TFP evaluates it:  K = exp(2 log amp + log k(r / ls)).
#include "common.h"
#include "psd.h"

// the MV variant keeps a cross-lane sum inside the unrolled row loop, which blocks the unroll there
#pragma clang diagnostic ignored "-Wpass-failed"

namespace vgposp {

constexpr int KM_ROWS = 128;
constexpr int KM_COLS = 128;
constexpr int KM_MAXD = 8;

__device__ __forceinline__ int km_tri_root(int64_t id) {
  int64_t t = (int64_t)((sqrt(8.0 * (double)id + 1.0) - 1.0) * 0.5);
  while ((t + 1) * (t + 2) / 2 <= id) ++t;
  while (t * (t + 1) / 2 > id) --t;
  return (int)t;
}

// One 128 x 128 tile per workgroup; a lower-triangular launch enumerates only the tiles on or
// below the diagonal (blockIdx.x = ti (ti + 1) / 2 + tj).  Stores are non-temporal: K is far
// larger than the caches and is next read by the factorization.
// MV (full, batch 1): also the tile's share of K v — part[row][column tile] = sum over the tile's
// columns of K[row][col] v[col], one wave sum per row (kernel_matvec_reduce_kernel adds the
// column tiles in a fixed order), so K is never re-read for the product.
template <int KIND, int D, bool MV>
__global__ __launch_bounds__(256) void kernel_matrix_kernel(const double* X1, int64_t n1,
                                                            const double* X2, int64_t n2, int d,
                                                            const double* amp, const double* ls,
                                                            const double* diag_shift, int uplo,
                                                            double* K, int64_t ldk,
                                                            int64_t stride_k, int vec,
                                                            int tri_grid, const double* v = nullptr,
                                                            double* part = nullptr) {
  __shared__ double xs[KM_ROWS * KM_MAXD];  // the tile's X1 rows, read back as LDS broadcasts
  const int b = blockIdx.z;
  int64_t r0, c0;
  if (tri_grid) {
    const int ti = km_tri_root(blockIdx.x);
    r0 = (int64_t)ti * KM_ROWS;
    c0 = (int64_t)(blockIdx.x - ti * (ti + 1) / 2) * KM_COLS;
  } else {
    r0 = (int64_t)blockIdx.y * KM_ROWS;
    c0 = (int64_t)blockIdx.x * KM_COLS;
  }
  const int dd = D > 0 ? D : d;
  const int nrow = (int)min((int64_t)KM_ROWS, n1 - r0);
  for (int e = threadIdx.x; e < nrow * dd; e += 256) xs[e] = X1[r0 * dd + e];
  const double a = amp[b], l = ls[b];
  const double two_log_amp = 2.0 * log(a);
  const double inv_ls = 1.0 / l;
  const double inv_ls2 = 1.0 / (l * l);
  const double shift = diag_shift ? diag_shift[b] : 0.0;
  double* Kb = K + (int64_t)b * stride_k;

  const int tx = threadIdx.x & 63;   // column pair
  const int ty = threadIdx.x >> 6;   // row phase (0..3)
  const int64_t ca = c0 + 2 * tx, cb = ca + 1;
  double xa[KM_MAXD], xb[KM_MAXD];
#pragma unroll
  for (int k = 0; k < KM_MAXD; ++k) {
    xa[k] = (k < dd && ca < n2) ? X2[ca * dd + k] : 0.0;
    xb[k] = (k < dd && cb < n2) ? X2[cb * dd + k] : 0.0;
  }
  const double wa = (MV && ca < n2) ? v[ca] : 0.0, wb = (MV && cb < n2) ? v[cb] : 0.0;
  __syncthreads();
#pragma unroll 4
  for (int i = ty; i < nrow; i += 4) {
    const int64_t r = r0 + i;
    double da = 0.0, db = 0.0;
#pragma unroll
    for (int k = 0; k < KM_MAXD; ++k) {
      if (k < dd) {
        const double xr = xs[i * dd + k];
        const double ea = xr - xa[k], eb = xr - xb[k];
        da += ea * ea;
        db += eb * eb;
      }
    }
    double va = kfun<KIND>(da, two_log_amp, inv_ls, inv_ls2);
    double vb = kfun<KIND>(db, two_log_amp, inv_ls, inv_ls2);
    if (diag_shift) {
      if (ca == r) va += shift;
      if (cb == r) vb += shift;
    }
    double* row = Kb + r * ldk;
    const bool oka = ca < n2 && (uplo != VGPOSP_LOWER || ca <= r);
    const bool okb = cb < n2 && (uplo != VGPOSP_LOWER || cb <= r);
    if (vec && oka && okb) {
      typedef double d2v __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(d2v{va, vb}, reinterpret_cast<d2v*>(row + ca));
    } else {
      if (oka) __builtin_nontemporal_store(va, row + ca);
      if (okb) __builtin_nontemporal_store(vb, row + cb);
    }
    if (MV) {
      const double sum = wave_sum(va * wa + vb * wb);
      if (tx == 0) part[r * gridDim.x + blockIdx.x] = sum;
    }
  }
}

// out[r] = sum over the column tiles of part[r][tile]: one workgroup per row, a fixed summation
// order (deterministic).
__global__ __launch_bounds__(256) void kernel_matvec_reduce_kernel(int64_t ntiles,
                                                                   const double* part, double* out) {
  __shared__ double red[4];
  const int64_t r = blockIdx.x;
  const double* row = part + r * ntiles;
  double s = 0.0;
  for (int64_t t = threadIdx.x; t < ntiles; t += 256) s += row[t];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[r] = (red[0] + red[1]) + (red[2] + red[3]);
}

template <int KIND, bool MV = false>
static void launch_kind(dim3 g, hipStream_t s, const double* X1, int64_t n1, const double* X2,
                        int64_t n2, int d, const double* amp, const double* ls,
                        const double* shift, int uplo, double* K, int64_t ldk, int64_t stride,
                        int vec, int tri_grid, const double* v = nullptr, double* part = nullptr) {
  switch (d) {
    case 1: hipLaunchKernelGGL((kernel_matrix_kernel<KIND, 1, MV>), g, dim3(256), 0, s, X1, n1, X2, n2, d, amp, ls, shift, uplo, K, ldk, stride, vec, tri_grid, v, part); break;
    case 2: hipLaunchKernelGGL((kernel_matrix_kernel<KIND, 2, MV>), g, dim3(256), 0, s, X1, n1, X2, n2, d, amp, ls, shift, uplo, K, ldk, stride, vec, tri_grid, v, part); break;
    case 3: hipLaunchKernelGGL((kernel_matrix_kernel<KIND, 3, MV>), g, dim3(256), 0, s, X1, n1, X2, n2, d, amp, ls, shift, uplo, K, ldk, stride, vec, tri_grid, v, part); break;
    default: hipLaunchKernelGGL((kernel_matrix_kernel<KIND, 0, MV>), g, dim3(256), 0, s, X1, n1, X2, n2, d, amp, ls, shift, uplo, K, ldk, stride, vec, tri_grid, v, part); break;
  }
}

}  // namespace vgposp

using namespace vgposp;

extern "C" int vgposp_kernel_matrix(int kind, const double* X1, int64_t n1, const double* X2,
                                    int64_t n2, int d, const double* amp, const double* ls,
                                    const double* diag_shift, int batch, int uplo, double* K,
                                    int64_t ldk, int64_t stride_k, void* stream) {
  clear_error();
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);
  VG_CHECK_ARG(X1 != nullptr || n1 == 0, 2);
  VG_CHECK_ARG(n1 >= 0, 3);
  VG_CHECK_ARG(X2 != nullptr || n2 == 0, 4);
  VG_CHECK_ARG(n2 >= 0, 5);
  VG_CHECK_ARG(d >= 1 && d <= KM_MAXD, 6);
  VG_CHECK_ARG(amp != nullptr, 7);
  VG_CHECK_ARG(ls != nullptr, 8);
  VG_CHECK_ARG(batch >= 1 && batch <= 65535, 10);
  VG_CHECK_ARG(uplo == VGPOSP_FULL || uplo == VGPOSP_LOWER, 11);
  VG_CHECK_ARG(K != nullptr || n1 == 0 || n2 == 0, 12);
  VG_CHECK_ARG(ldk >= n2, 13);
  VG_CHECK_ARG(batch == 1 || stride_k >= ldk * n1, 14);
  if (n1 == 0 || n2 == 0) return 0;
  // a lower launch is square (n1 == n2 for the symmetric K): only the tiles on or below the diagonal
  const int64_t tr = ceil_div(n1, KM_ROWS);
  dim3 g = (uplo == VGPOSP_LOWER && n1 == n2)
               ? dim3((unsigned)(tr * (tr + 1) / 2), 1u, (unsigned)batch)
               : dim3((unsigned)ceil_div(n2, KM_COLS), (unsigned)tr, (unsigned)batch);
  const int tri_grid = uplo == VGPOSP_LOWER && n1 == n2;
  const int vec = (reinterpret_cast<uintptr_t>(K) % 16 == 0) && (ldk % 2 == 0) &&
                  (batch == 1 || stride_k % 2 == 0);
  hipStream_t s = as_stream(stream);
  const double outs = (uplo == VGPOSP_LOWER) ? 0.5 * (double)n1 * (double)(n1 + 1) : (double)n1 * n2;
  ProfScope ps("kernel_matrix", s, 0.0, 8.0 * (batch * outs + (double)d * (n1 + n2)));
  switch (kind) {
    case VGPOSP_KERNEL_EQ: launch_kind<VGPOSP_KERNEL_EQ>(g, s, X1, n1, X2, n2, d, amp, ls, diag_shift, uplo, K, ldk, stride_k, vec, tri_grid); break;
    case VGPOSP_KERNEL_MATERN12: launch_kind<VGPOSP_KERNEL_MATERN12>(g, s, X1, n1, X2, n2, d, amp, ls, diag_shift, uplo, K, ldk, stride_k, vec, tri_grid); break;
    case VGPOSP_KERNEL_MATERN32: launch_kind<VGPOSP_KERNEL_MATERN32>(g, s, X1, n1, X2, n2, d, amp, ls, diag_shift, uplo, K, ldk, stride_k, vec, tri_grid); break;
    default: launch_kind<VGPOSP_KERNEL_MATERN52>(g, s, X1, n1, X2, n2, d, amp, ls, diag_shift, uplo, K, ldk, stride_k, vec, tri_grid); break;
  }
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t vgposp_kernel_matrix_matvec_workspace_bytes(int64_t n1, int64_t n2) {
  if (n1 <= 0 || n2 <= 0) return 0;
  return 8 * (size_t)(ceil_div(n2, KM_COLS) * n1);
}

extern "C" int vgposp_kernel_matrix_matvec(int kind, const double* X1, int64_t n1,
                                           const double* X2, int64_t n2, int d, const double* amp,
                                           const double* ls, double* K, int64_t ldk,
                                           const double* v, double* out, void* ws, size_t ws_bytes,
                                           void* stream) {
  clear_error();
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);
  VG_CHECK_ARG(X1 != nullptr, 2);
  VG_CHECK_ARG(n1 >= 1, 3);
  VG_CHECK_ARG(X2 != nullptr, 4);
  VG_CHECK_ARG(n2 >= 1, 5);
  VG_CHECK_ARG(d >= 1 && d <= KM_MAXD, 6);
  VG_CHECK_ARG(amp != nullptr, 7);
  VG_CHECK_ARG(ls != nullptr, 8);
  VG_CHECK_ARG(K != nullptr, 9);
  VG_CHECK_ARG(ldk >= n2, 10);
  VG_CHECK_ARG(v != nullptr, 11);
  VG_CHECK_ARG(out != nullptr, 12);
  VG_CHECK_ARG(ws != nullptr, 13);
  const int64_t ntiles = ceil_div(n2, KM_COLS);
  if (ws_bytes < 8 * (size_t)(ntiles * n1)) {
    set_error("vgposp_kernel_matrix_matvec: workspace %zu < %zu bytes", ws_bytes,
              8 * (size_t)(ntiles * n1));
    return VGPOSP_E_WS;
  }
  double* part = static_cast<double*>(ws);
  const dim3 g((unsigned)ntiles, (unsigned)ceil_div(n1, KM_ROWS), 1u);
  const int vec = (reinterpret_cast<uintptr_t>(K) % 16 == 0) && (ldk % 2 == 0);
  hipStream_t s = as_stream(stream);
  {
    ProfScope ps("kernel_matrix", s, 0.0, 8.0 * ((double)n1 * n2 + (double)d * (n1 + n2) + n2));
    switch (kind) {
      case VGPOSP_KERNEL_EQ: launch_kind<VGPOSP_KERNEL_EQ, true>(g, s, X1, n1, X2, n2, d, amp, ls, nullptr, VGPOSP_FULL, K, ldk, 0, vec, 0, v, part); break;
      case VGPOSP_KERNEL_MATERN12: launch_kind<VGPOSP_KERNEL_MATERN12, true>(g, s, X1, n1, X2, n2, d, amp, ls, nullptr, VGPOSP_FULL, K, ldk, 0, vec, 0, v, part); break;
      case VGPOSP_KERNEL_MATERN32: launch_kind<VGPOSP_KERNEL_MATERN32, true>(g, s, X1, n1, X2, n2, d, amp, ls, nullptr, VGPOSP_FULL, K, ldk, 0, vec, 0, v, part); break;
      default: launch_kind<VGPOSP_KERNEL_MATERN52, true>(g, s, X1, n1, X2, n2, d, amp, ls, nullptr, VGPOSP_FULL, K, ldk, 0, vec, 0, v, part); break;
    }
    VG_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(kernel_matvec_reduce_kernel, dim3((unsigned)n1), dim3(256), 0, s, ntiles, part,
                     out);
  VG_LAUNCH_CHECK();
  return 0;
}
