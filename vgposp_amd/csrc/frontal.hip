// Multifrontal Cholesky + selected inverse of the tapered covariance (config C4, exact).
//
// Algorithm 3 (snippets_a3.py:43-364) on the beta-decay tapered cov_vv
// (main_architecture_2_sampledistribution.py:355-421) needs diag((Sigma + eps I)^-1) for every
// candidate (round 0: tf_denominator over V \ {y}, snippets_a2.py:138-218).  Sigma is a sparse SPD
// stencil matrix, so that diagonal comes from a nested-dissection factorization (the symbolic plan
// is vgposp_amd/nested_dissection.py) and the Takahashi recurrences, front by front:
//
//   factor (bottom-up):   F_PP = L L^T,  M = L^-1,  L_UP = F_UP M^T,  F_UU -= L_UP L_UP^T,
//                         W = L_UP M  (= F_UP F_PP^-1)
//   selected inverse:     Q_UU = the parent's Q on U x U,  T = -Q_UU W,  Q_UP = T,
//   (top-down)            Q_PP = M^T M - W^T T
//
// A front is stored as three row-major blocks PP [p][p] (lower), UP [u][p] and UU [u][u]; a group
// of fronts (one tree level) is a strided batch, so every dense step is one batched fp64 MFMA
// launch (gemm.hip) or one batched recursive Cholesky (potrf.hip).  The sparse steps here:
//   front_assemble:   the original entries s(i, j) of the pivot columns, evaluated from the grid
//                     points on the fly (K is never stored)
//   front_extend_add: a child's update F_UU scattered into its parent's front
//   front_gather:     a child's Q_UU read out of its parent's Q front
//   front_diag:       diag(Q_PP) scattered to the pivots' grid indices
#include <cmath>

#include "common.h"
#include "psd.h"

namespace vgposp {

int gemm_launch_batched(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                        const double* A, int64_t lda, int64_t sA, const double* B, int64_t ldb,
                        int64_t sB, double beta, double* C, int64_t ldc, int64_t sC, int uplo_c,
                        int tri_a, int tri_b, int nsplit, double* part, int64_t sP, int batch,
                        hipStream_t stream);
int potrf_batched(double* A, int64_t n, int64_t lda, int64_t sA, int batch, int invert,
                  double* diag_out, int* info, void* ws, hipStream_t stream, bool use_part);
size_t potrf_ws_bytes_opt(int64_t n, bool use_part);

struct TaperArgs {
  const double* X;
  long long I0, I1, I2;
  double tla, inv_ls, inv_ls2, shift, jitter;
  const int* offs;  // [m1][3]
  int m1;
  const double* tau;
  int ntau;
};

static TaperArgs taper_args(const double* X, int64_t I0, int64_t I1, int64_t I2, double amp,
                            double ls, double shift, double jitter, const int* offs, int m,
                            const double* tau, int ntau) {
  return TaperArgs{X, I0, I1, I2, 2.0 * std::log(amp), 1.0 / ls, 1.0 / (ls * ls), shift, jitter,
                   offs, m - 1, tau, ntau};
}

// Lower-triangle element (max(a, b), min(a, b)) of a front stored as PP / UP / UU blocks; positions
// count P first, then U.
__device__ __forceinline__ size_t front_off(int r, int c, int p, int u, int& blk) {
  if (r < p) {
    blk = 0;
    return (size_t)r * p + c;
  }
  if (c < p) {
    blk = 1;
    return (size_t)(r - p) * p + c;
  }
  blk = 2;
  return (size_t)(r - p) * u + (c - p);
}

// One thread per pivot column pj of front blockIdx.y.  Entries with the row in a descendant
// (eliminated earlier) belong to that descendant's front; rows in this front's pivots are written
// only below the diagonal (each pair once); rows in an ancestor are located in the sorted U list.
template <int KIND>
__global__ __launch_bounds__(256) void front_assemble_kernel(
    TaperArgs a, const int* __restrict__ owner_ord, const int* __restrict__ owner_pos,
    const int* __restrict__ piv, int p, const int* __restrict__ U, int u,
    const int* __restrict__ ulen, const int* __restrict__ order, double* PP, double* UP) {
  const int s = blockIdx.y;
  const int pj = blockIdx.x * blockDim.x + threadIdx.x;
  if (pj >= p) return;
  double* pp = PP + (size_t)s * p * p;
  double* up = UP + (size_t)s * u * p;
  const int j = piv[(size_t)s * p + pj];
  if (j < 0) {  // padding pivot: identity
    pp[(size_t)pj * p + pj] = 1.0;
    return;
  }
  const int ord = order[s];
  const int* Us = U + (size_t)s * u;
  const int ul = ulen[s];
  const long long j0 = j / (a.I1 * a.I2), j1 = (j / a.I2) % a.I1, j2 = j % a.I2;
  const double x0 = a.X[3 * (size_t)j], x1 = a.X[3 * (size_t)j + 1], x2 = a.X[3 * (size_t)j + 2];
  pp[(size_t)pj * p + pj] = a.tau[0] * (kfun<KIND>(0.0, a.tla, a.inv_ls, a.inv_ls2) + a.shift) + a.jitter;
  for (int o = 0; o < a.m1; ++o) {
    const int o0 = a.offs[3 * o], o1 = a.offs[3 * o + 1], o2 = a.offs[3 * o + 2];
    const long long i0 = j0 + o0, i1 = j1 + o1, i2 = j2 + o2;
    if (i0 < 0 || i0 >= a.I0 || i1 < 0 || i1 >= a.I1 || i2 < 0 || i2 >= a.I2) continue;
    const int d2i = o0 * o0 + o1 * o1 + o2 * o2;
    if (d2i >= a.ntau) continue;
    const double t = a.tau[d2i];
    if (t == 0.0) continue;
    const int i = (int)((i0 * a.I1 + i1) * a.I2 + i2);
    const int oi = owner_ord[i];
    if (oi < ord) continue;  // a descendant's pivot: assembled in its front
    const double d0 = a.X[3 * (size_t)i] - x0, d1 = a.X[3 * (size_t)i + 1] - x1,
                 d2 = a.X[3 * (size_t)i + 2] - x2;
    const double v = t * kfun<KIND>(d0 * d0 + d1 * d1 + d2 * d2, a.tla, a.inv_ls, a.inv_ls2);
    if (oi == ord) {
      const int pi = owner_pos[i];
      if (pi > pj) pp[(size_t)pi * p + pj] = v;
    } else {
      int lo = 0, hi = ul;  // first k with Us[k] >= i
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (Us[mid] < i) lo = mid + 1;
        else hi = mid;
      }
      if (lo < ul && Us[lo] == i) up[(size_t)lo * p + pj] = v;
    }
  }
}

constexpr int XT = 64;  // square tile of the scatter / gather kernels (64 x 4 threads)

// Parent front += child's update (lower triangle) for the children of sibling index `sib`
// (siblings share a parent, so the two sibling passes never write the same parent concurrently).
// Child s's parent front sits at element offsets par_off[s] of the parent LEVEL's PP / UP / UU
// buffers, with padded sizes par_dim[s] = (p, u).
__global__ __launch_bounds__(256) void front_extend_add_kernel(
    const double* __restrict__ UUc, int uc, const int* __restrict__ pmap,
    const long long* __restrict__ par_off, const int* __restrict__ par_dim,
    const int* __restrict__ sibl, int sib, double* PP, double* UP, double* UU) {
  const int s = blockIdx.z;
  if (sibl[s] != sib) return;
  const int bx = blockIdx.x, by = blockIdx.y;
  if (bx > by) return;
  const int b = bx * XT + (threadIdx.x & (XT - 1));
  if (b >= uc) return;
  const int* m = pmap + (size_t)s * uc;
  const int mb = m[b];
  if (mb < 0) return;
  const double* src = UUc + (size_t)s * uc * uc;
  const int p = par_dim[2 * s], u = par_dim[2 * s + 1];
  double* base[3] = {PP + par_off[3 * s], UP + par_off[3 * s + 1], UU + par_off[3 * s + 2]};
  const int a1 = min(uc, (by + 1) * XT);
  for (int aa = by * XT + (threadIdx.x >> 6); aa < a1; aa += 4) {
    if (aa < b) continue;
    const int ma = m[aa];
    if (ma < 0) continue;
    const double v = src[(size_t)aa * uc + b];
    if (v == 0.0) continue;
    int blk;
    const size_t off = front_off(max(ma, mb), min(ma, mb), p, u, blk);
    base[blk][off] += v;
  }
}

// Child's full Q_UU [uc][uc] <- its parent's Q front at (pmap[a], pmap[b]); 0 on padding.
// Q_UU is symmetric: one workgroup per 64 x 64 tile pair on or below the diagonal reads the lower
// tile once and writes it and its mirror (transposed through LDS), so both stores are coalesced.
__global__ __launch_bounds__(256) void front_gather_kernel(
    const double* __restrict__ QPP, const double* __restrict__ QUP, const double* __restrict__ QUU,
    const int* __restrict__ pmap, const long long* __restrict__ par_off,
    const int* __restrict__ par_dim, int uc, double* __restrict__ out) {
  __shared__ double tile[XT][XT + 1];
  const int s = blockIdx.z;
  const int bx = blockIdx.x, by = blockIdx.y;
  if (bx > by) return;
  const int tx = threadIdx.x & (XT - 1), ty = threadIdx.x >> 6;
  const int* m = pmap + (size_t)s * uc;
  const int p = par_dim[2 * s], u = par_dim[2 * s + 1];
  const double* base[3] = {QPP + par_off[3 * s], QUP + par_off[3 * s + 1],
                           QUU + par_off[3 * s + 2]};
  double* dst = out + (size_t)s * uc * uc;
  const int b = bx * XT + tx;
  const int mb = b < uc ? m[b] : -1;
  for (int i = ty; i < XT; i += 4) {
    const int aa = by * XT + i;
    double v = 0.0;
    if (aa < uc) {
      const int ma = m[aa];
      if (ma >= 0 && mb >= 0) {
        int blk;
        const size_t off = front_off(max(ma, mb), min(ma, mb), p, u, blk);
        v = base[blk][off];
      }
      if (b < uc) dst[(size_t)aa * uc + b] = v;
    }
    tile[i][tx] = v;
  }
  if (bx == by) return;
  __syncthreads();
  // mirror: rows bx * 64 + i, columns by * 64 + tx
  for (int i = ty; i < XT; i += 4) {
    const int r = bx * XT + i, c = by * XT + tx;
    if (r < uc && c < uc) dst[(size_t)r * uc + c] = tile[tx][i];
  }
}

__global__ void front_diag_kernel(const double* __restrict__ QPP, int p, int nf,
                                  const int* __restrict__ piv, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)p * nf) return;
  const int s = (int)(e / p), k = (int)(e % p);
  const int j = piv[e];
  if (j >= 0) out[j] = QPP[(size_t)s * p * p + (size_t)k * p + k];
}

static size_t falign(size_t x) { return (x + 255) & ~(size_t)255; }

// Large batches fill the GPU through the batch dimension; only a few large fronts (the top of the
// tree) need the recursion's split-K partials.
static bool front_use_part(int nf) { return nf <= 4; }

size_t front_factor_ws(int64_t p, int64_t u, int nf) {
  return falign(potrf_ws_bytes_opt(p, front_use_part(nf)) * nf) + falign(8 * (size_t)u * p * nf);
}

}  // namespace vgposp

using namespace vgposp;

extern "C" size_t vgposp_front_factor_workspace_bytes(int64_t p, int64_t u, int nf) {
  if (p <= 0 || u < 0 || nf <= 0) return 0;
  return front_factor_ws(p, u, nf);
}

extern "C" int vgposp_front_factor(double* PP, double* UP, double* UU, int64_t p, int64_t u, int nf,
                                   int* info, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(PP != nullptr, 1);
  VG_CHECK_ARG(u == 0 || UP != nullptr, 2);
  VG_CHECK_ARG(u == 0 || UU != nullptr, 3);
  VG_CHECK_ARG(p >= 1 && p % 2 == 0, 4);
  VG_CHECK_ARG(u >= 0 && u % 2 == 0, 5);
  VG_CHECK_ARG(nf >= 1 && nf <= 65535, 6);
  VG_CHECK_ARG(info != nullptr, 7);
  VG_CHECK_ARG(ws != nullptr, 8);
  if (ws_bytes < front_factor_ws(p, u, nf)) {
    set_error("vgposp_front_factor: workspace %zu < %zu bytes", ws_bytes, front_factor_ws(p, u, nf));
    return VGPOSP_E_WS;
  }
  hipStream_t s = as_stream(stream);
  VG_HIP(vg_memset(info, 0, sizeof(int) * nf, s));
  const bool part = front_use_part(nf);
  char* w = static_cast<char*>(ws);
  double* tmp = reinterpret_cast<double*>(w + falign(potrf_ws_bytes_opt(p, part) * nf));
  // M = F_PP^-1's lower factor inverse, in place
  if (int rc = potrf_batched(PP, p, p, p * p, nf, 1, nullptr, info, ws, s, part)) return rc;
  if (u == 0) return 0;
  int rc;
  // L_UP = F_UP M^T  (M stored lower)
  if ((rc = gemm_launch_batched(0, 1, u, p, p, 1.0, UP, p, u * p, PP, p, p * p, 0.0, tmp, p, u * p,
                                VGPOSP_FULL, 0, 1, 1, nullptr, 0, nf, s)))
    return rc;
  // F_UU -= L_UP L_UP^T  (lower)
  if ((rc = gemm_launch_batched(0, 1, u, u, p, -1.0, tmp, p, u * p, tmp, p, u * p, 1.0, UU, u, u * u,
                                VGPOSP_LOWER, 0, 0, 1, nullptr, 0, nf, s)))
    return rc;
  // W = L_UP M
  return gemm_launch_batched(0, 0, u, p, p, 1.0, tmp, p, u * p, PP, p, p * p, 0.0, UP, p, u * p,
                             VGPOSP_FULL, 0, 1, 1, nullptr, 0, nf, s);
}

extern "C" int vgposp_front_selinv(const double* M, const double* W, const double* QUU, int64_t p,
                                   int64_t u, int nf, double* QPP, double* QUP, void* stream) {
  clear_error();
  VG_CHECK_ARG(M != nullptr, 1);
  VG_CHECK_ARG(u == 0 || W != nullptr, 2);
  VG_CHECK_ARG(u == 0 || QUU != nullptr, 3);
  VG_CHECK_ARG(p >= 1 && p % 2 == 0, 4);
  VG_CHECK_ARG(u >= 0 && u % 2 == 0, 5);
  VG_CHECK_ARG(nf >= 1 && nf <= 65535, 6);
  VG_CHECK_ARG(QPP != nullptr && QPP != M, 7);
  VG_CHECK_ARG(u == 0 || (QUP != nullptr && QUP != W), 8);
  hipStream_t s = as_stream(stream);
  int rc;
  // Q_PP = M^T M  (both operands lower triangular)
  if ((rc = gemm_launch_batched(1, 0, p, p, p, 1.0, M, p, p * p, M, p, p * p, 0.0, QPP, p, p * p,
                                VGPOSP_LOWER, 1, 1, 1, nullptr, 0, nf, s)))
    return rc;
  if (u == 0) return 0;
  // T = -Q_UU W
  if ((rc = gemm_launch_batched(0, 0, u, p, u, -1.0, QUU, u, u * u, W, p, u * p, 0.0, QUP, p, u * p,
                                VGPOSP_FULL, 0, 0, 1, nullptr, 0, nf, s)))
    return rc;
  // Q_PP -= W^T T
  return gemm_launch_batched(1, 0, p, p, u, -1.0, W, p, u * p, QUP, p, u * p, 1.0, QPP, p, p * p,
                             VGPOSP_LOWER, 0, 0, 1, nullptr, 0, nf, s);
}

extern "C" int vgposp_front_assemble(int kind, const double* X, int64_t I0, int64_t I1, int64_t I2,
                                     double amp, double ls, double diag_shift, double jitter,
                                     const int* offsets, int m, const double* tau, int ntau,
                                     const int* owner_ord, const int* owner_pos, const int* piv,
                                     int64_t p, const int* U, int64_t u, const int* ulen,
                                     const int* order, int nf, double* PP, double* UP,
                                     void* stream) {
  clear_error();
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);
  VG_CHECK_ARG(X != nullptr, 2);
  VG_CHECK_ARG(I0 >= 1 && I1 >= 1 && I2 >= 1 && I0 * I1 * I2 < (int64_t)INT32_MAX, 3);
  VG_CHECK_ARG(amp > 0.0, 6);
  VG_CHECK_ARG(ls > 0.0, 7);
  VG_CHECK_ARG(m >= 1 && (m == 1 || offsets != nullptr), 12);
  VG_CHECK_ARG(tau != nullptr && ntau >= 1, 13);
  VG_CHECK_ARG(owner_ord != nullptr && owner_pos != nullptr, 15);
  VG_CHECK_ARG(piv != nullptr, 17);
  VG_CHECK_ARG(p >= 1, 18);
  VG_CHECK_ARG(u == 0 || (U != nullptr && ulen != nullptr), 19);
  VG_CHECK_ARG(order != nullptr, 22);
  VG_CHECK_ARG(nf >= 1 && nf <= 65535, 23);
  VG_CHECK_ARG(PP != nullptr && (u == 0 || UP != nullptr), 24);
  hipStream_t s = as_stream(stream);
  TaperArgs a = taper_args(X, I0, I1, I2, amp, ls, diag_shift, jitter, offsets, m, tau, ntau);
  ProfScope ps("front_assemble", s, 0.0, 8.0 * (double)nf * p * m);
  dim3 g((unsigned)ceil_div(p, 256), (unsigned)nf);
  switch (kind) {
    case VGPOSP_KERNEL_EQ:
      hipLaunchKernelGGL(front_assemble_kernel<VGPOSP_KERNEL_EQ>, g, dim3(256), 0, s, a, owner_ord,
                         owner_pos, piv, (int)p, U, (int)u, ulen, order, PP, UP);
      break;
    case VGPOSP_KERNEL_MATERN12:
      hipLaunchKernelGGL(front_assemble_kernel<VGPOSP_KERNEL_MATERN12>, g, dim3(256), 0, s, a,
                         owner_ord, owner_pos, piv, (int)p, U, (int)u, ulen, order, PP, UP);
      break;
    case VGPOSP_KERNEL_MATERN32:
      hipLaunchKernelGGL(front_assemble_kernel<VGPOSP_KERNEL_MATERN32>, g, dim3(256), 0, s, a,
                         owner_ord, owner_pos, piv, (int)p, U, (int)u, ulen, order, PP, UP);
      break;
    default:
      hipLaunchKernelGGL(front_assemble_kernel<VGPOSP_KERNEL_MATERN52>, g, dim3(256), 0, s, a,
                         owner_ord, owner_pos, piv, (int)p, U, (int)u, ulen, order, PP, UP);
  }
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_front_extend_add(const double* UUc, int64_t uc, int nfc, const int* pmap,
                                       const int64_t* par_off, const int* par_dim,
                                       const int* sibling, int sib, double* PP, double* UP,
                                       double* UU, void* stream) {
  clear_error();
  VG_CHECK_ARG(UUc != nullptr || uc == 0, 1);
  VG_CHECK_ARG(uc >= 0, 2);
  VG_CHECK_ARG(nfc >= 1 && nfc <= 65535, 3);
  VG_CHECK_ARG(pmap != nullptr, 4);
  VG_CHECK_ARG(par_off != nullptr && par_dim != nullptr, 5);
  VG_CHECK_ARG(sibling != nullptr, 7);
  VG_CHECK_ARG(PP != nullptr, 9);
  if (uc == 0) return 0;
  hipStream_t s = as_stream(stream);
  ProfScope ps("front_extend_add", s, 0.0, 8.0 * 2.0 * nfc * uc * (double)uc);
  const unsigned t = (unsigned)ceil_div(uc, XT);
  hipLaunchKernelGGL(front_extend_add_kernel, dim3(t, t, (unsigned)nfc), dim3(256), 0, s, UUc,
                     (int)uc, pmap, reinterpret_cast<const long long*>(par_off), par_dim, sibling,
                     sib, PP, UP, UU);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_front_gather(const double* QPP, const double* QUP, const double* QUU,
                                   const int* pmap, const int64_t* par_off, const int* par_dim,
                                   int nfc, int64_t uc, double* QUUc, void* stream) {
  clear_error();
  VG_CHECK_ARG(QPP != nullptr, 1);
  VG_CHECK_ARG(pmap != nullptr, 4);
  VG_CHECK_ARG(par_off != nullptr && par_dim != nullptr, 5);
  VG_CHECK_ARG(nfc >= 1 && nfc <= 65535, 7);
  VG_CHECK_ARG(uc >= 0, 8);
  VG_CHECK_ARG(QUUc != nullptr || uc == 0, 9);
  if (uc == 0) return 0;
  hipStream_t s = as_stream(stream);
  ProfScope ps("front_gather", s, 0.0, 8.0 * 2.0 * nfc * uc * (double)uc);
  const unsigned t = (unsigned)ceil_div(uc, XT);
  hipLaunchKernelGGL(front_gather_kernel, dim3(t, t, (unsigned)nfc), dim3(256), 0, s, QPP, QUP, QUU,
                     pmap, reinterpret_cast<const long long*>(par_off), par_dim, (int)uc, QUUc);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_front_diag(const double* QPP, int64_t p, int nf, const int* piv, double* out,
                                 void* stream) {
  clear_error();
  VG_CHECK_ARG(QPP != nullptr, 1);
  VG_CHECK_ARG(p >= 1, 2);
  VG_CHECK_ARG(nf >= 1, 3);
  VG_CHECK_ARG(piv != nullptr, 4);
  VG_CHECK_ARG(out != nullptr, 5);
  hipStream_t s = as_stream(stream);
  const int64_t n = p * nf;
  hipLaunchKernelGGL(front_diag_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, QPP,
                     (int)p, nf, piv, out);
  VG_LAUNCH_CHECK();
  return 0;
}
