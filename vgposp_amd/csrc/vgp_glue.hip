// The element-wise and reduction glue of the VGP training step (vgposp_amd/vgp_training.py):
// everything of the reference's variational_loss + its TF gradient
// (variational_Gaussian_process_example.py:51-102) that is not a GEMM, a factorization, a kernel
// assembly or a kernel VJP.  Each was a chain of small framework kernels (and one-element kernels
// for every scalar); here each phase is one launch over M x M (or M) data that sits in L2:
//   vgp_sinv     P0 (lower) -> symmetric in place, Sinv = Kzz + P0 / s + pj I (+ the Kzz
//                matrices factored in the same batch)
//   sym_lower    A (lower) -> symmetric in place
//   lincomb      out = sum_k c_k (s + shift)^e_k X_k  (+ a diagonal term), M x M or vectors
//   vgp_kzz_bar  the adjoint of Kzz (symmetrised, as the Kzz VJP wants it) and G = (2/s) Sinv_bar
//   dots         up to 16 dot products / sums of logs / traces, deterministic two-pass
//   vgp_scalars  loss, d/damp, d/dls, d/dnoise from those sums (negated: the minimised loss)
// All scalars that depend on trained values (s, amp) are read on device: no host sync in the step.
#include <cmath>

#include "common.h"

namespace vgposp {

constexpr int DOT_BLOCKS = 512;  // partial sums per dot product (16.7M-entry products need them)
constexpr int MAX_DOTS = 16;
constexpr int MAX_TERMS = 4;

__global__ __launch_bounds__(256) void vgp_sinv_kernel(int64_t n, double* P0, int64_t ld,
                                                       const double* Kzz, const double* s,
                                                       double pj, double jitter, double* F,
                                                       int nf) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * n) return;
  const int64_t i = e / n, j = e - i * n;
  const double p = j <= i ? P0[i * ld + j] : P0[j * ld + i];
  const double k = Kzz[i * n + j];
  double v = k + p / s[0];
  if (i == j) v += pj;
  F[e] = v;
  if (nf == 4) {  // the three Kzz-only matrices the step factors in the same batch
    F[n * n + e] = i == j ? k + jitter : k;
    F[2 * n * n + e] = i == j ? k + (s[0] + 1e-6) : k;
    F[3 * n * n + e] = k;
  }
  if (j > i) P0[i * ld + j] = p;  // only the strict upper triangle is written, only lower read
}

__global__ __launch_bounds__(256) void sym_lower_kernel(int64_t n, double* A, int64_t ld) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * n) return;
  const int64_t i = e / n, j = e - i * n;
  if (j > i) A[i * ld + j] = A[j * ld + i];
}

struct LinComb {
  const double* x[MAX_TERMS];
  double c[MAX_TERMS];
  int e[MAX_TERMS];
  int nterms;
  double diag_c;
  int diag_e;
  double diag_scale;
};

__device__ __forceinline__ double ipow(double b, int e) {
  double r = 1.0;
  const double f = e < 0 ? 1.0 / b : b;
  for (int k = e < 0 ? -e : e; k > 0; --k) r *= f;
  return r;
}

// out[i][j] = sum_k (c_k * base^e_k) * X_k[i][j], on i == j times diag_scale plus
// diag_c base^diag_e; base = s + shift
__global__ __launch_bounds__(256) void lincomb_kernel(int64_t rows, int64_t cols, int64_t ld,
                                                      LinComb lc, const double* s, double shift,
                                                      double* out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * cols) return;
  const int64_t i = e / cols, j = e - i * cols;
  const double base = s ? s[0] + shift : 1.0;
  double v = 0.0;
  for (int k = 0; k < lc.nterms; ++k) {
    const double f = lc.e[k] ? lc.c[k] * ipow(base, lc.e[k]) : lc.c[k];
    v += f * lc.x[k][i * ld + j];
  }
  if (i == j) {
    v *= lc.diag_scale;
    if (lc.diag_c != 0.0) v += lc.diag_c * (lc.diag_e ? ipow(base, lc.diag_e) : 1.0);
  }
  out[i * ld + j] = v;
}

struct KzzBar {
  const double *u, *v, *qv, *mb, *t, *cb;                            // [n]
  const double *HHt, *PHH, *Kpinv, *QAQA, *Kzzinv, *LiLi, *Sc, *LiA;  // [n][n]
};

// Kbar(i, j) of Kzz (vgp_training.py's reverse pass, term by term) and Sinv_bar(i, j).
__device__ __forceinline__ double sinv_bar(const KzzBar& a, int64_t n, int64_t i, int64_t j,
                                           double w) {
  const int64_t ij = i * n + j, ji = j * n + i;
  return -0.5 * w * a.LiLi[ij] - 0.5 * (a.cb[i] * a.t[j] + a.t[i] * a.cb[j]) +
         0.5 * (a.Sc[ij] + a.Sc[ji]);
}

__device__ __forceinline__ double kzz_bar(const KzzBar& a, int64_t n, int64_t i, int64_t j,
                                          double w, double si) {
  const int64_t ij = i * n + j;
  const double kpb = -0.5 * w * (a.Kpinv[ij] - a.qv[i] * a.qv[j] - a.QAQA[ij]);
  return -a.u[i] * a.v[j] - (0.5 * si) * a.HHt[ij] + si * a.PHH[ij] + kpb + w * a.Kzzinv[ij] +
         a.mb[i] * a.t[j] * si + sinv_bar(a, n, i, j, w) + a.LiA[ij];
}

__global__ __launch_bounds__(256) void vgp_kzz_bar_kernel(int64_t n, KzzBar a, const double* s,
                                                          double w, double* KzzS, double* G) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * n) return;
  const int64_t i = e / n, j = e - i * n;
  const double si = 1.0 / s[0];
  KzzS[e] = kzz_bar(a, n, i, j, w, si) + kzz_bar(a, n, j, i, w, si);
  G[e] = (2.0 * si) * sinv_bar(a, n, i, j, w);
}

struct Dots {
  const double* x[MAX_DOTS];
  const double* y[MAX_DOTS];
  int64_t incx[MAX_DOTS], incy[MAX_DOTS], len[MAX_DOTS];
  int op[MAX_DOTS];  // 0: sum x*y (y null: sum x), 1: sum log(x)
};

__global__ __launch_bounds__(256) void dots_partial_kernel(Dots d, double* part) {
  __shared__ double red[4];
  const int p = blockIdx.y;
  const int64_t n = d.len[p];
  const double* x = d.x[p];
  const double* y = d.y[p];
  const int64_t incx = d.incx[p], incy = d.incy[p], st = (int64_t)DOT_BLOCKS * 256;
  const int op = d.op[p];
  auto term = [&](int64_t i) {
    const double xv = x[i * incx];
    return op == 1 ? log(xv) : (y ? xv * y[i * incy] : xv);
  };
  // four independent chains: a 16.7M-entry product is 128 terms per thread
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    a0 += term(i);
    a1 += term(i + st);
    a2 += term(i + 2 * st);
    a3 += term(i + 3 * st);
  }
  for (; i < n; i += st) a0 += term(i);
  double acc = (a0 + a1) + (a2 + a3);
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[p * DOT_BLOCKS + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// one wave per dot product, fixed summation order
__global__ __launch_bounds__(1024) void dots_final_kernel(int np, const double* part, double* out) {
  const int p = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (p >= np) return;
  double v = 0.0;
  for (int b = lane; b < DOT_BLOCKS; b += 64) v += part[p * DOT_BLOCKS + b];
  v = wave_sum(v);
  if (lane == 0) out[p] = v;
}

// The ELBO E and the scalar adjoints (see vgp_training.py for the derivation), from the sums
// S[VGP_S_*] of vgposp.h.  out = (-E, -dE/damp, -dE/dls, -dE/dnoise).
__global__ void vgp_scalars_kernel(const double* S, const double* s_, const double* a_,
                                   const double* g1, const double* g2, const double* g3, double nb,
                                   double M, double w, double j, double* out) {
  if (threadIdx.x != 0) return;
  const double s = s_[0], a = a_[0];
  const double rr = S[VGPOSP_S_RR], s2 = s + j;
  const double obs = -0.5 * rr / s2 - 0.5 * nb * log(2.0 * M_PI * s2);
  const double T = 0.5 * (nb * a * a - S[VGPOSP_S_KZB_H] + S[VGPOSP_S_Q_HHT]) / s;
  const double logdetA = 2.0 * S[VGPOSP_S_LOGDET_K] - S[VGPOSP_S_LOGDET_S];
  const double KL = S[VGPOSP_S_LOGDET_P] - logdetA + 0.5 * (-M + S[VGPOSP_S_PA2] + S[VGPOSP_S_QM2]);
  const double E = obs - T - w * KL;
  const double trKpb = -0.5 * w * (S[VGPOSP_S_TR_KPINV] - S[VGPOSP_S_QV2] - S[VGPOSP_S_TR_QAQA]);
  double sb = 0.5 * rr / (s2 * s2) - 0.5 * nb / s2;
  sb = sb + T / s;
  sb = sb + trKpb;
  sb = sb - S[VGPOSP_S_MB_M] / s;
  sb = sb - 0.5 * S[VGPOSP_S_G_P0] / s;  // <Sinv_bar, P0> / s^2 with G = (2 / s) Sinv_bar
  const double ab = -nb * a / s + 0.5 * g1[0] + g2[0] + g3[0];
  const double lb = 0.5 * g1[1] + g2[1] + g3[1];
  out[0] = -E;
  out[1] = -ab;
  out[2] = -lb;
  out[3] = -sb;
}

static dim3 grid1(int64_t n) { return dim3((unsigned)ceil_div(n, 256)); }

}  // namespace vgposp

using namespace vgposp;

extern "C" int vgposp_vgp_sinv(double* P0, int64_t n, int64_t ldp, const double* Kzz,
                               const double* s, double pj, double jitter, double* F, int nf,
                               void* stream) {
  clear_error();
  VG_CHECK_ARG(P0 != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(ldp >= n, 3);
  VG_CHECK_ARG(Kzz != nullptr, 4);
  VG_CHECK_ARG(s != nullptr, 5);
  VG_CHECK_ARG(F != nullptr, 8);
  VG_CHECK_ARG(nf == 1 || nf == 4, 9);
  hipLaunchKernelGGL(vgp_sinv_kernel, grid1(n * n), dim3(256), 0, as_stream(stream), n, P0, ldp, Kzz,
                     s, pj, jitter, F, nf);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_sym_from_lower(double* A, int64_t n, int64_t lda, void* stream) {
  clear_error();
  VG_CHECK_ARG(A != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(lda >= n, 3);
  hipLaunchKernelGGL(sym_lower_kernel, grid1(n * n), dim3(256), 0, as_stream(stream), n, A, lda);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_lincomb(int64_t rows, int64_t cols, int64_t ld, int nterms,
                              const double* const* X, const double* coef, const int* spow,
                              double diag_scale, double diag_coef, int diag_spow, const double* s,
                              double shift, double* out, void* stream) {
  clear_error();
  VG_CHECK_ARG(rows >= 1, 1);
  VG_CHECK_ARG(cols >= 1, 2);
  VG_CHECK_ARG(ld >= cols, 3);
  VG_CHECK_ARG(nterms >= 0 && nterms <= MAX_TERMS, 4);
  VG_CHECK_ARG(nterms == 0 || (X != nullptr && coef != nullptr && spow != nullptr), 5);
  VG_CHECK_ARG(out != nullptr, 13);
  LinComb lc{};
  lc.nterms = nterms;
  for (int k = 0; k < nterms; ++k) {
    VG_CHECK_ARG(X[k] != nullptr, 5);
    VG_CHECK_ARG(spow[k] == 0 || s != nullptr, 11);
    lc.x[k] = X[k];
    lc.c[k] = coef[k];
    lc.e[k] = spow[k];
  }
  VG_CHECK_ARG(diag_spow == 0 || s != nullptr, 11);
  lc.diag_scale = diag_scale;
  lc.diag_c = diag_coef;
  lc.diag_e = diag_spow;
  hipLaunchKernelGGL(lincomb_kernel, grid1(rows * cols), dim3(256), 0, as_stream(stream), rows, cols,
                     ld, lc, s, shift, out);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_vgp_kzz_bar(int64_t n, const double* const* vecs, const double* const* mats,
                                  const double* s, double w, double* KzzS, double* G,
                                  void* stream) {
  clear_error();
  VG_CHECK_ARG(n >= 1, 1);
  VG_CHECK_ARG(vecs != nullptr, 2);
  VG_CHECK_ARG(mats != nullptr, 3);
  VG_CHECK_ARG(s != nullptr, 4);
  VG_CHECK_ARG(KzzS != nullptr, 6);
  VG_CHECK_ARG(G != nullptr, 7);
  for (int k = 0; k < 6; ++k) VG_CHECK_ARG(vecs[k] != nullptr, 2);
  for (int k = 0; k < 8; ++k) VG_CHECK_ARG(mats[k] != nullptr, 3);
  KzzBar a{vecs[0], vecs[1], vecs[2], vecs[3], vecs[4], vecs[5],
           mats[0], mats[1], mats[2], mats[3], mats[4], mats[5], mats[6], mats[7]};
  hipLaunchKernelGGL(vgp_kzz_bar_kernel, grid1(n * n), dim3(256), 0, as_stream(stream), n, a, s, w,
                     KzzS, G);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t vgposp_dots_workspace_bytes(int ndots) {
  return ndots > 0 ? 8 * (size_t)ndots * DOT_BLOCKS : 0;
}

extern "C" int vgposp_dots(int ndots, const double* const* x, const int64_t* incx,
                           const double* const* y, const int64_t* incy, const int64_t* len,
                           const int* op, double* out, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(ndots >= 1 && ndots <= MAX_DOTS, 1);
  VG_CHECK_ARG(x != nullptr && incx != nullptr && y != nullptr && incy != nullptr, 2);
  VG_CHECK_ARG(len != nullptr, 6);
  VG_CHECK_ARG(op != nullptr, 7);
  VG_CHECK_ARG(out != nullptr, 8);
  VG_CHECK_ARG(ws != nullptr, 9);
  if (ws_bytes < vgposp_dots_workspace_bytes(ndots)) {
    set_error("vgposp_dots: workspace %zu < %zu bytes", ws_bytes, vgposp_dots_workspace_bytes(ndots));
    return VGPOSP_E_WS;
  }
  Dots d{};
  for (int p = 0; p < ndots; ++p) {
    VG_CHECK_ARG(x[p] != nullptr, 2);
    VG_CHECK_ARG(len[p] >= 0, 6);
    VG_CHECK_ARG(op[p] == 0 || op[p] == 1, 7);
    d.x[p] = x[p];
    d.y[p] = y[p];
    d.incx[p] = incx[p];
    d.incy[p] = incy[p];
    d.len[p] = len[p];
    d.op[p] = op[p];
  }
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(dots_partial_kernel, dim3(DOT_BLOCKS, (unsigned)ndots), dim3(256), 0, st, d,
                     part);
  VG_LAUNCH_CHECK();
  hipLaunchKernelGGL(dots_final_kernel, dim3(1), dim3(64 * ndots), 0, st, ndots, part, out);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_vgp_scalars(const double* sums, const double* s, const double* amp,
                                  const double* g1, const double* g2, const double* g3, double nb,
                                  double m, double w, double jitter, double* out, void* stream) {
  clear_error();
  VG_CHECK_ARG(sums != nullptr, 1);
  VG_CHECK_ARG(s != nullptr, 2);
  VG_CHECK_ARG(amp != nullptr, 3);
  VG_CHECK_ARG(g1 != nullptr && g2 != nullptr && g3 != nullptr, 4);
  VG_CHECK_ARG(out != nullptr, 11);
  hipLaunchKernelGGL(vgp_scalars_kernel, dim3(1), dim3(64), 0, as_stream(stream), sums, s, amp, g1,
                     g2, g3, nb, m, w, jitter, out);
  VG_LAUNCH_CHECK();
  return 0;
}
