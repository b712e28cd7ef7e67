// Greedy mutual-information sensor placement, dense-exact, all on device.
//
// The reference (placement_algorithm2.py:151-219) evaluates, per candidate y,
//   nom_y   = sigma_yy - Sigma_yA pinv(Sigma_AA) Sigma_Ay                 (:371-388)
//   denom_y = sigma_yy - Sigma_yAbar pinv(Sigma_AbarAbar) Sigma_Abary     (:408-413)
// with an SVD pinv of an (N-|A|-1)^2 matrix per evaluation.  Here both are maintained for ALL
// candidates incrementally:
//   * Sigma = L L^T is factored once and inverted in the same sweep (potrf.hip): M = L^-1 in the
//     lower triangle, Sigma kept in the strictly upper triangle, diag(Sigma) saved.
//   * nom: rank-1 Cholesky rows W (W[t] = L_AA^-1 Sigma_{A,:} row t): nom_y -= w_y^2.
//   * denom = 1 / P_yy with P = (Sigma_SS)^-1, S = V \ A.  P_yy starts at Q_yy = |M e_y|^2 and is
//     downdated per selection with q = Q e_a = M^T (M e_a) (one triangular mat-vec, the HBM-bound
//     step) through rows V (V[t] = L_{Q_AA}^-1 Q_{A,:}): P_yy -= v_y^2.
// The lazy cache policy is emulated exactly: fresh deltas are computed for every candidate, every
// stale entry whose key exceeds the best fresh key is refreshed in bulk (the reference would refresh
// all of them before it could stop), and the remaining re-score loop runs in one workgroup over
// per-chunk maxima.  Keys order by value, ties by LOWER index (argmax_cache_linear, :53-67).
#include <algorithm>
#include <cfloat>

#include "common.h"

namespace vgposp {

int potrf_one(double* A, int64_t n, int64_t lda, int invert, double* diag_out, int* info,
              void* ws, hipStream_t stream, bool early = false);
size_t potrf_ws_bytes(int64_t n);
int partial_inverse(double* A, int64_t n, int64_t lda, int64_t c0, int64_t c1, double* tmp,
                    void* ws, hipStream_t s);
size_t partial_inverse_tmp_bytes(int64_t n, int64_t c0, int64_t c1);

constexpr int RC = 512;     // rows per chunk of the transposed mat-vec
constexpr int CT = 256;     // columns per mat-vec workgroup
constexpr int CH = 1024;    // candidates per chunk / per update workgroup
constexpr int MAXCH = 2048; // chunks held in LDS by the select kernel -> n <= 2^21
constexpr double DELTA_EPS = 1e-8;  // placement_algorithm2.py:198

// Variant parameters, written by vgposp_greedy_init_ex into the workspace (device memory) so the
// per-round entry points keep their signatures:
//   prm[0] jitter  eps added to the diagonal of Sigma_AA and Sigma_AbarAbar (0 for
//                  placement_algorithm2.py; 1e-6 for snippets_a2.tf_nominator :161-163)
//   prm[1] thr     |nom| or |denom| below thr -> delta = 0 (1e-8 at :198; 1e-7 at snippets_a2 :480)
//   prm[2] cinit   initial lazy-cache value (+inf at :164; INF = 1e8 at snippets_a2 :690)
struct GreedyWS {
  double *prm, *sdiag, *nom, *prec, *delta, *cache, *W, *V, *part, *xcol, *piv, *fval, *cval;
  long long *fidx, *cidx, *cnt;
  unsigned char *fresh, *selmask;
  size_t bytes;
};

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

static GreedyWS greedy_layout(void* base, int64_t n, int kmax) {
  GreedyWS w{};
  const int64_t nrc = ceil_div(n, RC), nch = ceil_div(n, CH);
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p ? p + off : nullptr;
    off += align_up(bytes);
    return r;
  };
  w.prm = (double*)take(8 * 8);
  w.sdiag = (double*)take(n * 8);
  w.nom = (double*)take(n * 8);
  w.prec = (double*)take(n * 8);
  w.delta = (double*)take(n * 8);
  w.cache = (double*)take(n * 8);
  w.W = (double*)take((size_t)kmax * n * 8);
  w.V = (double*)take((size_t)kmax * n * 8);
  w.part = (double*)take((size_t)nrc * n * 8);
  w.xcol = (double*)take(n * 8);
  w.piv = (double*)take((2 + 2 * (size_t)kmax) * 8);
  w.fval = (double*)take(nch * 8);
  w.fidx = (long long*)take(nch * 8);
  w.cval = (double*)take(nch * 8);
  w.cidx = (long long*)take(nch * 8);
  w.cnt = (long long*)take(8 * 8);
  w.fresh = (unsigned char*)take(n);
  w.selmask = (unsigned char*)take(n);
  (void)take(potrf_ws_bytes(n));  // factorization scratch (last)
  w.bytes = off;
  return w;
}

static void* greedy_fact_ws(void* base, const GreedyWS& w, int64_t n) {
  return static_cast<char*>(base) + w.bytes - align_up(potrf_ws_bytes(n));
}

// Block-wide (value, index) arg-max for blockDim == 1024.  Result valid in all threads.
__device__ __forceinline__ void block_keymax(double& v, long long& i) {
  __shared__ double sv[16];
  __shared__ long long si[16];
  wave_keymax(v, i);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) {
    sv[w] = v;
    si[w] = i;
  }
  __syncthreads();
  const int nw = blockDim.x >> 6;
  v = (l < nw) ? sv[l] : -DBL_MAX;
  i = (l < nw) ? si[l] : -1;
  wave_keymax(v, i);  // every wave reduces the same 16 entries
}

// Saves diag(Sigma), shifts the diagonal by the jitter (the factorization is of Sigma + eps I:
// the inverse of Sigma_SS + eps I is the Schur complement of the A block of (Sigma + eps I)^-1),
// and fills the cache with its initial value.
__global__ void greedy_init_kernel(double* S, int64_t n, int64_t lda, double jitter, double thr,
                                   double cinit, GreedyWS w) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const double d = S[i * lda + i];
    w.sdiag[i] = d;
    if (jitter != 0.0) S[i * lda + i] = d + jitter;
    w.cache[i] = cinit;
    w.selmask[i] = 0;
  }
  if (i < 8) w.cnt[i] = 0;
  if (i == 0) {
    w.prm[0] = jitter;
    w.prm[1] = thr;
    w.prm[2] = cinit;
  }
}

// x = M e_a restricted to rows >= a (the selected column of L^-1), a = selected[round-1].  With a
// partitioned inverse only the owner of column a holds it: the others write zeros (the caller
// sum-all-reduces xcol), i.e. the column is taken only when a is in [own0, own1).
__global__ void greedy_extract_kernel(const double* M, int64_t n, int64_t lda,
                                      const int64_t* selected, int round, double* xcol,
                                      int64_t own0, int64_t own1) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t a = selected[round - 1];
  const bool own = a >= own0 && a < own1;
  if (r < n) xcol[r] = (own && r >= a) ? M[r * lda + a] : 0.0;
}

// part[rc][c] = sum_{r in chunk rc, r >= max(c, a)} M[r][c] * f(r, c)
//   SQ: f = M[r][c]          (column norms: Q_cc = |M e_c|^2)
//   else f = xcol[r]          (q = M^T x)
// Each thread owns a column pair (one 16-byte load per row, non-temporal: L^-1 is streamed once
// per round), four rows in flight; the pair's diagonal row contributes to its first column only.
constexpr int TRMV_COLS = 2 * CT;  // columns per workgroup

template <bool SQ>
__device__ __forceinline__ double trmv_f(double m, const double* xcol, int64_t r) {
  return SQ ? m * m : m * xcol[r];
}

template <bool SQ>
__global__ __launch_bounds__(CT) void greedy_trmv_kernel(const double* M, int64_t n, int64_t lda,
                                                         const int64_t* selected, int round,
                                                         const double* xcol, double* part,
                                                         int64_t cbeg, int64_t cend, int vec) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  const int64_t cb = (cbeg & ~(int64_t)1) + (int64_t)blockIdx.x * TRMV_COLS;
  const int64_t r0 = (int64_t)blockIdx.y * RC;
  const int64_t r1 = min(r0 + RC, n);
  if (cb >= r1) return;  // tile strictly above the diagonal: never read by the reducer
  const int64_t a = SQ ? 0 : selected[round - 1];
  const int64_t c = cb + 2 * threadIdx.x;
  if (c >= cend) return;
  const bool two = c + 1 < cend;
  double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;  // column c: s, column c + 1: t
  int64_t r = max(max(r0, a), c);
  if (r == c && r < r1) {  // diagonal of column c; (c, c + 1) is above the diagonal
    s0 += trmv_f<SQ>(M[r * lda + c], xcol, r);
    ++r;
  }
  const double* p = M + r * lda + c;
  if (vec && c + 1 < n) {
    for (; r + 3 < r1; r += 4, p += 4 * lda) {
      const d2v m0 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
      const d2v m1 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p + lda));
      const d2v m2 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p + 2 * lda));
      const d2v m3 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p + 3 * lda));
      s0 += trmv_f<SQ>(m0.x, xcol, r) + trmv_f<SQ>(m2.x, xcol, r + 2);
      s1 += trmv_f<SQ>(m1.x, xcol, r + 1) + trmv_f<SQ>(m3.x, xcol, r + 3);
      t0 += trmv_f<SQ>(m0.y, xcol, r) + trmv_f<SQ>(m2.y, xcol, r + 2);
      t1 += trmv_f<SQ>(m1.y, xcol, r + 1) + trmv_f<SQ>(m3.y, xcol, r + 3);
    }
    for (; r < r1; ++r, p += lda) {
      const d2v m0 = *reinterpret_cast<const d2v*>(p);
      s0 += trmv_f<SQ>(m0.x, xcol, r);
      t0 += trmv_f<SQ>(m0.y, xcol, r);
    }
  } else {
    for (; r < r1; ++r, p += lda) {
      s0 += trmv_f<SQ>(p[0], xcol, r);
      if (c + 1 < n) t0 += trmv_f<SQ>(p[1], xcol, r);
    }
  }
  if (c >= cbeg) part[blockIdx.y * n + c] = s0 + s1;
  if (two) part[blockIdx.y * n + c + 1] = t0 + t1;
}

// denom = conditional variance of y given V \ (A u {y}) with eps on that block's diagonal:
// 1 / [(Sigma_SS + eps I)^-1]_yy - eps (Sherman-Morrison on the y entry of the jitter).
__device__ __forceinline__ double delta_of(double nom, double prec, double eps, double thr) {
  const double den = 1.0 / prec - eps;
  if (fabs(den) < thr || fabs(nom) < thr) return 0.0;  // :198 / snippets_a2.py:440-487
  return nom / den;
}

// Round 0: nom = diag(Sigma), prec = Q_ii.  Round t>0: rank-1 updates with a = selected[t-1].
// Then delta for every unselected candidate and per-workgroup best fresh key.
__global__ __launch_bounds__(CH) void greedy_update_kernel(const double* S, int64_t n, int64_t lda,
                                                           const int64_t* selected, int round,
                                                           GreedyWS w, int64_t cbeg, int64_t cend) {
  const int64_t i = (cbeg / CH + (int64_t)blockIdx.x) * CH + threadIdx.x;
  const double eps = w.prm[0], thr = w.prm[1];
  if (i >= cbeg && i < cend) {
    const int64_t nrc = (n + RC - 1) / RC;
    double q = 0.0;
    if (round == 0) {
      for (int64_t rc = i / RC; rc < nrc; ++rc) q += w.part[rc * n + i];
      w.prec[i] = q;
      w.nom[i] = w.sdiag[i];
    } else {
      const int64_t a = selected[round - 1];
      const int t1 = round - 1;  // new row index in W / V
      for (int64_t rc = max(i, a) / RC; rc < nrc; ++rc) q += w.part[rc * n + i];
      double s = (i < a) ? S[i * lda + a] : (i > a ? S[a * lda + i] : w.sdiag[a]);
      for (int t = 0; t < t1; ++t) {
        s -= w.piv[2 + t] * w.W[(int64_t)t * n + i];
        q -= w.piv[2 + t1 + t] * w.V[(int64_t)t * n + i];
      }
      // pivot of the Cholesky of Sigma_AA + eps I: nom_a + eps
      const double noma = w.piv[0] + eps, preca = w.piv[1];
      const double wy = noma > 0.0 ? s / sqrt(noma) : 0.0;
      const double vy = preca > 0.0 ? q / sqrt(preca) : 0.0;
      w.W[(int64_t)t1 * n + i] = wy;
      w.V[(int64_t)t1 * n + i] = vy;
      w.nom[i] -= wy * wy;
      w.prec[i] -= vy * vy;
    }
    if (!w.selmask[i]) w.delta[i] = delta_of(w.nom[i], w.prec[i], eps, thr);
  }
}

// Best fresh key F* per workgroup over all candidates (delta is complete on every rank here).
__global__ __launch_bounds__(CH) void greedy_fresh_max_kernel(int64_t n, GreedyWS w) {
  const int64_t i = (int64_t)blockIdx.x * CH + threadIdx.x;
  double bv = -DBL_MAX;
  long long bi = -1;
  if (i < n && !w.selmask[i]) {
    bv = w.delta[i];
    bi = i;
  }
  block_keymax(bv, bi);
  if (threadIdx.x == 0) {
    w.fval[blockIdx.x] = bv;
    w.fidx[blockIdx.x] = bi;
  }
}

// Reduce the nf per-workgroup keys in `val/idx` (all threads get the result).
__device__ __forceinline__ void reduce_keys(const double* val, const long long* idx, int64_t nf,
                                            double& v, long long& i) {
  v = -DBL_MAX;
  i = -1;
  for (int64_t e = threadIdx.x; e < nf; e += blockDim.x) {
    // idx < 0: a chunk with no candidate left (wave_keymax returns (0.0, -1) for it); it must not
    // enter the comparison, or its 0.0 would shut out a real candidate with a value <= 0
    if (idx[e] >= 0 && key_gt(val[e], idx[e], v, i)) {
      v = val[e];
      i = idx[e];
    }
  }
  block_keymax(v, i);
}

// Bulk refresh: stale entries with key > best fresh key F* are re-scored (guaranteed by the
// reference's loop before it can stop), then per-chunk maxima of the cache.
__global__ __launch_bounds__(CH) void greedy_refresh_kernel(int64_t n, GreedyWS w) {
  const int64_t nch = (n + CH - 1) / CH;
  double fv;
  long long fi;
  reduce_keys(w.fval, w.fidx, nch, fv, fi);
  const int64_t i = (int64_t)blockIdx.x * CH + threadIdx.x;
  double bv = -DBL_MAX;
  long long bi = -1;
  int refreshed = 0;
  if (i < n && !w.selmask[i]) {
    double c = w.cache[i];
    if (key_gt(c, i, fv, fi)) {
      c = w.delta[i];
      w.cache[i] = c;
      w.fresh[i] = 1;
      refreshed = 1;
    } else {
      w.fresh[i] = 0;
    }
    bv = c;
    bi = i;
  }
  // count refreshes (one atomic per wave)
  unsigned long long ball = __ballot(refreshed);
  if ((threadIdx.x & 63) == 0 && ball) atomicAdd((unsigned long long*)&w.cnt[0], (unsigned long long)__popcll(ball));
  block_keymax(bv, bi);
  if (threadIdx.x == 0) {
    w.cval[blockIdx.x] = bv;
    w.cidx[blockIdx.x] = bi;
  }
}

// ---- placement algorithm 3 (snippets_a3.py:43-330): the cache is refreshed only inside the
// index-space window around the last pick; entries outside keep their stale values. ----

// Round 0 (snippets_a3.py:67-119): every candidate is scored once, cache = delta.
__global__ __launch_bounds__(CH) void greedy_cache_all_kernel(int64_t n, GreedyWS w) {
  const int64_t i = (int64_t)blockIdx.x * CH + threadIdx.x;
  if (i < n) w.cache[i] = w.selmask[i] ? 0.0 : w.delta[i];
  if (i == 0) w.cnt[0] = n;
}

// Rounds >= 1 (:196-318): for (j0, j1, j2) in [i - cutoff, i + cutoff) clipped to the grid
// (upper bound exclusive, as the reference's while loops), cache[yj] = delta[yj] or 0 for yj in A;
// cache[y*] = 0.  cnt[0] = number of window entries (the reference's body_D calls).
__global__ __launch_bounds__(256) void greedy_window_kernel(const int64_t* selected, int round,
                                                            int64_t I0, int64_t I1, int64_t I2,
                                                            int cutoff, GreedyWS w) {
  const int64_t a = selected[round - 1];
  const int64_t s0 = I1 * I2;
  const int64_t i0 = a / s0, i1 = (a - i0 * s0) / I2, i2 = a - i0 * s0 - i1 * I2;
  const int64_t lo0 = max(i0 - cutoff, (int64_t)0), hi0 = min(i0 + cutoff, I0);
  const int64_t lo1 = max(i1 - cutoff, (int64_t)0), hi1 = min(i1 + cutoff, I1);
  const int64_t lo2 = max(i2 - cutoff, (int64_t)0), hi2 = min(i2 + cutoff, I2);
  const int64_t W0 = max(hi0 - lo0, (int64_t)0), W1 = max(hi1 - lo1, (int64_t)0),
                W2 = max(hi2 - lo2, (int64_t)0);
  const int64_t total = W0 * W1 * W2;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j0 = lo0 + t / (W1 * W2), r = t % (W1 * W2);
    const int64_t j1 = lo1 + r / W2, j2 = lo2 + r % W2;
    const int64_t yj = j0 * s0 + j1 * I2 + j2;
    w.cache[yj] = w.selmask[yj] ? 0.0 : w.delta[yj];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.cache[a] = 0.0;
    w.cnt[0] = total;
  }
}

// Per-chunk maxima of the cache over unselected candidates (sparse_argmax_cache_linear, :24-50).
__global__ __launch_bounds__(CH) void greedy_cache_max_kernel(int64_t n, GreedyWS w) {
  const int64_t i = (int64_t)blockIdx.x * CH + threadIdx.x;
  double bv = -DBL_MAX;
  long long bi = -1;
  if (i < n && !w.selmask[i]) {
    bv = w.cache[i];
    bi = i;
  }
  block_keymax(bv, bi);
  if (threadIdx.x == 0) {
    w.fval[blockIdx.x] = bv;
    w.fidx[blockIdx.x] = bi;
  }
}

// One workgroup: the remaining re-score loop of placement_algorithm2.py:183-208, then selection.
// mode: 0 = full greedy (placement_algorithm_1), 1 = lazy (placement_algorithm_2),
//       2 = window (placement algorithm 3: arg-max of the cache maxima in fval / fidx).
__global__ __launch_bounds__(CH) void greedy_select_kernel(int64_t n, int round, int mode,
                                                           int64_t* selected, double* sel_delta,
                                                           int64_t* evals, GreedyWS w,
                                                           int64_t cbeg, int64_t cend) {
  __shared__ double cv[MAXCH];
  __shared__ long long ci[MAXCH];
  __shared__ long long ychosen;
  const int64_t nch = (n + CH - 1) / CH;
  double v;
  long long y = -1;
  long long loop_evals = 0;
  const bool lazy = mode == 1;
  if (!lazy) {
    reduce_keys(w.fval, w.fidx, nch, v, y);
  } else {
    for (int64_t c = threadIdx.x; c < nch; c += blockDim.x) {
      cv[c] = w.cval[c];
      ci[c] = w.cidx[c];
    }
    __syncthreads();
    for (int64_t it = 0; it <= n; ++it) {
      reduce_keys(cv, ci, nch, v, y);
      if (y < 0) break;
      if (w.fresh[y]) break;  // arg-max is up to date -> select (:187-189)
      // re-score y (:193-208) and recompute its chunk maximum
      const double dy = w.delta[y];
      __syncthreads();
      if (threadIdx.x == 0) {
        w.cache[y] = dy;
        w.fresh[y] = 1;
      }
      ++loop_evals;
      __syncthreads();
      const int64_t c = y / CH;
      const int64_t j = c * CH + threadIdx.x;
      double bv = -DBL_MAX;
      long long bi = -1;
      if (j < n && !w.selmask[j]) {
        bv = (j == y) ? dy : w.cache[j];
        bi = j;
      }
      block_keymax(bv, bi);
      if (threadIdx.x == 0) {
        cv[c] = bv;
        ci[c] = bi;
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) ychosen = y;
  __syncthreads();
  y = ychosen;
  if (y < 0) {
    if (threadIdx.x == 0) {
      selected[round] = -1;
      if (sel_delta) sel_delta[round] = 0.0;
    }
    return;
  }
  // pivot data for the next update: nom_y, P_yy, W[0..round)[y], V[0..round)[y].  Only the rank
  // owning y's candidate slab holds them; the others write zeros (summed across ranks).
  const bool own = y >= cbeg && y < cend;
  if (threadIdx.x == 0) {
    selected[round] = y;
    if (sel_delta) sel_delta[round] = mode == 2 ? w.cache[y] : w.delta[y];
    if (evals) evals[round] = mode != 0 ? w.cnt[0] + loop_evals : n - round;
    w.cnt[0] = 0;
    w.selmask[y] = 1;
    w.piv[0] = own ? w.nom[y] : 0.0;
    w.piv[1] = own ? w.prec[y] : 0.0;
  }
  for (int t = threadIdx.x; t < round; t += blockDim.x) {
    w.piv[2 + t] = own ? w.W[(int64_t)t * n + y] : 0.0;
    w.piv[2 + round + t] = own ? w.V[(int64_t)t * n + y] : 0.0;
  }
}

}  // namespace vgposp

using namespace vgposp;

extern "C" size_t vgposp_greedy_workspace_bytes(int64_t n, int kmax) {
  if (n <= 0 || kmax <= 0) return 0;
  return greedy_layout(nullptr, n, kmax).bytes;
}

extern "C" int vgposp_greedy_init_ex(double* Sigma, int64_t n, int64_t lda, int kmax,
                                     double jitter, double threshold, double cache_init, int* info,
                                     void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(Sigma != nullptr, 1);
  VG_CHECK_ARG(n >= 1 && n <= (int64_t)MAXCH * CH, 2);
  VG_CHECK_ARG(lda >= n, 3);
  VG_CHECK_ARG(kmax >= 1 && kmax <= n, 4);
  VG_CHECK_ARG(jitter >= 0.0 && jitter < 1e300, 5);
  VG_CHECK_ARG(threshold >= 0.0, 6);
  VG_CHECK_ARG(cache_init == cache_init, 7);
  VG_CHECK_ARG(info != nullptr, 8);
  VG_CHECK_ARG(ws != nullptr, 9);
  GreedyWS w = greedy_layout(ws, n, kmax);
  if (ws_bytes < w.bytes) {
    set_error("vgposp_greedy_init: workspace %zu < %zu bytes", ws_bytes, w.bytes);
    return VGPOSP_E_WS;
  }
  hipStream_t s = as_stream(stream);
  VG_HIP(vg_memset(info, 0, sizeof(int), s));
  hipLaunchKernelGGL(greedy_init_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, Sigma,
                     n, lda, jitter, threshold, cache_init, w);
  VG_LAUNCH_CHECK();
  // early: after a failed pivot (a singular cov_vv) every later launch of the factorization and
  // inverse reads `info` on the device and exits, so the host's jitter retry does not pay for a
  // whole O(n^3) factorization + inverse first — and nothing here synchronises the host
  int rc = potrf_one(Sigma, n, lda, /*invert=*/1, nullptr, info, greedy_fact_ws(ws, w, n), s,
                     /*early=*/true);
  if (rc) return rc;
  // Q_ii = |M e_i|^2 -> part (reduced in the round-0 update)
  dim3 g((unsigned)ceil_div(n, TRMV_COLS), (unsigned)ceil_div(n, RC));
  const int vec = (reinterpret_cast<uintptr_t>(Sigma) % 16 == 0) && (lda % 2 == 0);
  ProfScope ps("greedy_colsq", s, (double)n * (n + 1), 8.0 * (0.5 * (double)n * (n + 1) + (double)ceil_div(n, RC) * n));
  hipLaunchKernelGGL(greedy_trmv_kernel<true>, g, dim3(CT), 0, s, Sigma, n, lda, nullptr, 0,
                     nullptr, w.part, (int64_t)0, n, vec);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_greedy_init(double* Sigma, int64_t n, int64_t lda, int kmax, int* info,
                                  void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(info != nullptr, 5);  // argument numbers of this signature
  VG_CHECK_ARG(ws != nullptr, 6);
  return vgposp_greedy_init_ex(Sigma, n, lda, kmax, 0.0, DELTA_EPS, __builtin_huge_val(), info,
                               ws, ws_bytes, stream);
}

static int greedy_check(const char* fn, const double* Sigma, int64_t n, int64_t lda, int kmax,
                        int round, void* ws, size_t ws_bytes, GreedyWS* w) {
  if (Sigma == nullptr) { set_error("%s: bad argument 1", fn); return -1; }
  if (!(n >= 1 && n <= (int64_t)MAXCH * CH)) { set_error("%s: bad argument 2", fn); return -2; }
  if (lda < n) { set_error("%s: bad argument 3", fn); return -3; }
  if (!(kmax >= 1 && kmax <= n)) { set_error("%s: bad argument 4", fn); return -4; }
  if (!(round >= 0 && round < kmax)) { set_error("%s: bad argument 5", fn); return -5; }
  if (ws == nullptr) { set_error("%s: workspace is null", fn); return VGPOSP_E_WS; }
  *w = greedy_layout(ws, n, kmax);
  if (ws_bytes < w->bytes) {
    set_error("%s: workspace %zu < %zu bytes", fn, ws_bytes, w->bytes);
    return VGPOSP_E_WS;
  }
  return 0;
}

extern "C" int vgposp_greedy_update_ex(const double* Sigma, int64_t n, int64_t lda, int kmax,
                                       int round, int64_t c0, int64_t c1, const int64_t* selected,
                                       int extract, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  GreedyWS w;
  int rc = greedy_check(__func__, Sigma, n, lda, kmax, round, ws, ws_bytes, &w);
  if (rc) return rc;
  VG_CHECK_ARG(c0 >= 0 && c0 <= c1 && c1 <= n, 6);
  VG_CHECK_ARG(selected != nullptr || round == 0, 8);
  hipStream_t s = as_stream(stream);
  if (c1 == c0) return 0;
  if (round > 0) {
    if (extract) {
      hipLaunchKernelGGL(greedy_extract_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                         Sigma, n, lda, selected, round, w.xcol, (int64_t)0, n);
      VG_LAUNCH_CHECK();
    }
    dim3 g((unsigned)ceil_div(c1 - (c0 & ~(int64_t)1), TRMV_COLS), (unsigned)ceil_div(n, RC));
    const int vec = (reinterpret_cast<uintptr_t>(Sigma) % 16 == 0) && (lda % 2 == 0);
    // algorithmic: the lower triangle of L^-1 in rows >= a, columns [c0, c1) (a is device-side;
    // bench.py recomputes the exact bytes from the selections)
    ProfScope ps("greedy_trmv", s, 0.0, 8.0 * (0.5 * (double)n * (n + 1) + 2.0 * n));
    hipLaunchKernelGGL(greedy_trmv_kernel<false>, g, dim3(CT), 0, s, Sigma, n, lda, selected,
                       round, w.xcol, w.part, c0, c1, vec);
    VG_LAUNCH_CHECK();
  }
  {
    ProfScope psu("greedy_update", s, 0.0, 8.0 * (double)(c1 - c0) * (6 + 2.0 * round));
    const int64_t b0 = c0 / CH, b1 = ceil_div(c1, CH);
    // grid covers the CH-aligned blocks spanning [c0, c1); blockIdx is offset by b0
    hipLaunchKernelGGL(greedy_update_kernel, dim3((unsigned)(b1 - b0)), dim3(CH), 0, s, Sigma, n,
                       lda, selected, round, w, c0, c1);
    VG_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int vgposp_greedy_update(const double* Sigma, int64_t n, int64_t lda, int kmax,
                                    int round, int64_t c0, int64_t c1, const int64_t* selected,
                                    void* ws, size_t ws_bytes, void* stream) {
  return vgposp_greedy_update_ex(Sigma, n, lda, kmax, round, c0, c1, selected, 1, ws, ws_bytes,
                                 stream);
}

extern "C" int vgposp_greedy_extract(const double* Sigma, int64_t n, int64_t lda, int kmax,
                                     int round, int64_t own0, int64_t own1,
                                     const int64_t* selected, void* ws, size_t ws_bytes,
                                     void* stream) {
  clear_error();
  GreedyWS w;
  int rc = greedy_check(__func__, Sigma, n, lda, kmax, round, ws, ws_bytes, &w);
  if (rc) return rc;
  VG_CHECK_ARG(round >= 1, 5);
  VG_CHECK_ARG(own0 >= 0 && own0 <= own1 && own1 <= n, 6);
  VG_CHECK_ARG(selected != nullptr, 8);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(greedy_extract_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                     Sigma, n, lda, selected, round, w.xcol, own0, own1);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t vgposp_greedy_slab_tmp_bytes(int64_t n, int64_t c0, int64_t c1) {
  if (n <= 0 || c0 < 0 || c1 <= c0 || c1 > n) return 0;
  return partial_inverse_tmp_bytes(n, c0, c1);
}

static int check_prepare(const char* fn, double* Sigma, int64_t n, int64_t lda, int kmax,
                         double jitter, double threshold, double cache_init, int* info, void* ws,
                         size_t ws_bytes, GreedyWS* w) {
  if (Sigma == nullptr) { set_error("%s: bad argument 1", fn); return -1; }
  if (!(n >= 1 && n <= (int64_t)MAXCH * CH)) { set_error("%s: bad argument 2", fn); return -2; }
  if (lda < n) { set_error("%s: bad argument 3", fn); return -3; }
  if (!(kmax >= 1 && kmax <= n)) { set_error("%s: bad argument 4", fn); return -4; }
  if (!(jitter >= 0.0 && jitter < 1e300)) { set_error("%s: bad argument 5", fn); return -5; }
  if (!(threshold >= 0.0)) { set_error("%s: bad argument 6", fn); return -6; }
  if (cache_init != cache_init) { set_error("%s: bad argument 7", fn); return -7; }
  if (info == nullptr) { set_error("%s: info is null", fn); return -8; }
  if (ws == nullptr) { set_error("%s: workspace is null", fn); return VGPOSP_E_WS; }
  *w = greedy_layout(ws, n, kmax);
  if (ws_bytes < w->bytes) {
    set_error("%s: workspace %zu < %zu bytes", fn, ws_bytes, w->bytes);
    return VGPOSP_E_WS;
  }
  return 0;
}

extern "C" int vgposp_greedy_prepare(double* Sigma, int64_t n, int64_t lda, int kmax,
                                     double jitter, double threshold, double cache_init, int* info,
                                     void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  GreedyWS w;
  if (int rc = check_prepare(__func__, Sigma, n, lda, kmax, jitter, threshold, cache_init, info,
                             ws, ws_bytes, &w))
    return rc;
  hipStream_t s = as_stream(stream);
  VG_HIP(vg_memset(info, 0, sizeof(int), s));
  hipLaunchKernelGGL(greedy_init_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, Sigma,
                     n, lda, jitter, threshold, cache_init, w);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_greedy_fact_ws(void* ws, int64_t n, int kmax, void** fws,
                                     size_t* fws_bytes) {
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(kmax >= 1, 3);
  VG_CHECK_ARG(fws != nullptr && fws_bytes != nullptr, 4);
  GreedyWS w = greedy_layout(ws, n, kmax);
  *fws = greedy_fact_ws(ws, w, n);
  *fws_bytes = potrf_ws_bytes(n);
  return 0;
}

extern "C" int vgposp_greedy_finish_slab(double* Sigma, int64_t n, int64_t lda, int kmax,
                                         int64_t c0, int64_t c1, double* tmp, size_t tmp_bytes,
                                         void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(Sigma != nullptr, 1);
  VG_CHECK_ARG(n >= 1 && n <= (int64_t)MAXCH * CH, 2);
  VG_CHECK_ARG(lda >= n, 3);
  VG_CHECK_ARG(kmax >= 1 && kmax <= n, 4);
  VG_CHECK_ARG(c0 >= 0 && c0 <= c1 && c0 % 128 == 0, 5);
  VG_CHECK_ARG(c1 <= n && (c1 % 128 == 0 || c1 == n), 6);
  VG_CHECK_ARG(c1 == c0 || (tmp != nullptr && tmp_bytes >= partial_inverse_tmp_bytes(n, c0, c1)),
               7);
  VG_CHECK_ARG(ws != nullptr, 9);
  GreedyWS w = greedy_layout(ws, n, kmax);
  if (ws_bytes < w.bytes) {
    set_error("vgposp_greedy_finish_slab: workspace %zu < %zu bytes", ws_bytes, w.bytes);
    return VGPOSP_E_WS;
  }
  if (c1 == c0) return 0;
  hipStream_t s = as_stream(stream);
  int rc = partial_inverse(Sigma, n, lda, c0, c1, tmp, greedy_fact_ws(ws, w, n), s);
  if (rc) return rc;
  // Q_ii = |M e_i|^2 for the slab's columns -> part (reduced in the round-0 update)
  dim3 g((unsigned)ceil_div(c1 - (c0 & ~(int64_t)1), TRMV_COLS), (unsigned)ceil_div(n, RC));
  const int vec = (reinterpret_cast<uintptr_t>(Sigma) % 16 == 0) && (lda % 2 == 0);
  ProfScope ps("greedy_colsq", s, 0.0, 0.0);
  hipLaunchKernelGGL(greedy_trmv_kernel<true>, g, dim3(CT), 0, s, Sigma, n, lda, nullptr, 0,
                     nullptr, w.part, c0, c1, vec);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_greedy_init_slab(double* Sigma, int64_t n, int64_t lda, int kmax,
                                       double jitter, double threshold, double cache_init,
                                       int64_t c0, int64_t c1, double* tmp, size_t tmp_bytes,
                                       int* info, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VG_CHECK_ARG(c0 >= 0 && c0 <= c1 && c0 % 128 == 0, 8);
  VG_CHECK_ARG(c1 <= n && (c1 % 128 == 0 || c1 == n), 9);
  VG_CHECK_ARG(c1 == c0 || (tmp != nullptr && tmp_bytes >= partial_inverse_tmp_bytes(n, c0, c1)),
               10);
  int rc = vgposp_greedy_prepare(Sigma, n, lda, kmax, jitter, threshold, cache_init, info, ws,
                                 ws_bytes, stream);
  if (rc) return rc;
  GreedyWS w = greedy_layout(ws, n, kmax);
  if ((rc = potrf_one(Sigma, n, lda, /*invert=*/0, nullptr, info, greedy_fact_ws(ws, w, n),
                      as_stream(stream))))
    return rc;
  return vgposp_greedy_finish_slab(Sigma, n, lda, kmax, c0, c1, tmp, tmp_bytes, ws, ws_bytes,
                                   stream);
}

extern "C" int vgposp_greedy_xcol(void* ws, int64_t n, int kmax, double** xcol) {
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(kmax >= 1, 3);
  VG_CHECK_ARG(xcol != nullptr, 4);
  *xcol = greedy_layout(ws, n, kmax).xcol;
  return 0;
}

extern "C" int vgposp_greedy_select(int64_t n, int kmax, int round, int lazy, int64_t c0,
                                    int64_t c1, int64_t* selected, double* sel_delta,
                                    int64_t* evals, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  GreedyWS w;
  double dummy = 0.0;
  int rc = greedy_check(__func__, &dummy, n, n, kmax, round, ws, ws_bytes, &w);
  if (rc) return rc;
  VG_CHECK_ARG(c0 >= 0 && c0 <= c1 && c1 <= n, 5);
  VG_CHECK_ARG(selected != nullptr, 7);
  hipStream_t s = as_stream(stream);
  const unsigned nch = (unsigned)ceil_div(n, CH);
  hipLaunchKernelGGL(greedy_fresh_max_kernel, dim3(nch), dim3(CH), 0, s, n, w);
  VG_LAUNCH_CHECK();
  if (lazy) {
    ProfScope psr("greedy_refresh", s, 0.0, 8.0 * 3.0 * n);
    hipLaunchKernelGGL(greedy_refresh_kernel, dim3(nch), dim3(CH), 0, s, n, w);
    VG_LAUNCH_CHECK();
  }
  ProfScope pss("greedy_select", s, 0.0, 0.0);
  hipLaunchKernelGGL(greedy_select_kernel, dim3(1), dim3(CH), 0, s, n, round, lazy ? 1 : 0,
                     selected, sel_delta, evals, w, c0, c1);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_greedy_select_window(int64_t n, int kmax, int round, int64_t I0, int64_t I1,
                                           int64_t I2, int cutoff, int64_t c0, int64_t c1,
                                           int64_t* selected, double* sel_delta, int64_t* evals,
                                           void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  GreedyWS w;
  double dummy = 0.0;
  int rc = greedy_check(__func__, &dummy, n, n, kmax, round, ws, ws_bytes, &w);
  if (rc) return rc;
  VG_CHECK_ARG(I0 >= 1 && I1 >= 1 && I2 >= 1 && I0 * I1 * I2 == n, 4);
  VG_CHECK_ARG(cutoff >= 0, 7);
  VG_CHECK_ARG(c0 >= 0 && c0 <= c1 && c1 <= n, 8);
  VG_CHECK_ARG(selected != nullptr, 10);
  hipStream_t s = as_stream(stream);
  const unsigned nch = (unsigned)ceil_div(n, CH);
  {
    ProfScope psw("greedy_window", s, 0.0, 0.0);
    if (round == 0) {
      hipLaunchKernelGGL(greedy_cache_all_kernel, dim3(nch), dim3(CH), 0, s, n, w);
    } else {
      const int64_t span = 2 * (int64_t)cutoff;
      const int64_t total = span * span * span;
      const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 4096));
      hipLaunchKernelGGL(greedy_window_kernel, dim3(g), dim3(256), 0, s, selected, round, I0, I1,
                         I2, cutoff, w);
    }
    VG_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(greedy_cache_max_kernel, dim3(nch), dim3(CH), 0, s, n, w);
  VG_LAUNCH_CHECK();
  ProfScope pss("greedy_select", s, 0.0, 0.0);
  hipLaunchKernelGGL(greedy_select_kernel, dim3(1), dim3(CH), 0, s, n, round, 2, selected,
                     sel_delta, evals, w, c0, c1);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_greedy_step(const double* Sigma, int64_t n, int64_t lda, int kmax, int round,
                                  int lazy, int64_t* selected, double* sel_delta, int64_t* evals,
                                  void* ws, size_t ws_bytes, void* stream) {
  int rc = vgposp_greedy_update(Sigma, n, lda, kmax, round, 0, n, selected, ws, ws_bytes, stream);
  if (rc) return rc;
  return vgposp_greedy_select(n, kmax, round, lazy, 0, n, selected, sel_delta, evals, ws, ws_bytes,
                              stream);
}

extern "C" int vgposp_greedy_buffers(void* ws, int64_t n, int kmax, double** delta, double** piv,
                                     int64_t* piv_len) {
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(kmax >= 1, 3);
  GreedyWS w = greedy_layout(ws, n, kmax);
  if (delta) *delta = w.delta;
  if (piv) *piv = w.piv;
  if (piv_len) *piv_len = 2 + 2 * (int64_t)kmax;
  return 0;
}

extern "C" int vgposp_greedy_cache(void* ws, int64_t n, int kmax, double** cache) {
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(kmax >= 1, 3);
  VG_CHECK_ARG(cache != nullptr, 4);
  *cache = greedy_layout(ws, n, kmax).cache;
  return 0;
}

namespace vgposp {
__global__ void greedy_exclude_kernel(unsigned char* selmask, int64_t idx) { selmask[idx] = 1; }
}  // namespace vgposp

extern "C" int vgposp_greedy_exclude(void* ws, int64_t n, int kmax, int64_t idx, void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(kmax >= 1, 3);
  VG_CHECK_ARG(idx >= 0 && idx < n, 4);
  GreedyWS w = greedy_layout(ws, n, kmax);
  hipLaunchKernelGGL(greedy_exclude_kernel, dim3(1), dim3(1), 0, as_stream(stream), w.selmask, idx);
  VG_LAUNCH_CHECK();
  return 0;
}
