// Exact algorithm 3 on the sparse tapered covariance (config C4): the rounds.
//
// snippets_a3.sparse_placement_algorithm_3 (snippets_a3.py:43-364) re-scores, after each pick y*,
// the candidates of the index window [i_d - cutoff, i_d + cutoff) around y* with tf_nominator /
// tf_denominator over the FULL sets (snippets_a2.py:138-218, eps = 1e-6 on the conditioning
// block's diagonal):
//   nom_y   = s_yy - s_yA (S_AA + eps I)^-1 s_Ay
//   denom_y = s_yy - s_yB (S_BB + eps I)^-1 s_By,  B = V \ (A u {y})
//           = 1 / P_yy - eps,  P = ((S + eps I)_SS)^-1, S = V \ A,
//   P_yy    = Q_yy - Q_yA Q_AA^-1 Q_Ay,  Q = (S + eps I)^-1            (block inverse of Q)
// Q_yy comes from the multifrontal selected inverse (frontal.hip).  Each pick a adds one column
// q_a = Q e_a, from conjugate gradients on the stencil matrix (S + eps I: SPD, its coefficients
// are tabulated once per problem, [N][m]).  The conditioning blocks grow by one row per pick:
// LS = chol(S_AA + eps I) and LQ = chol(Q_AA), so a re-scored candidate costs two |A|-long
// forward substitutions.
//
// Arg-max: (value, index) keys per 256-entry block of the cache and per 64-block superblock; a
// window touches a few dozen blocks, so a round reads kilobytes, not the 16 MB cache.  Keys order by
// value, ties to the LOWER index (placement_algorithm2.py:24-50).
//
// Every launch only enqueues work: the pick lives in device memory (picks[round]) and every
// later kernel reads it there, so the whole run is free of host synchronisation.
#include <cmath>

#include "common.h"
#include "psd.h"

namespace vgposp {

constexpr int EB = 256;      // cache entries per block key
constexpr int ESB = 64;      // blocks per superblock key
constexpr int CG_BLOCKS = 1024;
constexpr int CG_T = 256;
constexpr int SEL_THREADS = 1024;

struct ExactWS {
  double* coef;       // [n][m]: coef[i][0] diagonal (S_ii + eps), coef[i][1 + o] = S(i, i + off_o)
  double* bval;       // [nblk]
  long long* bidx;
  double* sval;       // [nsb]
  long long* sidx;
  // CG on the box of half-width H around the pick (clipped into the grid): the Krylov vectors of
  // a solve of S e_a are exactly zero beyond H = iterations x stencil radius, so the box holds
  // every non-zero of the full-grid iteration.  Box-local vectors, [bv] each.
  double* r;          // residual
  double* p0;         // directions (two, alternating)
  double* p1;
  double* q;          // A p
  long long* boxlo;   // [kmax][3] box origin of each pick's column
  long long b0, b1, b2, H;
  double* part_pq;    // [CG_BLOCKS]
  double* part_rr;    // [CG_BLOCKS]
  double* rr;         // [maxit + 2] residual norms per iteration
  int* cgstate;       // [4]: done flag, iterations of the last solve
  double* LS;         // [kmax][kmax] chol(S_AA + eps I)
  double* LQ;         // [kmax][kmax] chol(Q_AA)
  double* Qcols;      // [kmax][bv]: Q e_{a_t} on pick t's box (zero outside it)
  size_t bytes;
};

constexpr int CG_MAXIT = 512;

static size_t ealign(size_t x) { return (x + 255) & ~(size_t)255; }

static ExactWS exact_layout(void* base, int64_t I0, int64_t I1, int64_t I2, int m, int kmax,
                            int64_t H) {
  ExactWS w{};
  const int64_t n = I0 * I1 * I2;
  w.H = H;
  w.b0 = std::min<int64_t>(2 * H + 1, I0);
  w.b1 = std::min<int64_t>(2 * H + 1, I1);
  w.b2 = std::min<int64_t>(2 * H + 1, I2);
  const int64_t bv = w.b0 * w.b1 * w.b2;
  const int64_t nblk = ceil_div(n, EB), nsb = ceil_div(nblk, ESB);
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t b) {
    char* r = p ? p + off : nullptr;
    off += ealign(b);
    return r;
  };
  w.coef = (double*)take(8 * (size_t)n * m);
  w.bval = (double*)take(8 * nblk);
  w.bidx = (long long*)take(8 * nblk);
  w.sval = (double*)take(8 * nsb);
  w.sidx = (long long*)take(8 * nsb);
  w.r = (double*)take(8 * (size_t)bv);
  w.p0 = (double*)take(8 * (size_t)bv);
  w.p1 = (double*)take(8 * (size_t)bv);
  w.q = (double*)take(8 * (size_t)bv);
  w.boxlo = (long long*)take(8 * 3 * (size_t)kmax);
  w.part_pq = (double*)take(8 * CG_BLOCKS);
  w.part_rr = (double*)take(8 * CG_BLOCKS);
  w.rr = (double*)take(8 * (CG_MAXIT + 2));
  w.cgstate = (int*)take(16);
  w.LS = (double*)take(8 * (size_t)kmax * kmax);
  w.LQ = (double*)take(8 * (size_t)kmax * kmax);
  w.Qcols = (double*)take(8 * (size_t)kmax * bv);
  w.bytes = off;
  return w;
}

struct EArgs {
  const double* X;
  long long I0, I1, I2;
  double tla, inv_ls, inv_ls2, shift, jitter, thr;
  const int* offs;
  int m1;
  const double* tau;
  int ntau;
  long long n;
  int kmax, cutoff;
};

template <int KIND>
__device__ __forceinline__ double sigma_diag(const EArgs& a) {
  return a.tau[0] * (kfun<KIND>(0.0, a.tla, a.inv_ls, a.inv_ls2) + a.shift);
}

// Tapered covariance entry S(i, j) for i != j (0 outside the support).
template <int KIND>
__device__ __forceinline__ double sigma_off(const EArgs& a, long long i, long long j) {
  const long long i0 = i / (a.I1 * a.I2), i1 = (i / a.I2) % a.I1, i2 = i % a.I2;
  const long long j0 = j / (a.I1 * a.I2), j1 = (j / a.I2) % a.I1, j2 = j % a.I2;
  const long long e0 = i0 - j0, e1 = i1 - j1, e2 = i2 - j2;
  const long long d2i = e0 * e0 + e1 * e1 + e2 * e2;
  if (d2i >= a.ntau) return 0.0;
  const double t = a.tau[d2i];
  if (t == 0.0) return 0.0;
  // only offsets of the support count (tau > 0 at this squared distance is the same test)
  const double d0 = a.X[3 * i] - a.X[3 * j], d1 = a.X[3 * i + 1] - a.X[3 * j + 1],
               d2 = a.X[3 * i + 2] - a.X[3 * j + 2];
  return t * kfun<KIND>(d0 * d0 + d1 * d1 + d2 * d2, a.tla, a.inv_ls, a.inv_ls2);
}

// Q e_{a_r} at grid node y: its box value, 0 outside the box.
__device__ __forceinline__ double qcol_at(const ExactWS& w, int r, long long y, long long I1,
                                          long long I2) {
  const long long* lo = w.boxlo + 3 * r;
  const long long l0 = y / (I1 * I2) - lo[0], l1 = (y / I2) % I1 - lo[1], l2 = y % I2 - lo[2];
  if (l0 < 0 || l0 >= w.b0 || l1 < 0 || l1 >= w.b1 || l2 < 0 || l2 >= w.b2) return 0.0;
  return w.Qcols[(size_t)r * (w.b0 * w.b1 * w.b2) + (l0 * w.b1 + l1) * w.b2 + l2];
}

__device__ __forceinline__ double delta_of(double nom, double den, double thr) {
  return (fabs(nom) < thr || fabs(den) < thr) ? 0.0 : nom / den;
}

// coef[i][0] = S_ii + eps, coef[i][1 + o] = S(i, i + off_o) (0 outside the grid)
template <int KIND>
__global__ __launch_bounds__(256) void exact_coef_kernel(EArgs a, double* __restrict__ coef) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int m = a.m1 + 1;
  double* c = coef + i * m;
  c[0] = sigma_diag<KIND>(a) + a.jitter;
  const long long i0 = i / (a.I1 * a.I2), i1 = (i / a.I2) % a.I1, i2 = i % a.I2;
  for (int o = 0; o < a.m1; ++o) {
    const int o0 = a.offs[3 * o], o1 = a.offs[3 * o + 1], o2 = a.offs[3 * o + 2];
    const long long j0 = i0 + o0, j1 = i1 + o1, j2 = i2 + o2;
    double v = 0.0;
    if (j0 >= 0 && j0 < a.I0 && j1 >= 0 && j1 < a.I1 && j2 >= 0 && j2 < a.I2)
      v = sigma_off<KIND>(a, i, (j0 * a.I1 + j1) * a.I2 + j2);
    c[1 + o] = v;
  }
}

// Round 0 (snippets_a3.py:77-124): A empty, nom = s_yy, denom = 1 / Q_yy - eps.
template <int KIND>
__global__ __launch_bounds__(256) void exact_score_kernel(EArgs a, const double* __restrict__ qdiag,
                                                          double* __restrict__ cache) {
  const long long y = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= a.n) return;
  const double nom = sigma_diag<KIND>(a);
  const double den = 1.0 / qdiag[y] - a.jitter;
  cache[y] = delta_of(nom, den, a.thr);
}

// One wave: key of block b (entries [b EB, (b+1) EB) of the cache, selected ones excluded).
__device__ __forceinline__ void wave_block_key(const double* cache, const unsigned char* sel,
                                               long long n, long long b, double* bval,
                                               long long* bidx) {
  const int lane = threadIdx.x & 63;
  double v = 0.0;
  long long idx = -1;
  for (int e = lane; e < EB; e += 64) {
    const long long y = b * EB + e;
    if (y < n && !sel[y]) {
      const double c = cache[y];
      if (key_gt(c, y, v, idx)) {
        v = c;
        idx = y;
      }
    }
  }
  wave_keymax(v, idx);
  if (lane == 0) {
    bval[b] = v;
    bidx[b] = idx;
  }
}

__device__ __forceinline__ void wave_super_key(const double* bval, const long long* bidx,
                                               long long nblk, long long sb, double* sval,
                                               long long* sidx) {
  const int lane = threadIdx.x & 63;
  double v = 0.0;
  long long idx = -1;
  const long long b = sb * ESB + lane;
  if (b < nblk) {
    v = bval[b];
    idx = bidx[b];
  }
  wave_keymax(v, idx);
  if (lane == 0) {
    sval[sb] = v;
    sidx[sb] = idx;
  }
}

__global__ __launch_bounds__(256) void exact_block_keys_kernel(const double* cache,
                                                               const unsigned char* sel,
                                                               long long n, double* bval,
                                                               long long* bidx, long long nblk) {
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b < nblk) wave_block_key(cache, sel, n, b, bval, bidx);
}

__global__ __launch_bounds__(256) void exact_super_keys_kernel(const double* bval,
                                                               const long long* bidx,
                                                               long long nblk, double* sval,
                                                               long long* sidx, long long nsb) {
  const long long sb = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sb < nsb) wave_super_key(bval, bidx, nblk, sb, sval, sidx);
}

// Workgroup-wide arg-max over the superblock keys -> the pick of round `round`
// (placement_algorithm2.py:24-50 via sparse_argmax_cache_linear); A <- A u {y*}, the cache entry of
// y* <- 0 (snippets_a3.py:162-168), its block keys refreshed; CG set up for q = Q e_{y*}.
__global__ __launch_bounds__(SEL_THREADS) void exact_select_kernel(
    double* cache, unsigned char* sel, long long I0, long long I1, long long I2, ExactWS w,
    long long nblk, long long nsb, int round, long long* picks, double* pick_delta, int solve) {
  const long long n = I0 * I1 * I2;
  __shared__ double sv[SEL_THREADS / 64];
  __shared__ long long si[SEL_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double v = 0.0;
  long long idx = -1;
  for (long long s = t; s < nsb; s += SEL_THREADS) {
    if (key_gt(w.sval[s], w.sidx[s], v, idx)) {
      v = w.sval[s];
      idx = w.sidx[s];
    }
  }
  wave_keymax(v, idx);
  if (lane == 0) {
    sv[wave] = v;
    si[wave] = idx;
  }
  __syncthreads();
  if (wave == 0) {
    v = lane < SEL_THREADS / 64 ? sv[lane] : 0.0;
    idx = lane < SEL_THREADS / 64 ? si[lane] : -1;
    wave_keymax(v, idx);
    if (lane == 0) {
      si[0] = idx;
      picks[round] = idx;
      if (pick_delta) pick_delta[round] = idx >= 0 ? cache[idx] : 0.0;
      if (idx >= 0) {
        sel[idx] = 1;
        cache[idx] = 0.0;
        if (solve) {
          // the column's box: [a - H, a + H] per axis, shifted inside the grid
          const long long a0 = idx / (I1 * I2), a1 = (idx / I2) % I1, a2 = idx % I2;
          const long long lo0 = min(max(a0 - w.H, 0LL), I0 - w.b0);
          const long long lo1 = min(max(a1 - w.H, 0LL), I1 - w.b1);
          const long long lo2 = min(max(a2 - w.H, 0LL), I2 - w.b2);
          w.boxlo[3 * round] = lo0;
          w.boxlo[3 * round + 1] = lo1;
          w.boxlo[3 * round + 2] = lo2;
          w.r[((a0 - lo0) * w.b1 + (a1 - lo1)) * w.b2 + (a2 - lo2)] = 1.0;
        }
      }
      w.rr[0] = 1.0;
      w.cgstate[0] = 0;
      w.cgstate[1] = 0;
    }
  }
  __syncthreads();
  const long long a = si[0];
  if (a < 0) return;
  const long long b = a / EB;
  if (wave == 0) wave_block_key(cache, sel, n, b, w.bval, w.bidx);
  __syncthreads();
  if (wave == 0) wave_super_key(w.bval, w.bidx, nblk, b / ESB, w.sval, w.sidx);
}

// Deterministic block reduction of the first `np` partials (every block computes the same sum).
__device__ __forceinline__ double sum_partials(const double* part, int np, double* red) {
  const int t = threadIdx.x;
  double s = 0.0;
  for (int i = t; i < np; i += CG_T) s += part[i];
  s = wave_sum(s);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  double tot = 0.0;
#pragma unroll
  for (int i = 0; i < CG_T / 64; ++i) tot += red[i];
  __syncthreads();
  return tot;
}

__device__ __forceinline__ void block_partial(double v, double* part, double* red) {
  v = wave_sum(v);
  const int t = threadIdx.x;
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < CG_T / 64; ++i) s += red[i];
    part[blockIdx.x] = s;
  }
}

// Box-local node l -> (grid coordinates, inside the active region of iteration it).  The
// iterate's support after `it` steps lies within `it` stencil radii of the pick in every axis; the
// kernels skip the rest of the box (its entries are and stay exactly zero).
struct BoxNode {
  long long g0, g1, g2;
  bool active;
};

__device__ __forceinline__ BoxNode box_node(const ExactWS& w, long long l, const long long* lo,
                                            long long a0, long long a1, long long a2,
                                            long long rad) {
  BoxNode b;
  const long long l0 = l / (w.b1 * w.b2), l1 = (l / w.b2) % w.b1, l2 = l % w.b2;
  b.g0 = lo[0] + l0;
  b.g1 = lo[1] + l1;
  b.g2 = lo[2] + l2;
  b.active = llabs(b.g0 - a0) <= rad && llabs(b.g1 - a1) <= rad && llabs(b.g2 - a2) <= rad;
  return b;
}

// CG iteration it, part A: beta from the last residual norms, p_it = r + beta p_{it-1} (computed
// for the neighbours on the fly, written for this thread's own nodes), q = (S + eps I) p_it and
// the partials of p_it . q.  Converged (|r|^2 <= tol2) -> every block returns; block 0 records it.
__global__ __launch_bounds__(CG_T) void exact_cg_a_kernel(ExactWS w, long long I0, long long I1,
                                                          long long I2, const int* offs, int m1,
                                                          int srad, int round,
                                                          const long long* picks, int it,
                                                          double tol2) {
  __shared__ double red[CG_T / 64];
  if (w.cgstate[0]) return;
  const double rr = w.rr[it];
  if (rr <= tol2) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      w.cgstate[0] = 1;
      w.cgstate[1] = it;
    }
    return;
  }
  const double beta = it == 0 ? 0.0 : rr / w.rr[it - 1];
  const double* pold = (it & 1) ? w.p0 : w.p1;  // p_{it-1}
  double* pnew = (it & 1) ? w.p1 : w.p0;        // p_it
  const long long a = picks[round];
  const long long a0 = a / (I1 * I2), a1 = (a / I2) % I1, a2 = a % I2;
  const long long* lo = w.boxlo + 3 * round;
  const long long bv = w.b0 * w.b1 * w.b2;
  const long long rad = min((long long)(it + 1) * srad, w.H);
  const int m = m1 + 1;
  double acc = 0.0;
  for (long long l = (long long)blockIdx.x * CG_T + threadIdx.x; l < bv; l += (long long)CG_BLOCKS * CG_T) {
    const BoxNode nd = box_node(w, l, lo, a0, a1, a2, rad);
    if (!nd.active) continue;
    const double pi = it == 0 ? w.r[l] : fma(beta, pold[l], w.r[l]);
    const double* c = w.coef + ((nd.g0 * I1 + nd.g1) * I2 + nd.g2) * m;
    double s = c[0] * pi;
    for (int o = 0; o < m1; ++o) {
      const double cv = c[1 + o];
      if (cv == 0.0) continue;  // outside the grid
      const long long j0 = nd.g0 + offs[3 * o] - lo[0], j1 = nd.g1 + offs[3 * o + 1] - lo[1],
                      j2 = nd.g2 + offs[3 * o + 2] - lo[2];
      if (j0 < 0 || j0 >= w.b0 || j1 < 0 || j1 >= w.b1 || j2 < 0 || j2 >= w.b2) continue;
      const long long j = (j0 * w.b1 + j1) * w.b2 + j2;
      const double pj = it == 0 ? w.r[j] : fma(beta, pold[j], w.r[j]);
      s = fma(cv, pj, s);
    }
    pnew[l] = pi;
    w.q[l] = s;
    acc = fma(pi, s, acc);
  }
  block_partial(acc, w.part_pq, red);
}

// CG iteration it, part B: alpha = |r|^2 / p.q, x += alpha p, r -= alpha q, partials of |r|^2.
__global__ __launch_bounds__(CG_T) void exact_cg_b_kernel(ExactWS w, long long I1, long long I2,
                                                          int srad, int round,
                                                          const long long* picks, int it,
                                                          double* __restrict__ x) {
  __shared__ double red[CG_T / 64];
  if (w.cgstate[0]) return;
  const double pq = sum_partials(w.part_pq, (int)gridDim.x, red);  // the A kernel's grid
  const double alpha = w.rr[it] / pq;
  const double* p = (it & 1) ? w.p1 : w.p0;
  const long long a = picks[round];
  const long long a0 = a / (I1 * I2), a1 = (a / I2) % I1, a2 = a % I2;
  const long long* lo = w.boxlo + 3 * round;
  const long long bv = w.b0 * w.b1 * w.b2;
  const long long rad = min((long long)(it + 1) * srad, w.H);
  double acc = 0.0;
  for (long long l = (long long)blockIdx.x * CG_T + threadIdx.x; l < bv; l += (long long)CG_BLOCKS * CG_T) {
    if (!box_node(w, l, lo, a0, a1, a2, rad).active) continue;
    x[l] = fma(alpha, p[l], x[l]);
    const double ri = fma(-alpha, w.q[l], w.r[l]);
    w.r[l] = ri;
    acc = fma(ri, ri, acc);
  }
  block_partial(acc, w.part_rr, red);
}

// |r|^2 of iteration it + 1 (one block; every CG_A block then reads it).
__global__ __launch_bounds__(CG_T) void exact_cg_c_kernel(ExactWS w, int it, int np) {
  __shared__ double red[CG_T / 64];
  if (w.cgstate[0]) return;
  const double rr = sum_partials(w.part_rr, np, red);
  if (threadIdx.x == 0) w.rr[it + 1] = rr;
}

constexpr int EX_KMAX = 128;  // picks per run of the exact path (k = 50 in config C4)

// After q_t = Q e_{a_t}: append row t of LQ = chol(Q_AA) and of LS = chol(S_AA + eps I), then
// re-score the window of a_t (snippets_a3.py:190-303; candidates in A -> 0) and refresh the block
// and superblock keys it touched.  One workgroup.
template <int KIND>
__global__ __launch_bounds__(SEL_THREADS) void exact_update_kernel(
    EArgs a, const double* __restrict__ qdiag, double* cache, const unsigned char* sel, ExactWS w,
    long long nblk, int round, const long long* picks) {
  __shared__ double rowbuf[2][EX_KMAX];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int km = a.kmax;
  const long long at = picks[round];
  if (at < 0) return;
  // row `round` of the two factors, one wave each, built in LDS
  if (wave < 2) {
    const double* L = wave == 0 ? w.LQ : w.LS;
    double* row = rowbuf[wave];
    for (int r = 0; r <= round; ++r) {
      const long long ar = picks[r];
      double v;
      if (wave == 0) v = qcol_at(w, round, ar, a.I1, a.I2);
      else v = (r == round) ? sigma_diag<KIND>(a) + a.jitter : sigma_off<KIND>(a, at, ar);
      double acc = 0.0;
      // off-diagonal: row . L[r][:r];  diagonal (r == round): |row[:r]|^2
      for (int s = lane; s < r; s += 64)
        acc = fma(row[s], r == round ? row[s] : L[(size_t)r * km + s], acc);
      acc = wave_sum(acc);
      v -= acc;
      if (lane == 0) row[r] = (r == round) ? sqrt(v) : v / L[(size_t)r * km + r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();
  if (t <= round) {
    w.LQ[(size_t)round * km + t] = rowbuf[0][t];
    w.LS[(size_t)round * km + t] = rowbuf[1][t];
  }
  __syncthreads();
  // window re-score: one thread per candidate; the new rows are read from LDS
  const long long ci0 = at / (a.I1 * a.I2), ci1 = (at / a.I2) % a.I1, ci2 = at % a.I2;
  const long long lo0 = max(ci0 - a.cutoff, 0LL), lo1 = max(ci1 - a.cutoff, 0LL),
                  lo2 = max(ci2 - a.cutoff, 0LL);
  const long long w0 = max(min(ci0 + a.cutoff, a.I0) - lo0, 0LL),
                  w1 = max(min(ci1 + a.cutoff, a.I1) - lo1, 0LL),
                  w2 = max(min(ci2 + a.cutoff, a.I2) - lo2, 0LL);
  const long long nw = w0 * w1 * w2;
  const double syy = sigma_diag<KIND>(a);
  for (long long e = t; e < nw; e += SEL_THREADS) {
    const long long y = ((lo0 + e / (w1 * w2)) * a.I1 + lo1 + (e / w2) % w1) * a.I2 + lo2 + e % w2;
    if (sel[y]) {
      cache[y] = 0.0;
      continue;
    }
    // nominator |LS^-1 s_Ay|^2, denominator |LQ^-1 q_Ay|^2 (forward substitutions)
    double zs[EX_KMAX], zq[EX_KMAX];
    double ns = 0.0, nq = 0.0;
    for (int r = 0; r <= round; ++r) {
      const long long ar = picks[r];
      double vs = sigma_off<KIND>(a, ar, y);
      double vq = qcol_at(w, r, y, a.I1, a.I2);
      const double* ls = r == round ? rowbuf[1] : w.LS + (size_t)r * km;
      const double* lq = r == round ? rowbuf[0] : w.LQ + (size_t)r * km;
      for (int s = 0; s < r; ++s) {
        vs = fma(-ls[s], zs[s], vs);
        vq = fma(-lq[s], zq[s], vq);
      }
      vs /= ls[r];
      vq /= lq[r];
      zs[r] = vs;
      zq[r] = vq;
      ns = fma(vs, vs, ns);
      nq = fma(vq, vq, nq);
    }
    const double nom = syy - ns;
    const double den = 1.0 / (qdiag[y] - nq) - a.jitter;
    cache[y] = delta_of(nom, den, a.thr);
  }
  __syncthreads();
  if (t == 0) cache[at] = 0.0;
  __syncthreads();
  // refresh the block keys of the window rows (each (j0, j1) row is one contiguous i2 run)
  const long long nrow = w0 * w1;
  for (long long rr = wave; rr < nrow; rr += SEL_THREADS / 64) {
    const long long y0 = ((lo0 + rr / w1) * a.I1 + lo1 + rr % w1) * a.I2 + lo2;
    const long long y1 = y0 + w2 - 1;
    for (long long b = y0 / EB; b <= y1 / EB; ++b) wave_block_key(cache, sel, a.n, b, w.bval, w.bidx);
  }
  __syncthreads();
  for (long long rr = wave; rr < nrow; rr += SEL_THREADS / 64) {
    const long long y0 = ((lo0 + rr / w1) * a.I1 + lo1 + rr % w1) * a.I2 + lo2;
    const long long y1 = y0 + w2 - 1;
    for (long long sb = y0 / EB / ESB; sb <= y1 / EB / ESB; ++sb)
      wave_super_key(w.bval, w.bidx, nblk, sb, w.sval, w.sidx);
  }
}

}  // namespace vgposp

using namespace vgposp;

namespace {

#define VGPOSP_EXACT_CHECK_COMMON()                                                          \
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);             \
  VG_CHECK_ARG(X != nullptr, 2);                                                          \
  VG_CHECK_ARG(I0 >= 1 && I1 >= 1 && I2 >= 1, 3);                                         \
  VG_CHECK_ARG(amp > 0.0, 6);                                                             \
  VG_CHECK_ARG(ls > 0.0, 7);                                                              \
  VG_CHECK_ARG(m >= 1 && (m == 1 || offsets != nullptr), 12);                             \
  VG_CHECK_ARG(tau != nullptr && ntau >= 1, 13);                                          \
  VG_CHECK_ARG(kmax >= 1 && kmax <= EX_KMAX, 15);                                         \
  VG_CHECK_ARG(cutoff >= 0, 16);                                                          \
  VG_CHECK_ARG(radius >= 1, 17);                                                          \
  VG_CHECK_ARG(cg_iters >= 1 && cg_iters <= CG_MAXIT, 18);                                \
  VG_CHECK_ARG(qdiag != nullptr, 19);                                                     \
  VG_CHECK_ARG(cache != nullptr, 20);                                                     \
  VG_CHECK_ARG(selected != nullptr, 21);                                                  \
  VG_CHECK_ARG(ws != nullptr, 22)

EArgs make_eargs(const double* X, int64_t I0, int64_t I1, int64_t I2, double amp, double ls,
                 double shift, double jitter, double thr, const int* offs, int m, const double* tau,
                 int ntau, int kmax, int cutoff) {
  EArgs a;
  a.X = X;
  a.I0 = I0;
  a.I1 = I1;
  a.I2 = I2;
  a.tla = 2.0 * std::log(amp);
  a.inv_ls = 1.0 / ls;
  a.inv_ls2 = 1.0 / (ls * ls);
  a.shift = shift;
  a.jitter = jitter;
  a.thr = thr;
  a.offs = offs;
  a.m1 = m - 1;
  a.tau = tau;
  a.ntau = ntau;
  a.n = I0 * I1 * I2;
  a.kmax = kmax;
  a.cutoff = cutoff;
  return a;
}

template <int KIND>
int exact_prepare_t(const EArgs& a, const double* qdiag, double* cache, unsigned char* sel,
                    const ExactWS& w, hipStream_t s) {
  const long long n = a.n;
  const long long nblk = ceil_div(n, EB), nsb = ceil_div(nblk, ESB);
  VG_HIP(vg_memset(sel, 0, n, s));
  hipLaunchKernelGGL(exact_coef_kernel<KIND>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, a,
                     w.coef);
  VG_LAUNCH_CHECK();
  {
    ProfScope ps("exact_score", s, 0.0, 16.0 * n);
    hipLaunchKernelGGL(exact_score_kernel<KIND>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                       a, qdiag, cache);
    VG_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(exact_block_keys_kernel, dim3((unsigned)ceil_div(nblk, 4)), dim3(256), 0, s,
                     cache, sel, n, w.bval, w.bidx, nblk);
  VG_LAUNCH_CHECK();
  hipLaunchKernelGGL(exact_super_keys_kernel, dim3((unsigned)ceil_div(nsb, 4)), dim3(256), 0, s,
                     w.bval, w.bidx, nblk, w.sval, w.sidx, nsb);
  VG_LAUNCH_CHECK();
  return 0;
}

template <int KIND>
int exact_round_t(const EArgs& a, const double* qdiag, double* cache, unsigned char* sel,
                  const ExactWS& w, int round, int last, long long* picks, double* pick_delta,
                  int radius, int cg_iters, double cg_tol, hipStream_t s) {
  const long long n = a.n;
  const long long nblk = ceil_div(n, EB), nsb = ceil_div(nblk, ESB);
  const long long bv = w.b0 * w.b1 * w.b2;
  double* x = last ? nullptr : w.Qcols + (size_t)round * bv;
  if (x) {
    VG_HIP(vg_memset(w.r, 0, 8 * (size_t)bv, s));
    VG_HIP(vg_memset(w.p0, 0, 8 * (size_t)bv, s));
    VG_HIP(vg_memset(w.p1, 0, 8 * (size_t)bv, s));
    VG_HIP(vg_memset(x, 0, 8 * (size_t)bv, s));
  }
  {
    ProfScope ps("exact_select", s, 0.0, 16.0 * nsb);
    hipLaunchKernelGGL(exact_select_kernel, dim3(1), dim3(SEL_THREADS), 0, s, cache, sel, a.I0, a.I1,
                       a.I2, w, nblk, nsb, round, picks, pick_delta, x != nullptr ? 1 : 0);
    VG_LAUNCH_CHECK();
  }
  if (!x) return 0;
  {
    const int m = a.m1 + 1;
    ProfScope ps("exact_cg", s, 0.0, (double)cg_iters * 8.0 * bv * (m + 9));
    const double tol2 = cg_tol * cg_tol;
    const unsigned blocks = (unsigned)std::min<long long>(CG_BLOCKS, ceil_div(bv, CG_T));
    for (int it = 0; it < cg_iters; ++it) {
      hipLaunchKernelGGL(exact_cg_a_kernel, dim3(blocks), dim3(CG_T), 0, s, w, a.I0, a.I1, a.I2,
                         a.offs, a.m1, radius, round, picks, it, tol2);
      VG_LAUNCH_CHECK();
      hipLaunchKernelGGL(exact_cg_b_kernel, dim3(blocks), dim3(CG_T), 0, s, w, a.I1, a.I2, radius,
                         round, picks, it, x);
      VG_LAUNCH_CHECK();
      hipLaunchKernelGGL(exact_cg_c_kernel, dim3(1), dim3(CG_T), 0, s, w, it, (int)blocks);
      VG_LAUNCH_CHECK();
    }
  }
  {
    ProfScope ps("exact_update", s, 0.0, 0.0);
    hipLaunchKernelGGL(exact_update_kernel<KIND>, dim3(1), dim3(SEL_THREADS), 0, s, a, qdiag, cache,
                       sel, w, nblk, round, picks);
    VG_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace

extern "C" size_t vgposp_exact_workspace_bytes(int64_t I0, int64_t I1, int64_t I2, int m, int kmax,
                                               int radius, int cg_iters) {
  if (I0 <= 0 || I1 <= 0 || I2 <= 0 || m <= 0 || kmax <= 0 || radius < 1 || cg_iters < 1) return 0;
  return exact_layout(nullptr, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters).bytes;
}

extern "C" int vgposp_exact_prepare(int kind, const double* X, int64_t I0, int64_t I1, int64_t I2,
                                    double amp, double ls, double diag_shift, double jitter,
                                    double threshold, const int* offsets, int m, const double* tau,
                                    int ntau, int kmax, int cutoff, int radius, int cg_iters,
                                    const double* qdiag, double* cache, uint8_t* selected, void* ws,
                                    size_t ws_bytes, void* stream) {
  clear_error();
  VGPOSP_EXACT_CHECK_COMMON();
  const ExactWS w = exact_layout(ws, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters);
  if (ws_bytes < w.bytes) {
    set_error("vgposp_exact_prepare: workspace %zu < %zu bytes", ws_bytes, w.bytes);
    return VGPOSP_E_WS;
  }
  const EArgs a = make_eargs(X, I0, I1, I2, amp, ls, diag_shift, jitter, threshold, offsets, m, tau,
                             ntau, kmax, cutoff);
  hipStream_t s = as_stream(stream);
  switch (kind) {
    case VGPOSP_KERNEL_EQ: return exact_prepare_t<VGPOSP_KERNEL_EQ>(a, qdiag, cache, selected, w, s);
    case VGPOSP_KERNEL_MATERN12: return exact_prepare_t<VGPOSP_KERNEL_MATERN12>(a, qdiag, cache, selected, w, s);
    case VGPOSP_KERNEL_MATERN32: return exact_prepare_t<VGPOSP_KERNEL_MATERN32>(a, qdiag, cache, selected, w, s);
    default: return exact_prepare_t<VGPOSP_KERNEL_MATERN52>(a, qdiag, cache, selected, w, s);
  }
}

extern "C" int vgposp_exact_round(int kind, const double* X, int64_t I0, int64_t I1, int64_t I2,
                                  double amp, double ls, double diag_shift, double jitter,
                                  double threshold, const int* offsets, int m, const double* tau,
                                  int ntau, int kmax, int cutoff, int radius, int cg_iters,
                                  const double* qdiag, double* cache, uint8_t* selected, void* ws,
                                  size_t ws_bytes, int round, int last, int64_t* picks,
                                  double* pick_delta, double cg_tol, void* stream) {
  clear_error();
  VGPOSP_EXACT_CHECK_COMMON();
  VG_CHECK_ARG(round >= 0 && round < kmax, 24);
  VG_CHECK_ARG(picks != nullptr, 26);
  VG_CHECK_ARG(cg_tol >= 0.0, 28);
  const ExactWS w = exact_layout(ws, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters);
  if (ws_bytes < w.bytes) {
    set_error("vgposp_exact_round: workspace %zu < %zu bytes", ws_bytes, w.bytes);
    return VGPOSP_E_WS;
  }
  const EArgs a = make_eargs(X, I0, I1, I2, amp, ls, diag_shift, jitter, threshold, offsets, m, tau,
                             ntau, kmax, cutoff);
  hipStream_t s = as_stream(stream);
  long long* pk = reinterpret_cast<long long*>(picks);
  switch (kind) {
    case VGPOSP_KERNEL_EQ:
      return exact_round_t<VGPOSP_KERNEL_EQ>(a, qdiag, cache, selected, w, round, last, pk, pick_delta, radius, cg_iters, cg_tol, s);
    case VGPOSP_KERNEL_MATERN12:
      return exact_round_t<VGPOSP_KERNEL_MATERN12>(a, qdiag, cache, selected, w, round, last, pk, pick_delta, radius, cg_iters, cg_tol, s);
    case VGPOSP_KERNEL_MATERN32:
      return exact_round_t<VGPOSP_KERNEL_MATERN32>(a, qdiag, cache, selected, w, round, last, pk, pick_delta, radius, cg_iters, cg_tol, s);
    default:
      return exact_round_t<VGPOSP_KERNEL_MATERN52>(a, qdiag, cache, selected, w, round, last, pk, pick_delta, radius, cg_iters, cg_tol, s);
  }
}

extern "C" int vgposp_exact_buffers(void* ws, int64_t I0, int64_t I1, int64_t I2, int m, int kmax,
                                    int radius, int cg_iters, double** qcols, int64_t** boxlo,
                                    int** cgstate) {
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  const ExactWS w = exact_layout(ws, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters);
  if (qcols) *qcols = w.Qcols;
  if (boxlo) *boxlo = reinterpret_cast<int64_t*>(w.boxlo);
  if (cgstate) *cgstate = w.cgstate;
  return 0;
}
