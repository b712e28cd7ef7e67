// PHASE-STAMPED BUILD of vgposp_amd/csrc/exact_greedy.hip (not built into the library): the
// product file as of round 5/6 with its -DVGPOSP_EXACT_DBG=1|2|3 instrumentation (thread 0 of the
// per-round kernels stamps phases with s_memrealtime; vgposp_exact_dbg copies the last 64 records
// out).  With VGPOSP_EXACT_DBG=0 it compiles to the same device code as the product file.
// Build: SRC=../../tools/variants/exact_greedy_dbg.hip tools/build_exact_variant.sh dbg -DVGPOSP_EXACT_DBG=1
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
//
// Bounded-lazy form (vgposp_exact_bounds / _argmax / _refine / _pick / _update): diag(Q) is not
// factored at all.  For every candidate y, K steps of CG on (S + eps I) x = e_y from x = 0 give
// g_K = sum_i alpha_i |r_i|^2 = e_y^T x_K <= Q_yy, and Q_yy - g_K = |x* - x_K|_A^2
// <= 4 rho^(2K) Q_yy (rho from a Gershgorin bound on the spectrum), so
// Q_yy <= g_K / (1 - 4 rho^(2K)).  The K-step Krylov vectors of e_y live on the nodes within K
// stencil steps of y (a few hundred), so one wave runs one candidate's K steps in registers + LDS.
// The cache then holds UPPER BOUNDS of the reference's cached deltas (delta is increasing in
// P_yy); whenever the arg-max lands on a candidate whose Q_yy is only bounded, the host refines
// it: its full CG column (the same Krylov-box solve a pick gets) gives Q_yy, and its cache entry
// becomes the reference's value (re-scored with the A of its last window re-score, lastA[y]).
// The arg-max is only taken when it lands on a refined candidate, so the picks are the
// reference's, and every pick's column is already there when it is picked.
#include <cmath>
#include <type_traits>

#include "common.h"
#include "psd.h"

namespace vgposp {

constexpr int EB = 256;      // cache entries per block key
constexpr int ESB = 64;      // blocks per superblock key
constexpr int CG_BLOCKS = 1024;
constexpr int CG_T = 256;
constexpr int CG_SEG = 16;  // lanes per diamond row of the 7-point CG walk (8, 32, 64: slower)
constexpr int CG_RPW = 64 / CG_SEG;  // diamond rows per wave
constexpr int SEL_THREADS = 1024;

// Pick t as the window re-score sees it: grid coordinates, point, and its CG column (box origin
// and element offset of its slot).  Written by the first kernel that stages pick t (the window /
// rows kernel of round t), so later rounds stage picks 0 .. t - 1 with ONE level of contiguous
// loads instead of picks -> X and slot_of_round -> boxlo chains.
struct PickRec {
  int g[3];
  int pick;  // the pick's index: a record whose pick (or slot) differs from the round's is stale
  double x[3];
  long long lo[3];
  long long base;
};

struct ExactWS {
  double* coef;       // [n][m]: coef[i][0] diagonal (S_ii + eps), coef[i][1 + o] = S(i, i + off_o)
  double* bval;       // [nblk]
  long long* bidx;
  double* sval;       // [nsb]
  long long* sidx;
  // CG on the box of half-width H around the pick (clipped into the grid): the Krylov vectors of
  // a solve of S e_a are exactly zero beyond H = iterations x stencil radius, so the box holds
  // every non-zero of the full-grid iteration.  Box-local vectors, [bv] each.
  double* r;          // [CG_B][bv] residual (one vector per column of a batch)
  double* p0;         // [CG_B][bv] directions (two, alternating)
  double* p1;
  double* q;          // [CG_B][bv] A p
  long long* boxlo;   // [kmax][3] box origin of each pick's column
  long long b0, b1, b2, H;
  double* part_pq;    // [CG_B][CG_BLOCKS]
  double* part_rr;    // [CG_B][CG_BLOCKS]
  double* rr;         // [CG_B][maxit + 2] residual norms per iteration
  int* cgstate;       // [CG_B][4]: done flag, iterations of the last solve
  double* LS;         // chol(S_AA + eps I), packed lower triangle (row r at r (r + 1) / 2)
  double* LQ;         // chol(Q_AA), packed likewise
  double* RS;         // [kmax]: 1 / diag(LS)
  double* RQ;         // [kmax]: 1 / diag(LQ)
  struct PickRec* prec;  // [kmax]: what a re-score needs of pick t (grid point, box), see PickRec
  double* Qcols;      // [nslots][bv]: Q e_c on candidate c's box (zero outside it)
  int* slot_of_round; // [kmax]: the column slot of pick t
  unsigned char* qexact;  // [n]: 1 = qdiag[y] is Q_yy; 0 = an upper bound from the K_lo-step
                          // bounds, 2 = a tightened (K_hi-step) upper bound
  unsigned char* lastA;   // [n]: |A| when y's cache entry was last scored (0: round 0)
  long long* cand;    // [2]: scratch (the arg-max candidate of the round-3 host loop)
  double* gersh;      // [2 + 2 CG_BLOCKS]: lambda_min / lambda_max bounds, then partials
  // device-side rounds (vgposp_exact_steps): the refine-or-pick decision never leaves the GPU
  int* ctl;           // [CTL_N]: see CTL_* below
  long long* rl_cand; // [nslots]: the refined candidate held in each column slot (-1: free)
  int* rl_age;        // [nslots]: refinement order (the oldest unpinned slot is recycled first)
  unsigned char* rl_pin;  // [nslots]: 1 = the slot is a pick's column (never recycled)
  long long* rf_cand; // [CG_B]: the pending refinement batch (-1: unused column)
  int* rf_slot;       // [CG_B]
  long long* rt_cand; // [CG_B]: the pending tightening list (ctl[CTL_NT] entries)
  // pre-tightening (vgposp_exact_pretighten): the best candidates of round 0 tightened at once
  long long* pt_list;      // [PT_MAX]
  unsigned* pt_hist;       // [PT_BINS] radix-select histogram
  long long* pt_state;     // [4]: threshold code, candidates still needed, pass, listed count
  int* pt_count;           // [1]: list entries (<= PT_MAX), as the LIST bounds kernel reads it
  size_t bytes;
};

// ctl[]: the rounds' control block (device memory; the host reads it once per refinement event)
constexpr int CTL_STALL = 0;     // the round whose arg-max needs a refinement (-1: none)
constexpr int CTL_NB = 1;        // candidates in the pending batch (rf_cand / rf_slot)
constexpr int CTL_UNPICKED = 2;  // refined candidates not (yet) picked
constexpr int CTL_EVENTS = 3;    // refinement batches in this run
constexpr int CTL_REFINED = 4;   // candidates refined in this run
constexpr int CTL_AGE = 5;       // refinement counter (rl_age)
constexpr int CTL_NT = 6;        // candidates in the pending tightening list (rt_cand)
constexpr int CTL_TIGHT = 7;     // candidates tightened in this run
constexpr int CTL_N = 8;

// coefficient rows padded to an even count of doubles (16-byte aligned rows: two-double loads)
__host__ __device__ constexpr int coef_stride(int m) { return (m + 1) & ~1; }

// column slots: one per pick, as many again for refined candidates that are not (yet) picked
__host__ __device__ __forceinline__ int exact_slots(int kmax) { return 2 * kmax; }

constexpr int PT_BINS = 4096;          // 12-bit digits of the radix select
constexpr long long PT_MAX = 65536;    // candidates pre-tightened per run (at most)

constexpr int CG_MAXIT = 512;
constexpr int CG_B = 32;      // columns solved together by one batched CG (blockIdx.y)

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
  w.coef = (double*)take(8 * (size_t)n * coef_stride(m));
  w.bval = (double*)take(8 * nblk);
  w.bidx = (long long*)take(8 * nblk);
  w.sval = (double*)take(8 * nsb);
  w.sidx = (long long*)take(8 * nsb);
  w.r = (double*)take(8 * (size_t)bv * CG_B);
  w.p0 = (double*)take(8 * (size_t)bv * CG_B);
  w.p1 = (double*)take(8 * (size_t)bv * CG_B);
  w.q = (double*)take(8 * (size_t)bv * CG_B);
  w.boxlo = (long long*)take(8 * 3 * (size_t)exact_slots(kmax));
  w.part_pq = (double*)take(8 * CG_BLOCKS * CG_B);
  w.part_rr = (double*)take(8 * CG_BLOCKS * CG_B);
  w.rr = (double*)take(8 * (CG_MAXIT + 2) * CG_B);
  w.cgstate = (int*)take(16 * CG_B);
  w.LS = (double*)take(8 * (size_t)kmax * (kmax + 1) / 2);
  w.LQ = (double*)take(8 * (size_t)kmax * (kmax + 1) / 2);
  w.RS = (double*)take(8 * (size_t)kmax);
  w.RQ = (double*)take(8 * (size_t)kmax);
  w.prec = (PickRec*)take(sizeof(PickRec) * (size_t)kmax);
  w.Qcols = (double*)take(8 * (size_t)exact_slots(kmax) * bv);
  w.slot_of_round = (int*)take(4 * (size_t)kmax);
  w.qexact = (unsigned char*)take((size_t)n);
  w.lastA = (unsigned char*)take((size_t)n);
  w.cand = (long long*)take(16);
  w.gersh = (double*)take(8 * (2 + 2 * (size_t)CG_BLOCKS));
  w.ctl = (int*)take(4 * CTL_N);
  w.rl_cand = (long long*)take(8 * (size_t)exact_slots(kmax));
  w.rl_age = (int*)take(4 * (size_t)exact_slots(kmax));
  w.rl_pin = (unsigned char*)take((size_t)exact_slots(kmax));
  w.rf_cand = (long long*)take(8 * CG_B);
  w.rf_slot = (int*)take(4 * CG_B);
  w.pt_list = (long long*)take(8 * (size_t)PT_MAX);
  w.pt_hist = (unsigned*)take(4 * (size_t)PT_BINS);
  w.pt_state = (long long*)take(8 * 4);
  w.pt_count = (int*)take(16);
  w.rt_cand = (long long*)take(8 * CG_B);
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
  // (32-bit coordinates: the exact path requires n < 2^31, vgposp_exact_prepare / _coef)
  const int I1 = (int)a.I1, I2 = (int)a.I2, I12 = I1 * I2, ii = (int)i, jj = (int)j;
  const int i0 = ii / I12, i1 = (ii - i0 * I12) / I2, i2 = ii - (ii / I2) * I2;
  const int j0 = jj / I12, j1 = (jj - j0 * I12) / I2, j2 = jj - (jj / I2) * I2;
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

// Column slot `slot` at grid node y: its box value, 0 outside the box.
__device__ __forceinline__ double qslot_at(const ExactWS& w, int slot, long long y, long long I1,
                                           long long I2) {
  const long long* lo = w.boxlo + 3 * slot;
  const int yi = (int)y, i12 = (int)(I1 * I2), i2s = (int)I2;  // (n < 2^31 on this path)
  const int y0 = yi / i12, y1 = (yi - y0 * i12) / i2s, y2 = yi - (yi / i2s) * i2s;
  const long long l0 = y0 - lo[0], l1 = y1 - lo[1], l2 = y2 - lo[2];
  if (l0 < 0 || l0 >= w.b0 || l1 < 0 || l1 >= w.b1 || l2 < 0 || l2 >= w.b2) return 0.0;
  return w.Qcols[(size_t)slot * (w.b0 * w.b1 * w.b2) + (l0 * w.b1 + l1) * w.b2 + l2];
}

// Q e_{a_r} (pick r's column) at grid node y.
__device__ __forceinline__ double qcol_at(const ExactWS& w, int r, long long y, long long I1,
                                          long long I2) {
  return qslot_at(w, w.slot_of_round[r], y, I1, I2);
}

__device__ __forceinline__ double delta_of(double nom, double den, double thr) {
  return (fabs(nom) < thr || fabs(den) < thr) ? 0.0 : nom / den;
}

// The cached delta from nom and P_yy = Q_yy - |LQ^-1 q_Ay|^2; with `exact` false P is an upper
// bound of P_yy and the result an upper bound of the delta (denom = 1/P - eps decreases in P; a
// denominator that may still reach the threshold is bounded by it).
__device__ __forceinline__ double delta_from(double nom, double P, bool exact, double eps,
                                             double thr) {
  const double den = 1.0 / P - eps;
  if (exact) return delta_of(nom, den, thr);
  if (fabs(nom) < thr) return 0.0;
  return nom / fmax(den, thr);
}

// coef[i][0] = S_ii + eps, coef[i][1 + o] = S(i, i + off_o) (0 outside the grid): row i into c
// (its padded stride of doubles)
template <int KIND>
__device__ __forceinline__ void coef_row(const EArgs& a, long long i, double* c) {
  const int m = a.m1 + 1;
  c[0] = sigma_diag<KIND>(a) + a.jitter;
  if (coef_stride(m) > m) c[m] = 0.0;
  // grid coordinates by 32-bit division (n < 2^31 on this path), and sigma_off's squared index
  // distance straight from the offset: sigma_off recomputed both nodes' coordinates with 64-bit
  // divisions (software sequences) for each of the m1 neighbours.  The same values.
  const int I1 = (int)a.I1, I2 = (int)a.I2, ii = (int)i;
  const int i0 = ii / (I1 * I2), ir = ii - i0 * (I1 * I2), i1 = ir / I2, i2 = ir - i1 * I2;
  for (int o = 0; o < a.m1; ++o) {
    const int o0 = a.offs[3 * o], o1 = a.offs[3 * o + 1], o2 = a.offs[3 * o + 2];
    const int j0 = i0 + o0, j1 = i1 + o1, j2 = i2 + o2;
    double v = 0.0;
    const int d2i = o0 * o0 + o1 * o1 + o2 * o2;
    if (j0 >= 0 && j0 < a.I0 && j1 >= 0 && j1 < I1 && j2 >= 0 && j2 < I2 && d2i < a.ntau &&
        a.tau[d2i] != 0.0) {
      const long long j = ((long long)j0 * I1 + j1) * I2 + j2;
      const double d0 = a.X[3 * i] - a.X[3 * j], d1 = a.X[3 * i + 1] - a.X[3 * j + 1],
                   d2 = a.X[3 * i + 2] - a.X[3 * j + 2];
      v = a.tau[d2i] * kfun<KIND>(d0 * d0 + d1 * d1 + d2 * d2, a.tla, a.inv_ls, a.inv_ls2);
    }
    c[1 + o] = v;
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void exact_coef_kernel(EArgs a, double* __restrict__ coef) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  coef_row<KIND>(a, i, coef + i * coef_stride(a.m1 + 1));
}

// The same rows for a stride of 8 (the 7-point stencil), written through LDS: a thread's eight
// 8-byte stores each touch 64 rows of its wave at once, partial lines (WRITE_SIZE read 4.8x the
// table's 64 bytes per row), so the block's 256 rows are assembled in LDS and stored as one
// contiguous 16 KB run of 16-byte stores.  The same values in the same places.
template <int KIND>
__global__ __launch_bounds__(256) void exact_coef8_kernel(EArgs a, double* __restrict__ coef) {
  __shared__ double rows[256 * 8];
  const long long i0 = (long long)blockIdx.x * 256, i = i0 + threadIdx.x;
  if (i < a.n) coef_row<KIND>(a, i, rows + threadIdx.x * 8);
  __syncthreads();
  const int nrow = (int)min(256LL, a.n - i0);
  double2* dst = reinterpret_cast<double2*>(coef + i0 * 8);
  const double2* src = reinterpret_cast<const double2*>(rows);
  for (int k = threadIdx.x; k < nrow * 4; k += 256) dst[k] = src[k];
}

// Gershgorin bounds of the spectrum of S + eps I from the coefficient table: per row
// c_ii -/+ sum_j |c_ij|; block partials of (min lower, max upper), then one block reduces them.
__global__ __launch_bounds__(256) void exact_gersh_kernel(const double* __restrict__ coef,
                                                          long long n, int m, double* part) {
  __shared__ double rl[4], rh[4];
  double lo = INFINITY, hi = -INFINITY;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const double* c = coef + i * coef_stride(m);
    double s = 0.0;
    for (int o = 1; o < m; ++o) s += fabs(c[o]);
    lo = fmin(lo, c[0] - s);
    hi = fmax(hi, c[0] + s);
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  if ((threadIdx.x & 63) == 0) {
    rl[threadIdx.x >> 6] = lo;
    rh[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 + blockIdx.x] = fmin(fmin(rl[0], rl[1]), fmin(rl[2], rl[3]));
    part[2 + CG_BLOCKS + blockIdx.x] = fmax(fmax(rh[0], rh[1]), fmax(rh[2], rh[3]));
  }
}

__global__ __launch_bounds__(64) void exact_gersh_final_kernel(double* part, int np) {
  double lo = INFINITY, hi = -INFINITY;
  for (int i = threadIdx.x; i < np; i += 64) {
    lo = fmin(lo, part[2 + i]);
    hi = fmax(hi, part[2 + CG_BLOCKS + i]);
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  if (threadIdx.x == 0) {
    part[0] = lo;
    part[1] = hi;
  }
}

// Upper bounds of Q_yy for y in [c0, c1): K CG steps on (S + eps I) x = e_y from x = 0, one wave
// per candidate.  The nodes within K stencil steps of y are a host table sorted by step distance
// (tab_off [T][3] offsets, tab_cnt[d] = nodes within d steps, tab_nb [T][m1] = table position of
// node + off_o or -1); lane l holds nodes l, l + 64, ... in registers, p is exchanged through a
// wave-private LDS vector.  Step it touches only the tab_cnt[it + 1] nodes A p_it can reach.
// qhi[y] = hi_scale * sum_i alpha_i |r_i|^2, hi_scale = (1 + margin) / (1 - 4 rho^(2K)).
// Upper bounds of Q_yy = e_y^T (S + eps I)^-1 e_y from K CG steps on (S + eps I) x = e_y, x0 = 0.
// The CG estimate g_K = sum_k gamma_k |r_k|^2 (gamma_k = alpha_k) is the Gauss-quadrature LOWER
// bound, and Q_yy - g_K = |x - x_K|_A^2.  Two upper bounds:
//  * mu = 0: g_K / (1 - 4 rho^2K) (hi_scale carries the factor): the Chebyshev bound on the CG
//    error, rho from the spectrum bounds;
//  * mu > 0 (0 < mu <= lambda_min, the Gershgorin lower bound): the Gauss-Radau bound
//    |x - x_K|_A^2 <= gamma^mu_K |r_K|^2 with gamma^mu_0 = 1 / mu and
//    gamma^mu_{k+1} = (gamma^mu_k - gamma_k) / (mu (gamma^mu_k - gamma_k) + delta_{k+1}),
//    delta_{k+1} = |r_{k+1}|^2 / |r_k|^2 (Golub & Meurant, "Matrices, Moments and Quadrature";
//    the CG form of Meurant & Tichy, Numer. Algorithms 2013, algorithm CGQ); hi_scale is then only
//    the rounding margin.  On the beta = 4 taper its bracket after K steps is about the Chebyshev
//    one after K + 1 (9e-7 at K = 4 against 8.5e-7 at K = 5): one CG step fewer per candidate.
__device__ __forceinline__ double radau_step(double gmu, double gamma, double mu, double delta) {
  const double d = gmu - gamma;
  return d / fma(mu, d, delta);
}

__device__ __forceinline__ double bound_value(double g, double gmu, double rrK, double mu,
                                              double hi_scale) {
  return mu > 0.0 ? hi_scale * fma(gmu, rrK, g) : hi_scale * g;
}

constexpr int BND_GRID = 65536;  // workgroups of an all-candidate bounds launch, at most
constexpr int BND_GRP_GRID = 16384;  // the same for the grouped kernel (exact_bounds_grp_kernel)
constexpr int BND_T = 256;
constexpr int BND_WAVES = BND_T / 64;
constexpr int BND_SMAX = 14;
constexpr int BND_TMAX = 64 * BND_SMAX;
constexpr int BND_NBMAX = 8192;

__global__ __launch_bounds__(BND_T) void exact_bounds_kernel(
    const double* __restrict__ coef, long long I0, long long I1, long long I2, int m1,
    const int* __restrict__ tab_off, const int* __restrict__ tab_nb,
    const int* __restrict__ tab_cnt, int T, int K, double hi_scale, double mu, long long c0,
    long long c1, double* __restrict__ qhi) {
  __shared__ double plds[BND_WAVES][BND_TMAX];
  __shared__ short nbl[BND_NBMAX];
  __shared__ short offl[3 * BND_TMAX];
  __shared__ int cntl[BND_SMAX * 4 + 1];
  for (int i = threadIdx.x; i < T * m1; i += BND_T) nbl[i] = (short)tab_nb[i];
  for (int i = threadIdx.x; i < 3 * T; i += BND_T) offl[i] = (short)tab_off[i];
  for (int i = threadIdx.x; i <= K; i += BND_T) cntl[i] = tab_cnt[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* pl = plds[wave];
  const int m = m1 + 1;
  // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs, so XCD x (= blockIdx.x
  // mod 8) walks its own contiguous eighth of the candidates and neighbouring candidates, whose
  // reach tables share most coefficient rows, meet in the same L2 (gridDim.x is a multiple of 8)
  const long long per_xcd = (c1 - c0 + 7) / 8, xlo = c0 + (blockIdx.x & 7) * per_xcd;
  const long long xhi = min(c1, xlo + per_xcd);
  for (long long y = xlo + (long long)(blockIdx.x >> 3) * BND_WAVES + wave; y < xhi;
       y += (long long)(gridDim.x >> 3) * BND_WAVES) {
    const long long y0 = y / (I1 * I2), y1 = (y / I2) % I1, y2 = y % I2;
    int gi[BND_SMAX];  // grid index (n < 2^31, checked by the caller) or -1
    double r[BND_SMAX], p[BND_SMAX], q[BND_SMAX];
#pragma unroll
    for (int s = 0; s < BND_SMAX; ++s) {
      const int j = s * 64 + lane;
      gi[s] = -1;
      r[s] = (j == 0) ? 1.0 : 0.0;   // node 0 is y itself
      p[s] = r[s];
      if (j < T) {
        const long long g0 = y0 + offl[3 * j], g1 = y1 + offl[3 * j + 1], g2 = y2 + offl[3 * j + 2];
        if (g0 >= 0 && g0 < I0 && g1 >= 0 && g1 < I1 && g2 >= 0 && g2 < I2)
          gi[s] = (int)((g0 * I1 + g1) * I2 + g2);
        pl[j] = r[s];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double rr = 1.0, g = 0.0, gmu = mu > 0.0 ? 1.0 / mu : 0.0;
    for (int it = 0; it < K; ++it) {
      const int cnt = cntl[it + 1];
      double pq = 0.0;
#pragma unroll
      for (int s = 0; s < BND_SMAX; ++s) {
        const int j = s * 64 + lane;
        q[s] = 0.0;
        if (s * 64 < cnt && j < cnt && gi[s] >= 0) {
          const double* c = coef + (size_t)gi[s] * coef_stride(m);
          double acc = c[0] * p[s];
          const short* nb = nbl + j * m1;
          for (int o = 0; o < m1; ++o) {
            const int jn = nb[o];
            if (jn >= 0) acc = fma(c[1 + o], pl[jn], acc);
          }
          q[s] = acc;
          pq = fma(p[s], acc, pq);
        }
      }
      pq = wave_sum(pq);
      const double alpha = rr / pq;
      g = fma(alpha, rr, g);
      if (it + 1 == K && mu <= 0.0) break;
      double rn = 0.0;
#pragma unroll
      for (int s = 0; s < BND_SMAX; ++s) {
        r[s] = fma(-alpha, q[s], r[s]);
        rn = fma(r[s], r[s], rn);
      }
      rn = wave_sum(rn);
      if (mu > 0.0) gmu = radau_step(gmu, alpha, mu, rn / rr);
      const double beta = rn / rr;
      rr = rn;
      if (it + 1 == K) break;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int s = 0; s < BND_SMAX; ++s) {
        const int j = s * 64 + lane;
        p[s] = fma(beta, p[s], r[s]);
        if (j < cnt) pl[j] = p[s];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) qhi[y] = bound_value(g, gmu, rr, mu, hi_scale);
  }
}

// The same bounds with the stencil size M1 and the slots per lane SM compile-time: a candidate's
// coefficients (SM x (M1 + 1) doubles per lane) are loaded into registers once, all loads in
// flight together, so its K steps run on registers and LDS only (the generic kernel above waits on
// one coefficient load at a time).  Neighbours outside the table read a zero LDS entry.
// A coefficient row (M doubles of the 16-byte-aligned padded row gi, zeros for gi < 0) in
// two-double loads.
template <int M>
__device__ __forceinline__ void load_coef_row(const double* __restrict__ coef, int gi, double* c) {
  constexpr int MS = coef_stride(M);
#pragma unroll
  for (int o = 0; o < MS; o += 2) {
    double2 v = make_double2(0.0, 0.0);
    if (gi >= 0) v = *reinterpret_cast<const double2*>(coef + (size_t)gi * MS + o);
    if (o < M) c[o] = v.x;
    if (o + 1 < M) c[o + 1] = v.y;
  }
}

// K CG steps on (Sigma + eps I) x = e_y from x = 0 with the candidate's coefficient rows c (slot s
// on lane s * 64 + lane, node 0 = y) and the lanes' neighbour byte offsets nbo into the wave's LDS
// vector pl: the upper bound of Q_yy (bound_value), on every lane.
template <int SM, int M1>
__device__ __forceinline__ double bounds_cg(const double (&c)[SM][M1 + 1],
                                            const unsigned (&nbo)[SM][(M1 + 1) / 2], double* pl,
                                            const int* cntl, int K, double hi_scale, double mu,
                                            int lane) {
  const char* plb = reinterpret_cast<const char*>(pl);
  double r[SM], p[SM], q[SM];
#pragma unroll
  for (int s = 0; s < SM; ++s) {
    const int j = s * 64 + lane;
    r[s] = (j == 0) ? 1.0 : 0.0;
    p[s] = r[s];
    pl[j] = r[s];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double rr = 1.0, g = 0.0, gmu = mu > 0.0 ? 1.0 / mu : 0.0;
  for (int it = 0; it < K; ++it) {
    const int cnt = cntl[it + 1];
    double pq = 0.0;
#pragma unroll
    for (int s = 0; s < SM; ++s) {
      q[s] = 0.0;
      if (s * 64 < cnt) {
        const int j = s * 64 + lane;
        double acc = c[s][0] * p[s];
#pragma unroll
        for (int o = 0; o < M1; ++o) {
          const unsigned off = (nbo[s][o >> 1] >> (16 * (o & 1))) & 0xffffu;
          acc = fma(c[s][1 + o], *reinterpret_cast<const double*>(plb + off), acc);
        }
        q[s] = j < cnt ? acc : 0.0;
        pq = fma(p[s], q[s], pq);
      }
    }
    pq = wave_sum(pq);
    const double alpha = rr / pq;
    g = fma(alpha, rr, g);
    if (it + 1 == K && mu <= 0.0) break;
    double rn = 0.0;
#pragma unroll
    for (int s = 0; s < SM; ++s) {
      r[s] = fma(-alpha, q[s], r[s]);
      rn = fma(r[s], r[s], rn);
    }
    rn = wave_sum(rn);
    // (one division for both: as two, the compiler kept both across the mu branch)
    const double beta = rn / rr;  // = delta_{k+1}
    if (mu > 0.0) gmu = radau_step(gmu, alpha, mu, beta);
    rr = rn;
    if (it + 1 == K) break;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int s = 0; s < SM; ++s) {
      p[s] = fma(beta, p[s], r[s]);
      if (s * 64 < cnt) pl[s * 64 + lane] = p[s];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // (the last step's pl reads fed wave_sum, so the next candidate's pl writes cannot pass them)
  return bound_value(g, gmu, rr, mu, hi_scale);
}

template <int SM, int M1, bool LIST = false>
__global__ __launch_bounds__(BND_T) void exact_bounds_reg_kernel(
    const double* __restrict__ coef, long long I0, long long I1, long long I2,
    const int* __restrict__ tab_off, const int* __restrict__ tab_nb,
    const int* __restrict__ tab_cnt, int T, int K, double hi_scale, double mu, long long c0,
    long long c1, double* __restrict__ qhi, const long long* __restrict__ list = nullptr,
    const int* __restrict__ list_count = nullptr) {
  constexpr int TP = SM * 64;
  __shared__ double plds[BND_WAVES][TP + 1];
  __shared__ short nbl[TP * M1];
  __shared__ short offl[3 * TP];
  __shared__ int cntl[4 * BND_SMAX + 1];
  for (int i = threadIdx.x; i < TP * M1; i += BND_T) {
    const int v = i < T * M1 ? tab_nb[i] : -1;
    nbl[i] = (short)(v >= 0 ? v : TP);
  }
  for (int i = threadIdx.x; i < 3 * TP; i += BND_T) offl[i] = (short)(i < 3 * T ? tab_off[i] : 0);
  for (int i = threadIdx.x; i <= K; i += BND_T) cntl[i] = tab_cnt[i];
  // (the wave index through readfirstlane: the candidate loop and its index decode are then
  // wave-uniform scalar work on the SALU instead of VALU slots)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* pl = plds[wave];
  if (lane == 0) pl[TP] = 0.0;
  __syncthreads();
  constexpr int M = M1 + 1;
  // the lane's neighbour byte offsets into pl, two per register: the reach table is relative, so
  // they are the same for every candidate and every step (read from LDS once, not once per gather)
  constexpr int NP = (M1 + 1) / 2;
  unsigned nbo[SM][NP];
#pragma unroll
  for (int s = 0; s < SM; ++s)
#pragma unroll
    for (int o = 0; o < NP; ++o) {
      const int j = s * 64 + lane;
      const unsigned lo = 8u * (unsigned)nbl[j * M1 + 2 * o];
      const unsigned hi = 2 * o + 1 < M1 ? 8u * (unsigned)nbl[j * M1 + 2 * o + 1] : 0u;
      nbo[s][o] = lo | (hi << 16);
    }
  // the lane's table offsets, likewise once: three signed bytes per slot (|offset| <= K <= 56)
  int ofr[SM];
#pragma unroll
  for (int s = 0; s < SM; ++s) {
    const int j = s * 64 + lane;
    ofr[s] = j < T ? ((offl[3 * j] + 128) | ((offl[3 * j + 1] + 128) << 8) |
                      ((offl[3 * j + 2] + 128) << 16))
                   : -1;
  }
  // 32-bit grid arithmetic (n < 2^31, checked by the caller): the 64-bit divisions and products
  // of the candidate's coordinates and its rows' indices were a large part of a candidate's cost
  const int I0i = (int)I0, I1i = (int)I1, I2i = (int)I2;
  const unsigned I12 = (unsigned)(I1i * I2i);
  // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs, so XCD x (= blockIdx.x
  // mod 8) walks its own contiguous eighth of the candidates and neighbouring candidates, whose
  // reach tables share most coefficient rows, meet in the same L2 (gridDim.x is a multiple of 8)
  // LIST: the candidates list[0 .. *list_count) (the tightening of a refinement event)
  const long long nlist = LIST ? (long long)*list_count : 0;
  const long long per_xcd = (c1 - c0 + 7) / 8, xlo = c0 + (blockIdx.x & 7) * per_xcd;
  const long long xhi = min(c1, xlo + per_xcd);
  for (long long it_y = LIST ? (long long)blockIdx.x * BND_WAVES + wave
                             : xlo + (long long)(blockIdx.x >> 3) * BND_WAVES + wave;
       LIST ? it_y < nlist : it_y < xhi;
       it_y += LIST ? (long long)gridDim.x * BND_WAVES : (long long)(gridDim.x >> 3) * BND_WAVES) {
    const long long y = LIST ? list[it_y] : it_y;
    const unsigned yu = (unsigned)y;
    const int y0 = (int)(yu / I12), yr = (int)(yu - (unsigned)y0 * I12);
    const int y1 = yr / I2i, y2 = yr - y1 * I2i;
    double c[SM][M];
#pragma unroll
    for (int s = 0; s < SM; ++s) {
      int gi = -1;
      if (ofr[s] >= 0) {
        const int g0 = y0 + (ofr[s] & 255) - 128, g1 = y1 + ((ofr[s] >> 8) & 255) - 128,
                  g2 = y2 + ((ofr[s] >> 16) & 255) - 128;
        if ((unsigned)g0 < (unsigned)I0i && (unsigned)g1 < (unsigned)I1i &&
            (unsigned)g2 < (unsigned)I2i)
          gi = (g0 * I1i + g1) * I2i + g2;
      }
      load_coef_row<M>(coef, gi, c[s]);
    }
    // (LIST: both bounds are valid, the smaller one is kept)
    const double ub = bounds_cg<SM, M1>(c, nbo, pl, cntl, K, hi_scale, mu, lane);
    if (lane == 0) qhi[y] = LIST ? fmin(qhi[y], ub) : ub;
  }
}

// Sum over the aligned groups of LPC lanes (LPC = 2, 4, 8, 16, 32 or 64), every lane of a group
// returning its group's sum.  Intra-row DPP for the small groups — quad_perm for xor 1 / 2, then
// row_half_mirror (lane i -> 7 - i within 8: the other quad's sum once each quad is uniform) and
// row_mirror (i -> 15 - i within 16: the other half-row's) — and the CDNA4 permlane swaps above
// 16.  Every step adds two group-uniform partial sums with a commutative +, so the lanes of a
// group end with bit-identical values.
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const unsigned hi =
      (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}

template <int LPC>
__device__ __forceinline__ double group_sum(double v) {
  static_assert(LPC == 2 || LPC == 4 || LPC == 8 || LPC == 16 || LPC == 32 || LPC == 64,
                "group of 2..64 lanes");
  v += dpp64<0xB1>(v);  // quad_perm [1,0,3,2]
  if constexpr (LPC >= 4) v += dpp64<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (LPC >= 8) v += dpp64<0x141>(v);  // row_half_mirror
  if constexpr (LPC >= 16) v += dpp64<0x140>(v); // row_mirror
  if constexpr (LPC >= 32) v = wave_step<16>(v, [](double a, double b) { return a + b; });
  if constexpr (LPC >= 64) v = wave_step<32>(v, [](double a, double b) { return a + b; });
  return v;
}

// One fp64 LDS load from a 32-bit LDS byte address.
__device__ __forceinline__ double lds_f64(unsigned addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) double*>((size_t)addr);
}

// bounds_cg with G candidates per wave: candidate g of the wave on lanes [g LPC, (g + 1) LPC),
// reach-table node j = s LPC + l on slot s of group lane l (T <= 64 nodes, so G slots per lane).
// The wave-uniform part of a CG step (the two reductions, three divisions, the Radau update) is
// then ONE instruction stream for G candidates instead of one per candidate, and the reductions
// are log2(LPC) intra-row steps.  pl: the group's 64 + 1 LDS doubles (the last one 0: the
// neighbour of a node outside the table); nba: the LDS byte addresses of each node's six
// neighbours in pl (fixed for the kernel, so a gather is one ds_read with no address VALU).
template <int G>
__device__ __forceinline__ double bounds_cg_grp(const double (&c)[G][7], const unsigned (&nba)[G][6],
                                                double* pl, const int* cntl, int K, double hi_scale,
                                                double mu, int l, int ctr) {
  constexpr int LPC = 64 / G;
  double r[G], p[G], q[G];
#pragma unroll
  for (int s = 0; s < G; ++s) {
    r[s] = (s == 0 && l == 0) ? 1.0 : 0.0;
    p[s] = r[s];
    pl[s * LPC + l] = r[s];  // (read from step 1 on: the slots step 0 leaves as they are)
  }
  // the Gauss-Radau recursion in projective form, gamma^mu = N / D (radau_step without its
  // division: gamma - alpha = (N - alpha D) / D, so N' = N - alpha D, D' = mu N' + delta D), and
  // alpha = rr / pq, delta = beta = rn / rr from ONE reciprocal of pq rr per step: the division
  // chain that every candidate pair's wave runs drops from three divisions per step to one
  double rr = 1.0, g = 0.0, gN = 1.0, gD = mu;
  for (int it = 0; it < K; ++it) {
    const int cnt = cntl[it + 1];
    double pq = 0.0;
    if (it == 0) {
      // p_0 = e_y: q_0 = S e_y is the centre's column, read off the coefficient rows — node 0's
      // diagonal, and for a neighbour of the centre (ctr = the offset that points back to it) its
      // coefficient toward it — and p_0 . q_0 is the centre's diagonal.  Bit-identical to the
      // gather and the group sum: every other term there is fma(c, 0, .) or + 0.
      double q0 = 0.0;
#pragma unroll
      for (int o = 0; o < 6; ++o) q0 = ctr == o ? c[0][1 + o] : q0;
      if (l == 0) q0 = c[0][0];
#pragma unroll
      for (int s = 0; s < G; ++s) q[s] = s == 0 && l < cnt ? q0 : 0.0;
      pq = __shfl(c[0][0], (threadIdx.x & 63) - l, 64);
    } else {
#pragma unroll
      for (int s = 0; s < G; ++s) {
        q[s] = 0.0;
        if (s * LPC < cnt) {
          double acc = c[s][0] * p[s];
#pragma unroll
          for (int o = 0; o < 6; ++o) acc = fma(c[s][1 + o], lds_f64(nba[s][o]), acc);
          q[s] = s * LPC + l < cnt ? acc : 0.0;
          pq = fma(p[s], q[s], pq);
        }
      }
      pq = group_sum<LPC>(pq);
    }
    const double inv = 1.0 / (pq * rr);
    const double alpha = rr * rr * inv;
    g = fma(alpha, rr, g);
    if (it + 1 == K && mu <= 0.0) break;
    double rn = 0.0;
#pragma unroll
    for (int s = 0; s < G; ++s) {
      r[s] = fma(-alpha, q[s], r[s]);
      rn = fma(r[s], r[s], rn);
    }
    rn = group_sum<LPC>(rn);
    const double beta = rn * pq * inv;  // = rn / rr = delta_{k+1}
    if (mu > 0.0) {
      gN = fma(-alpha, gD, gN);
      gD = fma(mu, gN, beta * gD);
    }
    rr = rn;
    if (it + 1 == K) break;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int s = 0; s < G; ++s) {
      p[s] = fma(beta, p[s], r[s]);
      if (s * LPC < cnt) pl[s * LPC + l] = p[s];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  return bound_value(g, mu > 0.0 ? gN / gD : 0.0, rr, mu, hi_scale);
}

// The all-candidate bounds of exact_bounds_reg_kernel<1, 6> (7-point stencil, reach table of
// T <= 64 nodes: K <= 3) with G candidates per wave (bounds_cg_grp): G consecutive candidates
// y .. y + G - 1 share most of their coefficient rows, so their loads meet in L1 / L2.
// Division of n < 2^31 by a divisor fixed for the launch, by multiply-high (Granlund-Montgomery,
// the "round-up" form): q = (umulhi(n, m) + n) >> l with l = ceil(log2 d),
// m = floor(2^32 (2^l - d) / d) + 1.  Exhaustively checked on the host for the grid sizes used;
// the candidate decode of the bounds pass spent ~60 instructions per candidate pair in two
// generic 32-bit divisions.
struct FastDiv {
  unsigned m;
  int l;
};

static FastDiv fast_div_for(unsigned d) {
  int l = 0;
  while ((1ull << l) < d) ++l;
  return FastDiv{(unsigned)((((1ull << 32) * ((1ull << l) - d)) / d) + 1), l};
}

__device__ __forceinline__ unsigned fast_div(unsigned n, FastDiv f) {
  return (__umulhi(n, f.m) + n) >> f.l;
}

// Candidates per wave: 2 and 4 measured 0.94-0.96 ms per 128^3 K = 3 pass against 1.41 ms for one
// (exact_bounds_reg_kernel<1, 6>), 8 spilled to AGPRs at one wave per SIMD (2.1 ms)
// (profiles/r5_c4_bounds_grouped.jsonl)
constexpr int BND_G = 2;  // candidates per wave (4: no faster, 8: spills)
template <int G>
__global__ __launch_bounds__(BND_T) void exact_bounds_grp_kernel(
    const double* __restrict__ coef, long long I0, long long I1, long long I2,
    const int* __restrict__ tab_off, const int* __restrict__ tab_nb,
    const int* __restrict__ tab_cnt, int T, int K, double hi_scale, double mu, long long c0,
    long long c1, double* __restrict__ qhi, FastDiv div12, FastDiv div2) {
  constexpr int LPC = 64 / G, M1 = 6, M = 7;
  __shared__ double plds[BND_WAVES][G][65];
  __shared__ short nbl[64 * M1];
  __shared__ short offl[3 * 64];
  __shared__ int cntl[4 * BND_SMAX + 1];
  for (int i = threadIdx.x; i < 64 * M1; i += BND_T) {
    const int v = i < T * M1 ? tab_nb[i] : -1;
    nbl[i] = (short)(v >= 0 ? v : 64);
  }
  for (int i = threadIdx.x; i < 3 * 64; i += BND_T) offl[i] = (short)(i < 3 * T ? tab_off[i] : 0);
  for (int i = threadIdx.x; i <= K; i += BND_T) cntl[i] = tab_cnt[i];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gl = lane / LPC, l = lane % LPC;
  double* pl = plds[wave][gl];
  if (l == 0) pl[64] = 0.0;
  __syncthreads();
  // node j = s LPC + l: its neighbours' LDS byte addresses in pl, and its table offset as three
  // signed bytes (-1: beyond the table)
  const unsigned plb = (unsigned)(size_t)(__attribute__((address_space(3))) void*)pl;
  unsigned nba[G][6];
  int ofr[G];
  // the offset of node l (slot 0) that points back to node 0, the centre (-1: none)
  int ctr = -1;
#pragma unroll
  for (int o = 0; o < 6; ++o) ctr = (l < T && nbl[l * M1 + o] == 0) ? o : ctr;
#pragma unroll
  for (int s = 0; s < G; ++s) {
    const int j = s * LPC + l;
#pragma unroll
    for (int o = 0; o < 6; ++o) nba[s][o] = plb + 8u * (unsigned)nbl[j * M1 + o];
    ofr[s] = j < T ? ((offl[3 * j] + 128) | ((offl[3 * j + 1] + 128) << 8) |
                      ((offl[3 * j + 2] + 128) << 16))
                   : -1;
  }
  const int I0i = (int)I0, I1i = (int)I1, I2i = (int)I2;
  const unsigned I12 = (unsigned)(I1i * I2i);
  // XCD-aware order as exact_bounds_reg_kernel: XCD x (= blockIdx.x mod 8) walks its own
  // contiguous eighth of [c0, c1), G candidates per wave
  const long long per_xcd = (c1 - c0 + 7) / 8, xlo = c0 + (blockIdx.x & 7) * per_xcd;
  const long long xhi = min(c1, xlo + per_xcd);
  for (long long yb = xlo + ((long long)(blockIdx.x >> 3) * BND_WAVES + wave) * G; yb < xhi;
       yb += (long long)(gridDim.x >> 3) * BND_WAVES * G) {
    const long long y = yb + gl;
    const bool live = y < xhi;
    const unsigned yu = (unsigned)(live ? y : yb);
    const int y0 = (int)fast_div(yu, div12), yr = (int)(yu - (unsigned)y0 * I12);
    const int y1 = (int)fast_div((unsigned)yr, div2), y2 = yr - y1 * I2i;
    double c[G][M];
#pragma unroll
    for (int s = 0; s < G; ++s) {
      int gi = -1;
      if (ofr[s] >= 0) {
        const int g0 = y0 + (ofr[s] & 255) - 128, g1 = y1 + ((ofr[s] >> 8) & 255) - 128,
                  g2 = y2 + ((ofr[s] >> 16) & 255) - 128;
        if ((unsigned)g0 < (unsigned)I0i && (unsigned)g1 < (unsigned)I1i &&
            (unsigned)g2 < (unsigned)I2i)
          gi = (g0 * I1i + g1) * I2i + g2;
      }
      load_coef_row<M>(coef, gi, c[s]);
    }
    const double ub = bounds_cg_grp<G>(c, nba, pl, cntl, K, hi_scale, mu, l, ctr);
    if (live && l == 0) qhi[y] = ub;
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void exact_score_kernel(EArgs a, const double* __restrict__ qdiag,
                                                          const unsigned char* __restrict__ qexact,
                                                          double* __restrict__ cache) {
  const long long y = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= a.n) return;
  const double nom = sigma_diag<KIND>(a);
  cache[y] = delta_from(nom, qdiag[y], qexact[y] == 1, a.jitter, a.thr);
}

// ---- pre-tightening (vgposp_exact_pretighten) -----------------------------------------------
// With two bound levels, every candidate starts on its K_lo-step bound, and any of them that
// reaches the arg-max during the rounds costs a refinement event (a host round trip, the stall
// kernel) to be tightened.  Those are the candidates at the top of the round-0 cache, so the M
// best (by their upper bound of delta) are tightened at once before the rounds: a three-pass
// radix select of the M-th largest key code (12-bit digits of key_enc's value code, bits 63..28:
// a bin is then 2^-24 of the value wide), the candidates at or above it listed, their K_hi
// bounds (the LIST bounds kernel), their round-0 entries re-scored, and the arg-max keys rebuilt.
// If ties at the threshold would list more than PT_MAX candidates, none is listed (the run then
// tightens on demand only): the set is never cut by the order of the list's atomics.

constexpr int PT_PASSES = 3;  // digits at bits 63..52, 51..40, 39..28 of the value code
__device__ __forceinline__ int pt_shift(int pass) { return 52 - 12 * pass; }

// Histogram of the digit at `shift` of the value codes of the candidates still on their first
// bound whose code matches `prefix` above the digit (pass 0: every such candidate).
__global__ __launch_bounds__(256) void exact_pt_hist_kernel(const double* cache,
                                                            const unsigned char* qexact,
                                                            long long n, const long long* state,
                                                            int pass, unsigned* hist) {
  __shared__ unsigned h[PT_BINS];
  for (int b = threadIdx.x; b < PT_BINS; b += 256) h[b] = 0;
  __syncthreads();
  const int shift = pt_shift(pass);
  const unsigned long long prefix = pass == 0 ? 0ull : (unsigned long long)state[0];
  const unsigned long long pmask = pass == 0 ? 0ull : ~((1ull << (shift + 12)) - 1);
  const int lane = threadIdx.x & 63;
  for (long long y0 = (long long)blockIdx.x * 256; y0 < n; y0 += (long long)gridDim.x * 256) {
    const long long y = y0 + threadIdx.x;
    bool act = false;
    unsigned bin = 0;
    if (y < n && qexact[y] == 0) {
      const unsigned long long c = key_enc(cache[y], y).v;
      act = (c & pmask) == prefix;
      bin = (unsigned)(c >> shift) & (PT_BINS - 1);
    }
    // one LDS atomic per distinct bin of the wave (the first pass puts nearly every code in a few
    // bins: lane-per-lane atomics on one address serialise)
    unsigned long long m = __ballot(act);
    while (m != 0ull) {
      const int l0 = __builtin_ctzll(m);
      const unsigned b0 = __shfl(bin, l0, 64);
      const unsigned long long same = __ballot(act && bin == b0);
      if (lane == l0) atomicAdd(&h[b0], (unsigned)__popcll(same));
      if (act && bin == b0) act = false;
      m &= ~same;
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < PT_BINS; b += 256)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// The digit of pass `pass`: walking the bins from the top, the one where the count of codes at
// or above it reaches the candidates still needed; state[0] gets the code prefix, state[1] the
// need left below the digits above it.  The histogram is cleared for the next pass.  One wave:
// the bins staged in LDS, lane l sums the l-th chunk of 64 from the top, a scan over the lanes
// finds the chunk, and its lane walks it (one thread walking the 4,096 bins in global memory
// took 143 us).
__global__ __launch_bounds__(64) void exact_pt_pick_kernel(long long* state, int pass,
                                                           unsigned* hist) {
  __shared__ unsigned h[PT_BINS];
  __shared__ long long s_res[2];
  const int lane = threadIdx.x;
  for (int b = lane; b < PT_BINS; b += 64) h[b] = hist[b];
  __syncthreads();
  constexpr int CH = PT_BINS / 64;
  const int top = PT_BINS - 1 - CH * lane;  // this lane's chunk: bins top .. top - CH + 1
  unsigned cs = 0;
  for (int j = 0; j < CH; ++j) cs += h[top - j];
  const long long need = state[1];
  // inclusive prefix of the chunk sums from the top chunk (lane 0) down
  long long incl = cs;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const unsigned long long hit = __ballot(incl >= need);
  if (hit == 0ull) {  // fewer candidates than needed: everything from digit 0 up
    if (lane == 63) {
      s_res[0] = 0;
      s_res[1] = incl;
    }
  } else if (lane == __ffsll((long long)hit) - 1) {
    long long cum = incl - cs;
    int d = top - CH + 1;
    for (int j = 0; j < CH; ++j) {
      if (cum + h[top - j] >= need) {
        d = top - j;
        break;
      }
      cum += h[top - j];
    }
    s_res[0] = d;
    s_res[1] = cum;
  }
  __syncthreads();
  if (lane == 0) {
    const int shift = pt_shift(pass);
    state[0] = (long long)((unsigned long long)state[0] |
                           ((unsigned long long)s_res[0] << shift));
    state[1] = need - s_res[1];
  }
  for (int b = lane; b < PT_BINS; b += 64) hist[b] = 0;
}

// List the candidates on their first bound with a code >= the threshold (at most PT_MAX; the
// order of the list does not matter: each candidate's bound is its own).
__global__ __launch_bounds__(256) void exact_pt_list_kernel(const double* cache,
                                                            const unsigned char* qexact,
                                                            long long n, long long* state,
                                                            long long* list, int* count) {
  const unsigned long long thr = (unsigned long long)state[0];
  const int lane = threadIdx.x & 63;
  for (long long y0 = (long long)blockIdx.x * 256; y0 < n; y0 += (long long)gridDim.x * 256) {
    const long long y = y0 + threadIdx.x;
    const bool in = y < n && qexact[y] == 0 && key_enc(cache[y], y).v >= thr;
    // one atomic per wave (lane-per-lane atomics on one counter serialise); the listed SET does
    // not depend on the order the waves get their ranges in
    const unsigned long long m = __ballot(in);
    if (m == 0ull) continue;
    unsigned long long base = 0;
    if (lane == __builtin_ctzll(m))
      base = atomicAdd((unsigned long long*)&state[3], (unsigned long long)__popcll(m));
    base = __shfl(base, __builtin_ctzll(m), 64);
    if (in) {
      const unsigned long long i = base + __popcll(m & ((1ull << lane) - 1ull));
      if (i < (unsigned long long)PT_MAX) list[i] = y;
    }
  }
  (void)count;
}

__global__ void exact_pt_init_kernel(long long* state, long long M) {
  if (threadIdx.x == 0) {
    state[0] = 0;
    state[1] = M;
    state[2] = 0;
    state[3] = 0;
  }
}

__global__ void exact_pt_count_kernel(const long long* state, int* count, int* ctl) {
  if (threadIdx.x == 0) {
    const int c = state[3] <= PT_MAX ? (int)state[3] : 0;
    count[0] = c;
    ctl[CTL_TIGHT] += c;
  }
}

// Round-0 entries of the listed candidates from their tightened bounds; qexact <- 2.
template <int KIND>
__global__ __launch_bounds__(256) void exact_pt_score_kernel(EArgs a, const double* qdiag,
                                                             unsigned char* qexact, double* cache,
                                                             const long long* list,
                                                             const int* count) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= *count) return;
  const long long y = list[i];
  cache[y] = delta_from(sigma_diag<KIND>(a), qdiag[y], false, a.jitter, a.thr);
  qexact[y] = 2;
}

// One wave: key of block b (entries [b EB, (b+1) EB) of the cache, selected ones excluded).
__device__ __forceinline__ void wave_block_key(const double* cache, const unsigned char* sel,
                                               long long n, long long b, double* bval,
                                               long long* bidx) {
  const int lane = threadIdx.x & 63;
  Key k{0ull, 0ull};
#pragma unroll
  for (int e = lane; e < EB; e += 64) {
    const long long y = b * EB + e;
    if (y < n && !sel[y]) {
      key_take_max(k, key_enc(cache[y], y));
    }
  }
  k = wave_keymax(k);
  if (lane == 0) {
    bval[b] = key_value(k);
    bidx[b] = key_index(k);
  }
}

// Up to NB blocks blk[q] (q < nb) at once, one wave: every block's entries are loaded before any
// key is reduced or stored, so the blocks' load latencies overlap.
template <int NB>
__device__ __forceinline__ void wave_block_keys(const double* cache, const unsigned char* sel,
                                                long long n, const long long* blk, int nb,
                                                double* bval, long long* bidx) {
  const int lane = threadIdx.x & 63;
  constexpr int PER = EB / 64;
  double c[NB][PER];
  unsigned char sl[NB][PER];
#pragma unroll
  for (int q = 0; q < NB; ++q)
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const long long y = q < nb ? blk[q] * EB + e * 64 + lane : n;
      c[q][e] = y < n ? cache[y] : 0.0;
      sl[q][e] = y < n ? sel[y] : 1;
    }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (q >= nb) break;
    Key k{0ull, 0ull};
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      key_take_max(k, key_enc(c[q][e], sl[q][e] ? -1 : blk[q] * EB + e * 64 + lane));
    }
    k = wave_keymax(k);
    if (lane == 0) {
      bval[blk[q]] = key_value(k);
      bidx[blk[q]] = key_index(k);
    }
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

// Workgroup-wide arg-max over the superblock keys (placement_algorithm2.py:24-50 via
// sparse_argmax_cache_linear); every thread returns it.
__device__ long long block_argmax(const ExactWS& w, long long nsb) {
  __shared__ double sv[SEL_THREADS / 64];
  __shared__ long long si[SEL_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double v = 0.0;
  long long idx = -1;
  for (long long s = t; s < nsb; s += SEL_THREADS) {
    if (w.sidx[s] >= 0 && key_gt(w.sval[s], w.sidx[s], v, idx)) {
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
    if (lane == 0) si[0] = idx;
  }
  __syncthreads();
  const long long r = si[0];
  __syncthreads();
  return r;
}

// Refresh the block key and superblock key of candidate y (one wave).
__device__ __forceinline__ void wave_refresh_keys(const double* cache, const unsigned char* sel,
                                                  const ExactWS& w, long long n, long long nblk,
                                                  long long y) {
  const long long b = y / EB;
  wave_block_key(cache, sel, n, b, w.bval, w.bidx);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  wave_super_key(w.bval, w.bidx, nblk, b / ESB, w.sval, w.sidx);
}

// The pick of round `round` (selected-inverse path): A <- A u {y*}, the cache entry of y* <- 0
// (snippets_a3.py:162-168), its keys refreshed; CG set up for q = Q e_{y*} in slot `round`.
__global__ __launch_bounds__(SEL_THREADS) void exact_select_kernel(
    double* cache, unsigned char* sel, long long I0, long long I1, long long I2, ExactWS w,
    long long nblk, long long nsb, int round, long long* picks, double* pick_delta) {
  const long long n = I0 * I1 * I2;
  const long long a = block_argmax(w, nsb);
  if (threadIdx.x == 0) {
    picks[round] = a;
    if (pick_delta) pick_delta[round] = a >= 0 ? cache[a] : 0.0;
    w.slot_of_round[round] = round;
    if (a >= 0) {
      sel[a] = 1;
      cache[a] = 0.0;
    }
  }
  __syncthreads();
  if (a >= 0 && threadIdx.x < 64) wave_refresh_keys(cache, sel, w, n, nblk, a);
}

// Column j of a batched CG solve: its vectors and scalars in the workspace.
struct CGCol {
  double *r, *p0, *p1, *q, *part_pq, *part_rr, *rr;
  int* state;
};

__device__ __forceinline__ CGCol cg_col(const ExactWS& w, int j) {
  const size_t bv = (size_t)(w.b0 * w.b1 * w.b2);
  CGCol c;
  c.r = w.r + j * bv;
  c.p0 = w.p0 + j * bv;
  c.p1 = w.p1 + j * bv;
  c.q = w.q + j * bv;
  c.part_pq = w.part_pq + (size_t)j * CG_BLOCKS;
  c.part_rr = w.part_rr + (size_t)j * CG_BLOCKS;
  c.rr = w.rr + (size_t)j * (CG_MAXIT + 2);
  c.state = w.cgstate + 4 * j;
  return c;
}

// 7-point stencil (the reference's beta = 4 taper): after `it` iterations the Krylov vectors of
// e_c are supported on the Manhattan ball |d0| + |d1| + |d2| <= it around c, an octahedron of
// about (4/3) R^3 nodes against the (2R + 1)^3 of the bounding cube (6x fewer at R = 29).  Its
// nodes are walked row by row: the (d0, d1) rows with |d0| + |d1| <= R (2R^2 + 2R + 1 of them),
// each a contiguous d2 run of 2 (R - |d0| - |d1|) + 1 nodes, one wave per row.
__device__ __forceinline__ long long diamond_rows(long long R) { return 2 * R * R + 2 * R + 1; }

// Row `rw` (< diamond_rows(R)) of the diamond, rows ordered by s = |d0| + |d1| (shell s >= 1 has
// 4 s rows) -> (d0, d1).
__device__ __forceinline__ void diamond_row(long long rw, long long& d0, long long& d1) {
  if (rw == 0) {
    d0 = d1 = 0;
    return;
  }
  // shell s: rows [2 s^2 - 2 s + 1, 2 s^2 + 2 s + 1)
  long long s = (long long)((sqrt(2.0 * (double)rw - 1.0) + 1.0) * 0.5);
  while (2 * s * s - 2 * s + 1 > rw) --s;
  while (2 * (s + 1) * (s + 1) - 2 * (s + 1) + 1 <= rw) ++s;
  const long long e = rw - (2 * s * s - 2 * s + 1);  // 0 .. 4 s - 1 around the diamond
  const long long side = e / s, k = e % s;
  switch (side) {
    case 0: d0 = s - k; d1 = k; break;        // ( s, 0) -> (0,  s)
    case 1: d0 = -k; d1 = s - k; break;       // ( 0, s) -> (-s, 0)
    case 2: d0 = -s + k; d1 = -k; break;      // (-s, 0) -> (0, -s)
    default: d0 = k; d1 = -s + k; break;      // ( 0,-s) -> ( s, 0)
  }
}

// A CG launch's 1-D grid over nb columns x nbx blocks.  With nb a multiple of 8 every column's
// blocks run on ONE XCD (workgroup id mod 8 = the XCD): column j on XCD j mod 8, so the
// neighbour rows a block gathers — written by the column's other blocks — are in that XCD's L2.
struct CGBlk {
  int col, bx, nbx;
};

__device__ __forceinline__ CGBlk cg_blk(int nb) {
  CGBlk b;
  b.nbx = (int)gridDim.x / nb;
  const int id = (int)blockIdx.x;
  if ((nb & 7) == 0) {
    const int x = id & 7, k = id >> 3;
    b.col = x + 8 * (k / b.nbx);
    b.bx = k % b.nbx;
  } else {
    b.col = id / b.nbx;
    b.bx = id % b.nbx;
  }
  return b;
}

// Start the CG solves of S x_j = e_{c_j} (c_j = centers[j], j = blockIdx.y) into column slots
// slots[j]: r, p0, p1 and the column zeroed except r = e_c, the box [c - H, c + H] per axis
// shifted inside the grid -> boxlo[slot], rr[0] = 1, state cleared (done when there is no
// candidate).
template <bool OCT>
__global__ __launch_bounds__(256) void exact_cg_start_kernel(ExactWS w, long long I0, long long I1,
                                                             long long I2, const int* slots,
                                                             const long long* centers) {
  const int j = blockIdx.y;
  const CGCol cc = cg_col(w, j);
  const long long c = centers[j];
  const int slot = slots[j];
  const long long bv = w.b0 * w.b1 * w.b2;
  double* x = w.Qcols + (size_t)slot * bv;
  long long lc = -1, lo0 = 0, lo1 = 0, lo2 = 0;
  if (c >= 0) {
    const long long a0 = c / (I1 * I2), a1 = (c / I2) % I1, a2 = c % I2;
    lo0 = min(max(a0 - w.H, 0LL), I0 - w.b0);
    lo1 = min(max(a1 - w.H, 0LL), I1 - w.b1);
    lo2 = min(max(a2 - w.H, 0LL), I2 - w.b2);
    lc = ((a0 - lo0) * w.b1 + (a1 - lo1)) * w.b2 + (a2 - lo2);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      w.boxlo[3 * slot] = lo0;
      w.boxlo[3 * slot + 1] = lo1;
      w.boxlo[3 * slot + 2] = lo2;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    cc.rr[0] = 1.0;
    cc.state[0] = c >= 0 ? 0 : 1;
    cc.state[1] = 0;
  }
  if (c < 0) return;  // an unused column of the batch: its slot (if any) belongs to someone else
  if (!OCT) {
    for (long long l = (long long)blockIdx.x * 256 + threadIdx.x; l < bv;
         l += (long long)gridDim.x * 256) {
      cc.r[l] = l == lc ? 1.0 : 0.0;
      cc.p0[l] = 0.0;
      cc.p1[l] = 0.0;
      x[l] = 0.0;
    }
    return;
  }
  // 7-point walk: r, p0 and p1 are read only on the Manhattan ball of radius H + 1 around c (the
  // walk's nodes, radius <= H, and their face neighbours), so only that ball (inside the box) is
  // cleared; the column x is read anywhere in the box (qslot_at) and is cleared whole.
  for (long long l = (long long)blockIdx.x * 256 + threadIdx.x; l < bv;
       l += (long long)gridDim.x * 256)
    x[l] = 0.0;
  const long long a0 = c / (I1 * I2), a1 = (c / I2) % I1, a2 = c % I2;
  const long long R = w.H + 1;
  const int lane = threadIdx.x & 63, sub = lane / CG_SEG, sl = lane % CG_SEG;
  const long long nrows = diamond_rows(R);
  for (long long rw = (((long long)blockIdx.x * 256 + threadIdx.x) >> 6) * CG_RPW + sub; rw < nrows;
       rw += (((long long)gridDim.x * 256) >> 6) * CG_RPW) {
    long long d0, d1;
    diamond_row(rw, d0, d1);
    const long long j0 = a0 + d0 - lo0, j1 = a1 + d1 - lo1;
    if (j0 < 0 || j0 >= w.b0 || j1 < 0 || j1 >= w.b1) continue;
    const long long h = R - (d0 < 0 ? -d0 : d0) - (d1 < 0 ? -d1 : d1);
    const long long base = (j0 * w.b1 + j1) * w.b2;
    const long long c2 = a2 - lo2;
    const long long k0 = max(c2 - h, 0LL), k1 = min(c2 + h, w.b2 - 1);
    for (long long k = k0 + sl; k <= k1; k += CG_SEG) {
      const long long l = base + k;
      cc.r[l] = l == lc ? 1.0 : 0.0;
      cc.p0[l] = 0.0;
      cc.p1[l] = 0.0;
    }
  }
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

__device__ __forceinline__ void block_partial(double v, double* part, double* red, int bx) {
  v = wave_sum(v);
  const int t = threadIdx.x;
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < CG_T / 64; ++i) s += red[i];
    part[bx] = s;
  }
}

// The active cube of CG iteration it: the nodes within (it + 1) stencil radii of the centre
// (the iterate's support), inside the column's box.  Thread t of the launch handles cube node t.
struct ActiveCube {
  long long c0, c1, c2, e1, e2, ne;
  long long lo0, lo1, lo2;
};

__device__ __forceinline__ ActiveCube active_cube(const ExactWS& w, long long I1, long long I2,
                                                  int slot, long long a, int it, int srad) {
  ActiveCube q;
  const long long a0 = a / (I1 * I2), a1 = (a / I2) % I1, a2 = a % I2;
  q.lo0 = w.boxlo[3 * slot];
  q.lo1 = w.boxlo[3 * slot + 1];
  q.lo2 = w.boxlo[3 * slot + 2];
  const long long rad = min((long long)(it + 1) * srad, w.H);
  q.c0 = max(a0 - rad, q.lo0);
  q.c1 = max(a1 - rad, q.lo1);
  q.c2 = max(a2 - rad, q.lo2);
  const long long e0 = min(a0 + rad, q.lo0 + w.b0 - 1) - q.c0 + 1;
  q.e1 = min(a1 + rad, q.lo1 + w.b1 - 1) - q.c1 + 1;
  q.e2 = min(a2 + rad, q.lo2 + w.b2 - 1) - q.c2 + 1;
  q.ne = e0 * q.e1 * q.e2;
  return q;
}

// Visit the active nodes of iteration `it` (grid coordinates): the active cube, thread t its
// t-th node; or (OCT) the Manhattan ball of radius it + 1 around the centre a, one wave per
// diamond row, lane l the row's l-th node (rows longer than 64 nodes: l, l + 64, ...).
// Thread `tid` of `nth` threads walking the region; waves take consecutive groups of CG_RPW
// diamond rows.
template <bool OCT, class F>
__device__ __forceinline__ void cg_walk(const ExactWS& w, const ActiveCube& q, long long I0,
                                        long long I1, long long I2, long long a, int it,
                                        long long tid, long long nth, F&& f) {
  if (!OCT) {
    for (long long t = tid; t < q.ne; t += nth) {
      const long long g0 = q.c0 + t / (q.e1 * q.e2), g1 = q.c1 + (t / q.e2) % q.e1,
                      g2 = q.c2 + t % q.e2;
      f(g0, g1, g2);
    }
    return;
  }
  const long long R = min((long long)it + 1, w.H);
  const long long a0 = a / (I1 * I2), a1 = (a / I2) % I1, a2 = a % I2;
  // CG_SEG lanes per diamond row (a row holds 2h + 1 <= 2R + 1 nodes, ~R/2 on average: one row
  // per wave left most lanes idle and quadrupled the waves of the late iterations)
  const int lane = threadIdx.x & 63, sub = lane / CG_SEG, sl = lane % CG_SEG;
  const long long nrows = diamond_rows(R);
  for (long long rw = (tid >> 6) * CG_RPW + sub; rw < nrows; rw += (nth >> 6) * CG_RPW) {
    long long d0, d1;
    diamond_row(rw, d0, d1);
    const long long g0 = a0 + d0, g1 = a1 + d1;
    if (g0 < 0 || g0 >= I0 || g1 < 0 || g1 >= I1) continue;
    const long long h = R - (d0 < 0 ? -d0 : d0) - (d1 < 0 ? -d1 : d1);
    const long long lo2 = max(a2 - h, 0LL), hi2 = min(a2 + h, I2 - 1);
    for (long long g2 = lo2 + sl; g2 <= hi2; g2 += CG_SEG) f(g0, g1, g2);
  }
}

// CG iteration it, part A, for column j = blockIdx.y of a batch: beta from the last residual
// norms, p_it = r + beta p_{it-1} (computed for the neighbours on the fly, written for this
// thread's own node), q = (S + eps I) p_it and the partials of p_it . q.  Converged
// (|r|^2 <= tol2) -> every block of the column returns; block 0 records it.  The launch covers
// the active cube (np_prev: the grid of the previous B launch, whose partials hold |r_it|^2).
template <bool OCT>
__global__ __launch_bounds__(CG_T) void exact_cg_a_kernel(ExactWS w, long long I0, long long I1,
                                                          long long I2, const int* offs, int m1,
                                                          int srad, const int* slots,
                                                          const long long* centers, int it,
                                                          int np_prev, double tol2, int nb) {
  __shared__ double red[CG_T / 64];
  const CGBlk bk = cg_blk(nb);
  const CGCol cc = cg_col(w, bk.col);
  if (cc.state[0]) return;
  // |r_it|^2 from the B kernel's partials (every block sums them in the same order)
  const double rr = it == 0 ? cc.rr[0] : sum_partials(cc.part_rr, np_prev, red);
  if (it > 0 && bk.bx == 0 && threadIdx.x == 0) cc.rr[it] = rr;
  if (rr <= tol2) {
    if (bk.bx == 0 && threadIdx.x == 0) {
      cc.state[0] = 1;
      cc.state[1] = it;
    }
    return;
  }
  const double beta = it == 0 ? 0.0 : rr / cc.rr[it - 1];
  const double* pold = (it & 1) ? cc.p0 : cc.p1;  // p_{it-1}
  double* pnew = (it & 1) ? cc.p1 : cc.p0;        // p_it
  const ActiveCube q = active_cube(w, I1, I2, slots[bk.col], centers[bk.col], it, srad);
  const int m = m1 + 1;
  double acc = 0.0;
  if constexpr (OCT) {
    // the 7-point stencil (m1 == 6): the six neighbour offsets in box-index units, and the node's
    // six neighbours loaded unconditionally — an index outside the box is replaced by the node's
    // own and its value by 0 — so all twelve loads issue back to back.  Same sum, same order: a
    // skipped term of the generic walk (coefficient 0 outside the grid, or outside the box) adds
    // fma(cv, 0 or pj, s) = s here.
    int od[6][3];
    long long dl[6];
#pragma unroll
    for (int o = 0; o < 6; ++o) {
      od[o][0] = offs[3 * o];
      od[o][1] = offs[3 * o + 1];
      od[o][2] = offs[3 * o + 2];
      dl[o] = ((long long)od[o][0] * w.b1 + od[o][1]) * w.b2 + od[o][2];
    }
    auto node7 = [&](long long g0, long long g1, long long g2) {
      const long long j0 = g0 - q.lo0, j1 = g1 - q.lo1, j2 = g2 - q.lo2;
      const long long l = (j0 * w.b1 + j1) * w.b2 + j2;
      const double* c = w.coef + ((g0 * I1 + g1) * I2 + g2) * coef_stride(7);
      double cv[7];
#pragma unroll
      for (int o = 0; o < 7; ++o) cv[o] = c[o];
      double rv[7], pv[7];
      bool in[7];
      in[0] = true;
#pragma unroll
      for (int o = 0; o < 6; ++o) {
        const long long k0 = j0 + od[o][0], k1 = j1 + od[o][1], k2 = j2 + od[o][2];
        in[1 + o] = k0 >= 0 && k0 < w.b0 && k1 >= 0 && k1 < w.b1 && k2 >= 0 && k2 < w.b2;
      }
#pragma unroll
      for (int o = 0; o < 7; ++o) {
        const long long jj = o == 0 ? l : (in[o] ? l + dl[o - 1] : l);
        rv[o] = cc.r[jj];
        pv[o] = it == 0 ? 0.0 : pold[jj];
      }
      const double pi = it == 0 ? rv[0] : fma(beta, pv[0], rv[0]);
      double s = cv[0] * pi;
#pragma unroll
      for (int o = 1; o < 7; ++o) {
        const double pj = it == 0 ? rv[o] : fma(beta, pv[o], rv[o]);
        s = fma(cv[o], in[o] ? pj : 0.0, s);
      }
      pnew[l] = pi;
      cc.q[l] = s;
      acc = fma(pi, s, acc);
    };
    cg_walk<OCT>(w, q, I0, I1, I2, centers[bk.col], it,
                 (long long)bk.bx * CG_T + threadIdx.x, (long long)bk.nbx * CG_T, node7);
    block_partial(acc, cc.part_pq, red, bk.bx);
    return;
  }
  auto node = [&](long long g0, long long g1, long long g2) {
    const long long l = ((g0 - q.lo0) * w.b1 + (g1 - q.lo1)) * w.b2 + (g2 - q.lo2);
    const double pi = it == 0 ? cc.r[l] : fma(beta, pold[l], cc.r[l]);
    const double* c = w.coef + ((g0 * I1 + g1) * I2 + g2) * coef_stride(m);
    double s = c[0] * pi;
    for (int o = 0; o < m1; ++o) {
      const double cv = c[1 + o];
      if (cv == 0.0) continue;  // outside the grid (inner loop: continue is the o-loop's)
      const long long j0 = g0 + offs[3 * o] - q.lo0, j1 = g1 + offs[3 * o + 1] - q.lo1,
                      j2 = g2 + offs[3 * o + 2] - q.lo2;
      if (j0 < 0 || j0 >= w.b0 || j1 < 0 || j1 >= w.b1 || j2 < 0 || j2 >= w.b2) continue;
      const long long j = (j0 * w.b1 + j1) * w.b2 + j2;
      const double pj = it == 0 ? cc.r[j] : fma(beta, pold[j], cc.r[j]);
      s = fma(cv, pj, s);
    }
    pnew[l] = pi;
    cc.q[l] = s;
    acc = fma(pi, s, acc);
  };
  cg_walk<OCT>(w, q, I0, I1, I2, centers[bk.col], it, (long long)bk.bx * CG_T + threadIdx.x,
               (long long)bk.nbx * CG_T, node);
  block_partial(acc, cc.part_pq, red, bk.bx);
}

// CG iteration it, part B: alpha = |r|^2 / p.q, x += alpha p, r -= alpha q, partials of |r|^2
// (same grid and cube as part A; x = the column slot's box vector).
template <bool OCT>
__global__ __launch_bounds__(CG_T) void exact_cg_b_kernel(ExactWS w, long long I0, long long I1,
                                                          long long I2, int srad, const int* slots,
                                                          const long long* centers, int it,
                                                          int nb) {
  __shared__ double red[CG_T / 64];
  const CGBlk bk = cg_blk(nb);
  const CGCol cc = cg_col(w, bk.col);
  if (cc.state[0]) return;
  const double pq = sum_partials(cc.part_pq, bk.nbx, red);  // the A kernel's grid
  const double alpha = cc.rr[it] / pq;
  const double* p = (it & 1) ? cc.p1 : cc.p0;
  const int slot = slots[bk.col];
  double* x = w.Qcols + (size_t)slot * (w.b0 * w.b1 * w.b2);
  const ActiveCube q = active_cube(w, I1, I2, slot, centers[bk.col], it, srad);
  double acc = 0.0;
  auto node = [&](long long g0, long long g1, long long g2) {
    const long long l = ((g0 - q.lo0) * w.b1 + (g1 - q.lo1)) * w.b2 + (g2 - q.lo2);
    x[l] = fma(alpha, p[l], x[l]);
    const double ri = fma(-alpha, cc.q[l], cc.r[l]);
    cc.r[l] = ri;
    acc = fma(ri, ri, acc);
  };
  cg_walk<OCT>(w, q, I0, I1, I2, centers[bk.col], it, (long long)bk.bx * CG_T + threadIdx.x,
               (long long)bk.nbx * CG_T, node);
  block_partial(acc, cc.part_rr, red, bk.bx);
}

// Top-B selection in one workgroup (the refinement batch of a stalled round).  Keys order by
// value, then LOWER index (key_gt: a strict total order on distinct indices, so every selection
// below is exact).  A wave extracts the B best of the items its lanes hold by B wave arg-maxes,
// each removing the winner from its lane; the 16 waves' lists are then merged the same way by
// wave 0.  (Round 3's version ran B block-wide arg-maxes with two barriers each per level: 750 us
// for B = 32.)
template <int P>
__device__ __forceinline__ void wave_topb(double (&v)[P], long long (&id)[P], int B, double* ov,
                                          long long* oi, int* taken = nullptr) {
  const int lane = threadIdx.x & 63;
  // the branch-free encoded order, held as two plain arrays and selected component-wise (an
  // array of Key structs selected as a whole went through scratch memory: 540 us per stall)
  unsigned long long kv[P], ki[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const Key e = key_enc(v[p], id[p]);
    kv[p] = e.v;
    ki[p] = e.i;
  }
  for (int b = 0; b < B; ++b) {
    Key best{kv[0], ki[0]};
#pragma unroll
    for (int p = 1; p < P; ++p) key_take_max(best, Key{kv[p], ki[p]});
    best = wave_keymax(best);
    if (lane == 0) {
      ov[b] = key_value(best);
      oi[b] = key_index(best);
    }
    if (best.v == 0ull) continue;  // fewer than B items: the rest stay -1
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bool hit = ki[p] == best.i;
      kv[p] = hit ? 0ull : kv[p];
      ki[p] = hit ? 0ull : ki[p];
    }
  }
  if (taken) {  // bit p: item p was among the B taken
    int m = 0;
#pragma unroll
    for (int p = 0; p < P; ++p) m |= (id[p] >= 0 && ki[p] == 0ull) ? (1 << p) : 0;
    *taken = m;
  }
}

// The exact top B of the n = 64 Q items staged in LDS (sv / si), one wave, by rank: item k's rank
// is the number of items with a greater key (a strict total order: keys carry distinct indices),
// so items of rank < B land at ov / oi[rank] in the order B wave arg-maxes would extract them;
// if fewer than B items are real, slot nreal gets the empty key (value 0, index -1), which ends the
// list.  Lane l holds items l Q .. l Q + Q - 1; taken (bit q): its item q was among the B.  The
// encoded keys are staged in kv_s / ki_s first, then every lane compares its items against all n
// broadcast LDS reads with no serial dependency — where B successive wave arg-maxes (each a
// six-step cross-lane reduction) were a serial chain of B.
template <int Q>
__device__ __forceinline__ void wave_rank_topb(const double* sv, const long long* si, int B,
                                               unsigned long long* kv_s, unsigned long long* ki_s,
                                               double* ov, long long* oi, int& taken) {
  const int lane = threadIdx.x & 63;
  constexpr int N = 64 * Q;
  unsigned long long mv[Q], mi[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int k = lane * Q + q;
    const Key e = key_enc(sv[k], si[k]);
    mv[q] = e.v;
    mi[q] = e.i;
    kv_s[k] = e.v;
    ki_s[k] = e.i;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int rank[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) rank[q] = 0;
#pragma unroll 16
  for (int j = 0; j < N; ++j) {  // (unrolled: sixteen broadcast reads in flight, not one)
    const Key o{kv_s[j], ki_s[j]};
#pragma unroll
    for (int q = 0; q < Q; ++q) rank[q] += key_enc_gt(o, Key{mv[q], mi[q]}) ? 1 : 0;
  }
  taken = 0;
  int real = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const bool live = mv[q] != 0ull;
    real += live ? 1 : 0;
    if (live && rank[q] < B) {
      ov[rank[q]] = key_value(Key{mv[q], mi[q]});
      oi[rank[q]] = key_index(Key{mv[q], mi[q]});
      taken |= 1 << q;
    }
  }
  real = (int)wave_sum((double)real);
  if (lane == 0 && real < B) {
    ov[real] = 0.0;
    oi[real] = -1;
  }
}

// The B best of `count` items (key(i, v, idx), i < count <= P * SEL_THREADS) -> out[0] = how many
// (<= B), out[1 ..] = their indices, best first.  sv / si: LDS scratch [16 B].  Whole workgroup.
constexpr int TOPW = 8;  // block_topb_keys' first pass: each wave's best TOPW

// out[0] = the number of leading valid indices among list[0 .. B) (the list ends at the first
// -1), out[1 ..] = those indices.  One wave, B <= 63.
__device__ __forceinline__ void topb_out(const long long* list, int B, long long* out) {
  const int lane = threadIdx.x & 63;
  const long long k = lane < B ? list[lane] : -1;
  const int c = __builtin_ctzll(__ballot(lane >= B || k < 0));
  if (lane < c) out[1 + lane] = k;
  if (lane == 0) out[0] = c;
}

template <int P, class KeyFn>
__device__ int block_topb_keys(int count, int B, KeyFn key, double* sv, long long* si,
                               long long* out, unsigned long long* dt = nullptr) {
  const int t = threadIdx.x, wave = t >> 6;
  constexpr int NW = SEL_THREADS / 64;
  double v[P];
  long long id[P];
  // items interleaved over the waves by 16-item chunks (chunk c of each SEL_THREADS group to wave
  // c mod NW, lanes 16 (c / NW) .. + 15): the best entries of a block are grid neighbours and
  // would otherwise share a wave and force the second pass, while a wave's loads stay four
  // contiguous 128-byte runs (one item per lane at a stride of NW items had every lane on its own
  // cache line)
  const int tw = (((t & 63) >> 4) * NW + wave) * 16 + (t & 15);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int i = tw + p * SEL_THREADS;
    v[p] = 0.0;
    id[p] = -1;
    if (i < count) key(i, v[p], id[p]);
  }
  // Pass 1: each wave's best TOPW entries, merged by wave 0.  The merged top B is exact unless
  // some wave had all TOPW of its entries taken (it may hold more of the top B): only then every
  // wave extracts its best B (pass 2).  (B passes of a wave arg-max per wave were 170 us of a
  // stall at 128^3; the first pass alone is a quarter of that.)
  __shared__ int s_full;
  if (B > TOPW) {
    wave_topb<P>(v, id, TOPW, sv + wave * TOPW, si + wave * TOPW);
    __syncthreads();
    if (dt != nullptr && t == 0) *dt = __builtin_amdgcn_s_memrealtime();  // (debug builds)
    if (wave == 0) {
      constexpr int Q1 = NW * TOPW / 64;  // items per lane; lanes 4s .. 4s + 3 hold wave s's
      static_assert(Q1 == 2 && TOPW == 8, "merge layout: two items per lane, four lanes per wave");
      double v1[Q1];
      long long id1[Q1];
      const int lane = t & 63;
#pragma unroll
      for (int q = 0; q < Q1; ++q) {
        v1[q] = sv[lane * Q1 + q];
        id1[q] = si[lane * Q1 + q];
      }
      int tk = 0;
      __shared__ unsigned long long s_kv[NW * TOPW], s_ki[NW * TOPW];
      (void)v1;
      (void)id1;
      wave_rank_topb<Q1>(sv, si, B, s_kv, s_ki, sv + NW * CG_B, si + NW * CG_B, tk);
      const unsigned long long m0 = __ballot(tk & 1), m1 = __ballot(tk & 2);
      int full = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w)
        full |= (((m0 >> (4 * w)) & 0xFull) == 0xFull) && (((m1 >> (4 * w)) & 0xFull) == 0xFull);
      if (lane == 0) s_full = full;
    }
    __syncthreads();
    if (!s_full) {
      if (wave == 0) topb_out(si + NW * CG_B, B, out);
      __syncthreads();
      return (int)out[0];
    }
  }
  wave_topb<P>(v, id, B, sv + wave * B, si + wave * B);
  __syncthreads();
  if (wave == 0) {
    constexpr int Q = (NW * CG_B + 63) / 64;
    double v2[Q];
    long long id2[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = (t & 63) + 64 * q;
      v2[q] = i < NW * B ? sv[i] : 0.0;
      id2[q] = i < NW * B ? si[i] : -1;
    }
    wave_topb<Q>(v2, id2, B, sv + NW * CG_B, si + NW * CG_B);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    topb_out(si + NW * CG_B, B, out);
  }
  __syncthreads();
  return (int)out[0];
}

// The B best cache entries over V \ A: they lie in the B best blocks, which lie in the B best
// superblocks (a key is its range's maximum).  Keys carry the candidate index, so a selected key
// names its block (y / EB) and superblock (y / (EB ESB)).  out[0] = count, out[1 ..] = the
// candidates, best first (out[1] is the arg-max).  The whole workgroup calls it.
__device__ void block_topb_entries(const double* cache, const unsigned char* sel, long long n,
                                   const ExactWS& w, long long nblk, long long nsb, int B,
                                   long long* out, unsigned long long* dt = nullptr) {
  // (dt: debug builds with VGPOSP_EXACT_DBG=3 stamp the three levels, dt[1] .. dt[4])
#define DBG_TB(k) \
  if (dt != nullptr && threadIdx.x == 0) dt[k] = __builtin_amdgcn_s_memrealtime();
  constexpr int NW = SEL_THREADS / 64;
  __shared__ double sv[NW * CG_B + CG_B];
  __shared__ long long si[NW * CG_B + CG_B];
  __shared__ long long sbs[CG_B + 1], blks[CG_B + 1];
  // superblocks (nsb <= 8 SEL_THREADS: 134 M candidates)
  auto skey = [&](int i, double& v, long long& k) {
    v = w.sval[i];
    k = w.sidx[i];
  };
  int ns = 0;
  if (nsb <= SEL_THREADS) ns = block_topb_keys<1>((int)nsb, B, skey, sv, si, sbs);
  else if (nsb <= 8 * SEL_THREADS) ns = block_topb_keys<8>((int)nsb, B, skey, sv, si, sbs);
  if (ns == 0) {  // (no candidate, or too many superblocks: the caller falls back to the arg-max)
    if (threadIdx.x == 0) out[0] = 0;
    __syncthreads();
    return;
  }
  DBG_TB(1)
  // blocks of those superblocks (their keys' candidates name them)
  const int nb = block_topb_keys<2>(ns * ESB, B, [&](int i, double& v, long long& k) {
    const long long b = (sbs[1 + i / ESB] / (EB * ESB)) * ESB + (i % ESB);
    v = b < nblk ? w.bval[b] : 0.0;
    k = b < nblk ? w.bidx[b] : -1;
  }, sv, si, blks);
  DBG_TB(2)
  // entries of those blocks
  block_topb_keys<8>(nb * EB, B, [&](int i, double& v, long long& k) {
    const long long y = (blks[1 + i / EB] / EB) * EB + (i % EB);
    const long long yc = y < n ? y : n - 1;  // (both loads issued together, neither behind the other)
    const double cv = cache[yc];
    const bool ok = y < n && !sel[yc];
    v = ok ? cv : 0.0;
    k = ok ? y : -1;
  }, sv, si, out, dt != nullptr ? dt + 3 : nullptr);
  DBG_TB(4)
#undef DBG_TB
}

__global__ __launch_bounds__(256) void exact_steps_reset_kernel(ExactWS w, int nslots, int kmax) {
  const int t = threadIdx.x;
  if (t < CTL_N) w.ctl[t] = t == CTL_STALL ? -1 : 0;
  for (int r = t; r < kmax; r += blockDim.x) w.prec[r].pick = -1;  // no record of this run yet
  for (int i = t; i < nslots; i += blockDim.x) {
    w.rl_cand[i] = -1;
    w.rl_age[i] = 0;
    w.rl_pin[i] = 0;
  }
  if (t < CG_B) {
    w.rf_cand[t] = -1;
    w.rf_slot[t] = -1;
  }
}


constexpr int EX_KMAX = 128;  // picks per run of the exact path (k = 50 in config C4)
constexpr int EX_SLOTS_MAX = 2 * EX_KMAX;  // column slots (exact_slots(kmax) <= this)
constexpr int ROWS_LDS = 8192;  // doubles: packed rows of both factors (each half) up to |A| = 90

// (A/B builds only, -DVGPOSP_EXACT_DBG=1: thread 0 of the per-round kernels stamps its phases with
// the 100 MHz real-time counter; vgposp_exact_dbg copies the last 64 records out.)
#ifndef VGPOSP_EXACT_DBG
#define VGPOSP_EXACT_DBG 0
#endif
#if VGPOSP_EXACT_DBG
__device__ unsigned long long g_exact_dbg[64][8];
__device__ unsigned int g_exact_dbg_n;
#define DBG_DECL unsigned long long dbg_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define DBG_T(k) \
  if (threadIdx.x == 0) dbg_t[k] = __builtin_amdgcn_s_memrealtime();
#define DBG_END(kind)                                                         \
  if (threadIdx.x == 0) {                                                     \
    dbg_t[7] = (kind);                                                        \
    const unsigned slot = atomicAdd(&g_exact_dbg_n, 1u) & 63u;                \
    for (int q = 0; q < 8; ++q) g_exact_dbg[slot][q] = dbg_t[q];              \
  }
#else
#define DBG_DECL
#define DBG_T(k)
#define DBG_END(kind)
#endif
#if VGPOSP_EXACT_DBG == 1
#define DBG_END_STEP() DBG_END(2)
#else
#define DBG_END_STEP()
#endif

// Rows of chol(Q_AA) / chol(S_AA + eps I) as packed lower triangles (row r at r (r + 1) / 2), in
// the workspace (P = const double*) or staged in LDS (P = an address-space-3 pointer, so the
// substitutions' loads are ds_reads: through a generic pointer they were flat loads, which the
// compiler must drain with vmcnt(0) AND lgkmcnt(0) before every use, exposing each row's load
// latency on the chain), with the reciprocals of their diagonals.
typedef const __attribute__((address_space(3))) double* lds_cdptr;

template <class P>
struct FRows {
  P lq;
  P ls;
  P rq;  // 1 / diag
  P rs;
  __device__ __forceinline__ int at(int r, int s) const { return r * (r + 1) / 2 + s; }
};
typedef FRows<const double*> GRows;
typedef FRows<lds_cdptr> LRows;

__device__ __forceinline__ GRows global_rows(const ExactWS& w) {
  return GRows{w.LQ, w.LS, w.RQ, w.RS};
}

// LDS of the staged rows: LQ's packed rows at sm, LS's at sm + ROWS_LDS / 2 (a row appended later
// lands in place; nr (nr + 1) <= ROWS_LDS), the reciprocal diagonals after them.
struct RowsLds {
  double rows[ROWS_LDS];
  double rq[EX_KMAX];
  double rs[EX_KMAX];
};

// Stage rows 0 .. nr-1 of both factors and their reciprocal diagonals: contiguous copies (the
// workspace holds them packed), the whole workgroup.  The caller synchronises before use.
__device__ __forceinline__ LRows stage_rows(const ExactWS& w, int nr, RowsLds& sm) {
  const int np = nr * (nr + 1) / 2;
  for (int e = threadIdx.x; e < np; e += blockDim.x) {
    sm.rows[e] = w.LQ[e];
    sm.rows[ROWS_LDS / 2 + e] = w.LS[e];
  }
  for (int r = threadIdx.x; r < nr; r += blockDim.x) {
    sm.rq[r] = w.RQ[r];
    sm.rs[r] = w.RS[r];
  }
  return LRows{(lds_cdptr)sm.rows, (lds_cdptr)(sm.rows + ROWS_LDS / 2), (lds_cdptr)sm.rq,
               (lds_cdptr)sm.rs};
}

// What a re-score needs of pick r, staged in LDS once per workgroup (the PickRec fields as
// arrays).
struct StagedPicks {
  int g[EX_KMAX][3];
  double x[EX_KMAX][3];
  long long lo[EX_KMAX][3];
  long long base[EX_KMAX];
};

// Picks 0 .. nA-1 (the whole workgroup calls it; the caller synchronises before use).  Picks
// 0 .. nA-2 come from the workspace's pick records when a record matches the round's pick and
// slot; pick nA-1 (this round's), and any record that does not match (a round staged by no
// earlier kernel of this run, e.g. through vgposp_exact_update), is derived from picks / X /
// slot_of_round / boxlo.  Only workgroup 0, and only for pick nA-1, writes a record back: a
// rebuilt older record stays private, so no workgroup can read one while it is written.
__device__ __forceinline__ void stage_picks(const EArgs& a, const ExactWS& w,
                                            const long long* picks, int nA, StagedPicks& sp) {
  const long long bv = w.b0 * w.b1 * w.b2;
  for (int r = threadIdx.x; r < nA; r += blockDim.x) {
    const long long i = picks[r];
    const int slot = w.slot_of_round[r];
    PickRec pr;
    bool ok = false;
    if (r + 1 < nA) {
      pr = w.prec[r];
      ok = pr.pick == (int)i && pr.base == (long long)slot * bv;
    }
    if (!ok) {
      pr.g[0] = (int)(i / (a.I1 * a.I2));
      pr.g[1] = (int)((i / a.I2) % a.I1);
      pr.g[2] = (int)(i % a.I2);
      pr.pick = (int)i;
      pr.x[0] = a.X[3 * i];
      pr.x[1] = a.X[3 * i + 1];
      pr.x[2] = a.X[3 * i + 2];
      pr.lo[0] = w.boxlo[3 * slot];
      pr.lo[1] = w.boxlo[3 * slot + 1];
      pr.lo[2] = w.boxlo[3 * slot + 2];
      pr.base = (long long)slot * bv;
      if (blockIdx.x == 0 && r + 1 == nA) w.prec[r] = pr;
    }
    for (int d = 0; d < 3; ++d) {
      sp.g[r][d] = pr.g[d];
      sp.x[r][d] = pr.x[d];
      sp.lo[r][d] = pr.lo[d];
    }
    sp.base[r] = pr.base;
  }
}

// A candidate (grid coordinates c, point xy) as the re-score sees it.
struct CandPoint {
  long long c0, c1, c2;
  double x0, x1, x2;
};

__device__ __forceinline__ CandPoint cand_point(const EArgs& a, long long y) {
  CandPoint c;
  c.c0 = y / (a.I1 * a.I2);
  c.c1 = (y / a.I2) % a.I1;
  c.c2 = y % a.I2;
  c.x0 = a.X[3 * y];
  c.x1 = a.X[3 * y + 1];
  c.x2 = a.X[3 * y + 2];
  return c;
}

// sigma_off(a, pick r, y) from the staged pick: the same operations in the same order, so the
// same bits.
template <int KIND>
__device__ __forceinline__ double sigma_off_staged(const EArgs& a, const StagedPicks& sp, int r,
                                                   const CandPoint& c) {
  const long long e0 = sp.g[r][0] - c.c0, e1 = sp.g[r][1] - c.c1, e2 = sp.g[r][2] - c.c2;
  const long long d2i = e0 * e0 + e1 * e1 + e2 * e2;
  if (d2i >= a.ntau) return 0.0;
  const double t = a.tau[d2i];
  if (t == 0.0) return 0.0;
  const double d0 = sp.x[r][0] - c.x0, d1 = sp.x[r][1] - c.x1, d2 = sp.x[r][2] - c.x2;
  return t * kfun<KIND>(d0 * d0 + d1 * d1 + d2 * d2, a.tla, a.inv_ls, a.inv_ls2);
}

// qcol_at(w, r, y) from the staged pick.
__device__ __forceinline__ double qcol_staged(const ExactWS& w, const StagedPicks& sp, int r,
                                              const CandPoint& c) {
  const long long l0 = c.c0 - sp.lo[r][0], l1 = c.c1 - sp.lo[r][1], l2 = c.c2 - sp.lo[r][2];
  if (l0 < 0 || l0 >= w.b0 || l1 < 0 || l1 >= w.b1 || l2 < 0 || l2 >= w.b2) return 0.0;
  return w.Qcols[sp.base[r] + (l0 * w.b1 + l1) * w.b2 + l2];
}

// The right-hand sides of a re-score: lane s holds s_{a_s y} and q_{a_s y} (and s + 64's).
// sp: the picks staged in LDS (stage_picks) or nullptr (read from the workspace).
struct RescoreVals {
  double vs0, vq0, vs1, vq1;
};

template <int KIND>
__device__ __forceinline__ RescoreVals wave_rescore_vals(const EArgs& a, const ExactWS& w,
                                                         const long long* picks, int nA,
                                                         long long y, const StagedPicks* sp) {
  const int lane = threadIdx.x & 63;
  double vs0 = 0.0, vq0 = 0.0, vs1 = 0.0, vq1 = 0.0;
  if (sp) {
    const CandPoint c = cand_point(a, y);
    if (lane < nA) {
      vs0 = sigma_off_staged<KIND>(a, *sp, lane, c);
      vq0 = qcol_staged(w, *sp, lane, c);
    }
    if (lane + 64 < nA) {
      vs1 = sigma_off_staged<KIND>(a, *sp, lane + 64, c);
      vq1 = qcol_staged(w, *sp, lane + 64, c);
    }
  } else {
    if (lane < nA) {
      vs0 = sigma_off<KIND>(a, picks[lane], y);
      vq0 = qcol_at(w, lane, y, a.I1, a.I2);
    }
    if (lane + 64 < nA) {
      vs1 = sigma_off<KIND>(a, picks[lane + 64], y);
      vq1 = qcol_at(w, lane + 64, y, a.I1, a.I2);
    }
  }
  return RescoreVals{vs0, vq0, vs1, vq1};
}

// The forward substitutions of a re-score, z = L^-1 v for both factors at once, column by column:
// lane s holds the running right-hand sides b_s (and b_{s+64}); at row r the unknown
// z_r = b_r / L_rr (times the staged reciprocal) is ONE wave-uniform value read from lane r, added
// into the running sums of squares in row order, kept on lane r, and removed from the rows below
// (b_s -= L_sr z_r on lanes r < s < rlim).  The chain per row is a lane read, a multiply and an
// FMA, where the row-oriented form (a wave sum per row) took two butterflies and a division.
struct Subst {
  double bs0, bq0, bs1, bq1;  // right-hand sides, then (lane r < done) z_r
  double ns, nq;              // sum of z_r^2 over the rows done, in row order
};

__device__ __forceinline__ Subst subst_begin(const RescoreVals& v) {
  return Subst{v.vs0, v.vq0, v.vs1, v.vq1, 0.0, 0.0};
}

// Rows [r0, r1), updating the right-hand sides of rows < rlim only.  Branch-free: every lane
// computes its update and selects (the same values the predicated form stores).  Column r + 1's
// factor entries are loaded while row r is eliminated, unconditionally
// (the last iteration re-reads column r1 - 1) so the count of loads in flight is static and the
// compiler can wait for the older ones only; a lane at or beyond rlim reads row rlim - 1's entry
// (in bounds, unused).
template <class R>
__device__ __forceinline__ void subst_rows(const R& L, int r0, int r1, int rlim, Subst& st) {
  if (r0 >= r1 || rlim <= 0) return;
  const int lane = threadIdx.x & 63;
  const int l0 = min(lane, rlim - 1), l1 = min(lane + 64, rlim - 1);
  double cs0 = L.ls[L.at(l0, r0)], cq0 = L.lq[L.at(l0, r0)];
  double cs1 = L.ls[L.at(l1, r0)], cq1 = L.lq[L.at(l1, r0)];
  // each lane's own rows' reciprocal diagonals, in registers: lane r forms z_r = b_r / L_rr
  // itself (the same multiply), so the chain reads no LDS for it
  const double rs0 = L.rs[l0], rq0 = L.rq[l0], rs1 = L.rs[l1], rq1 = L.rq[l1];
  for (int r = r0; r < r1; ++r) {
    const int rn = min(r + 1, r1 - 1);
    const double ns0 = L.ls[L.at(l0, rn)], nq0 = L.lq[L.at(l0, rn)];
    const double ns1 = L.ls[L.at(l1, rn)], nq1 = L.lq[L.at(l1, rn)];
    const double zs = wave_bcast(r < 64 ? st.bs0 * rs0 : st.bs1 * rs1, r & 63);
    const double zq = wave_bcast(r < 64 ? st.bq0 * rq0 : st.bq1 * rq1, r & 63);
    st.ns = fma(zs, zs, st.ns);
    st.nq = fma(zq, zq, st.nq);
    const bool own0 = lane == r, own1 = lane + 64 == r;
    const bool up0 = lane > r && lane < rlim, up1 = lane + 64 > r && lane + 64 < rlim;
    const double us0 = fma(-cs0, zs, st.bs0), uq0 = fma(-cq0, zq, st.bq0);
    const double us1 = fma(-cs1, zs, st.bs1), uq1 = fma(-cq1, zq, st.bq1);
    st.bs0 = own0 ? zs : (up0 ? us0 : st.bs0);
    st.bq0 = own0 ? zq : (up0 ? uq0 : st.bq0);
    st.bs1 = own1 ? zs : (up1 ? us1 : st.bs1);
    st.bq1 = own1 ? zq : (up1 ? uq1 : st.bq1);
    cs0 = ns0;
    cq0 = nq0;
    cs1 = ns1;
    cq1 = nq1;
  }
}

// The last row R of the system, once rows 0 .. R-1 are done with rlim = R: its right-hand side
// minus the dot product of row R with the z held on lanes 0 .. R-1 (one wave sum per factor).
template <class RT>
__device__ __forceinline__ void subst_last(const RT& L, int R, Subst& st) {
  const int lane = threadIdx.x & 63;
  double ds = 0.0, dq = 0.0;
  if (lane < R) {
    ds = L.ls[L.at(R, lane)] * st.bs0;
    dq = L.lq[L.at(R, lane)] * st.bq0;
  }
  if (lane + 64 < R) {
    ds = fma(L.ls[L.at(R, lane + 64)], st.bs1, ds);
    dq = fma(L.lq[L.at(R, lane + 64)], st.bq1, dq);
  }
  ds = wave_sum(ds);
  dq = wave_sum(dq);
  const double vs = wave_bcast(R < 64 ? st.bs0 : st.bs1, R & 63);
  const double vq = wave_bcast(R < 64 ? st.bq0 : st.bq1, R & 63);
  const double zs = (vs - ds) * L.rs[R], zq = (vq - dq) * L.rq[R];
  st.ns = fma(zs, zs, st.ns);
  st.nq = fma(zq, zq, st.nq);
}

// The whole system of nA rows, the one arithmetic every re-score uses (the window kernel runs the
// same two parts on either side of its barrier): rows 0 .. nA-2 column by column, row nA-1 by its
// dot product.
template <class R>
__device__ __forceinline__ void subst_all(const R& L, int nA, Subst& st) {
  if (nA <= 0) return;
  subst_rows(L, 0, nA - 1, nA - 1, st);
  subst_last(L, nA - 1, st);
}

template <int KIND>
__device__ __forceinline__ double rescore_delta(const EArgs& a, double qyy, bool exact,
                                                const Subst& st) {
  return delta_from(sigma_diag<KIND>(a) - st.ns, qyy - st.nq, exact, a.jitter, a.thr);
}

template <int KIND, class R>
__device__ double wave_rescore(const EArgs& a, const ExactWS& w, const R& L,
                               const long long* picks, int nA, long long y, double qyy,
                               bool exact, const StagedPicks* sp = nullptr) {
  Subst st = subst_begin(wave_rescore_vals<KIND>(a, w, picks, nA, y, sp));
  subst_all(L, nA, st);
  return rescore_delta<KIND>(a, qyy, exact, st);
}

// Bounded-lazy path, after the CG columns of the batch (cands[j] in slots[j], j < nb): each Q_cc
// is now known; the candidate's cache entry becomes the reference's value (scored with the A of
// its last re-score) and its keys are refreshed.  One workgroup: the candidates are re-scored one
// wave each, then the block keys of their blocks (two candidates may share one: both waves write
// the same key from the same cache) and after a barrier the superblock keys.
template <int KIND>
__global__ __launch_bounds__(SEL_THREADS) void exact_refine_end_kernel(EArgs a, double* qdiag,
                                                                       double* cache,
                                                                       unsigned char* sel,
                                                                       ExactWS w, long long nblk,
                                                                       int nb, const int* slots,
                                                                       const long long* cands,
                                                                       const long long* picks,
                                                                       int resume) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NWAVE = SEL_THREADS / 64;
  for (int j = wave; j < nb; j += NWAVE) {
    const long long c = cands[j];
    if (c < 0) continue;
    const double qcc = qslot_at(w, slots[j], c, a.I1, a.I2);
    const double d = wave_rescore<KIND>(a, w, global_rows(w), picks, (int)w.lastA[c], c, qcc, true);
    if (lane == 0) {
      qdiag[c] = qcc;
      w.qexact[c] = 1;
      cache[c] = d;
    }
  }
  __syncthreads();
  for (int j = wave; j < nb; j += NWAVE)
    if (cands[j] >= 0) wave_block_key(cache, sel, a.n, cands[j] / EB, w.bval, w.bidx);
  __syncthreads();
  for (int j = wave; j < nb; j += NWAVE)
    if (cands[j] >= 0) wave_super_key(w.bval, w.bidx, nblk, cands[j] / EB / ESB, w.sval, w.sidx);
  if (resume && threadIdx.x == 0) {  // device-side rounds: the stalled round may go on
    int done = 0;
    for (int j = 0; j < nb; ++j) done += cands[j] >= 0;
    w.ctl[CTL_UNPICKED] += done;
    w.ctl[CTL_REFINED] += done;
    w.ctl[CTL_EVENTS] += 1;
    w.ctl[CTL_STALL] = -1;
  }
}

// After the tightening bounds of a refinement event (the K_hi-step bounds of rt_cand): each
// candidate's cache entry is re-scored from its tighter upper bound with the A of its last re-score,
// its keys refreshed; the stall is cleared unless CG columns are pending too (their
// exact_refine_end_kernel clears it).  One workgroup.
template <int KIND>
__global__ __launch_bounds__(SEL_THREADS) void exact_tighten_end_kernel(EArgs a, const double* qdiag,
                                                                        double* cache,
                                                                        unsigned char* sel,
                                                                        ExactWS w, long long nblk,
                                                                        const long long* picks) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NWAVE = SEL_THREADS / 64;
  const int nt = w.ctl[CTL_NT];
  for (int j = wave; j < nt; j += NWAVE) {
    const long long c = w.rt_cand[j];
    const double d = wave_rescore<KIND>(a, w, global_rows(w), picks, (int)w.lastA[c], c, qdiag[c],
                                        false);
    if (lane == 0) {
      w.qexact[c] = 2;
      cache[c] = d;
    }
  }
  __syncthreads();
  for (int j = wave; j < nt; j += NWAVE)
    wave_block_key(cache, sel, a.n, w.rt_cand[j] / EB, w.bval, w.bidx);
  __syncthreads();
  for (int j = wave; j < nt; j += NWAVE)
    wave_super_key(w.bval, w.bidx, nblk, w.rt_cand[j] / EB / ESB, w.sval, w.sidx);
  __syncthreads();
  if (threadIdx.x == 0) {
    w.ctl[CTL_TIGHT] += nt;
    w.ctl[CTL_NT] = 0;
    if (w.ctl[CTL_NB] == 0) w.ctl[CTL_STALL] = -1;
  }
}

// After q_t = Q e_{a_t}: row t of LQ = chol(Q_AA) (wave 0) and of LS = chol(S_AA + eps I)
// (wave 1) from the staged picks and rows 0 .. round - 1 in L, column-oriented like the re-scores
// (subst_rows; lane r ends with z_r): written to the workspace with the diagonal's reciprocal and,
// with lds (the staged rows of this workgroup), appended there too.
template <int KIND, class R>
__device__ void wave_new_row(const EArgs& a, const ExactWS& w, int round, const R& L,
                             const StagedPicks& sp, RowsLds* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // (the staged forms of qcol_at(w, round, picks[r]) and sigma_off(a, at, picks[r]))
  auto val = [&](int r) {
    const CandPoint c{sp.g[r][0], sp.g[r][1], sp.g[r][2], sp.x[r][0], sp.x[r][1], sp.x[r][2]};
    if (wave == 0) return qcol_staged(w, sp, round, c);
    return r == round ? sigma_diag<KIND>(a) + a.jitter : sigma_off_staged<KIND>(a, sp, round, c);
  };
  const double v0 = lane <= round ? val(lane) : 0.0;
  const double v1 = lane + 64 <= round ? val(lane + 64) : 0.0;
  // both factors' rows through one Subst (the unused half mirrors the used one; the two waves
  // differ only in which half they keep)
  Subst st{v0, v0, v1, v1, 0.0, 0.0};
  const R Lw{wave == 0 ? L.lq : L.ls, wave == 0 ? L.lq : L.ls, wave == 0 ? L.rq : L.rs,
                      wave == 0 ? L.rq : L.rs};
  subst_rows(Lw, 0, round, round, st);
  const double vr = wave_bcast(round < 64 ? v0 : v1, round & 63);
  const double dg = sqrt(vr - st.ns);
  const double rdg = 1.0 / dg;
  const int off = round * (round + 1) / 2;
  double* Lg = (wave == 0 ? w.LQ : w.LS) + off;
  if (lane < round) Lg[lane] = st.bs0;
  if (lane + 64 < round) Lg[lane + 64] = st.bs1;
  if (lane == 0) {
    Lg[round] = dg;
    (wave == 0 ? w.RQ : w.RS)[round] = rdg;
  }
  if (lds) {
    __attribute__((address_space(3))) double* Ll =
        (__attribute__((address_space(3))) double*)(lds->rows + (wave == 0 ? 0 : ROWS_LDS / 2) + off);
    if (lane < round) Ll[lane] = st.bs0;
    if (lane + 64 < round) Ll[lane + 64] = st.bs1;
    if (lane == 0) {
      Ll[round] = dg;
      ((__attribute__((address_space(3))) double*)(wave == 0 ? lds->rq : lds->rs))[round] = rdg;
    }
  }
}

template <int KIND>
__device__ void block_factor_rows(const EArgs& a, const ExactWS& w, int round,
                                  const long long* picks, RowsLds& sm) {
  const int wave = threadIdx.x >> 6;
  const long long at = picks[round];
  if (at < 0) return;
  __shared__ StagedPicks sp;
  stage_picks(a, w, picks, round + 1, sp);
  if (round * (round + 1) <= ROWS_LDS) {
    const LRows L = stage_rows(w, round, sm);
    __syncthreads();
    if (wave > 1) return;
    wave_new_row<KIND>(a, w, round, L, sp, nullptr);
  } else {
    __syncthreads();
    if (wave > 1) return;
    wave_new_row<KIND>(a, w, round, global_rows(w), sp, nullptr);
  }
}


template <int KIND>
__global__ __launch_bounds__(128) void exact_rows_kernel(EArgs a, ExactWS w, int round,
                                                         const long long* picks) {
  __shared__ RowsLds sm;
  block_factor_rows<KIND>(a, w, round, picks, sm);
}

struct Window {
  long long lo0, lo1, lo2, w0, w1, w2;
};

__device__ __forceinline__ Window window_of(const EArgs& a, long long at) {
  Window v;
  const long long ci0 = at / (a.I1 * a.I2), ci1 = (at / a.I2) % a.I1, ci2 = at % a.I2;
  v.lo0 = max(ci0 - a.cutoff, 0LL);
  v.lo1 = max(ci1 - a.cutoff, 0LL);
  v.lo2 = max(ci2 - a.cutoff, 0LL);
  v.w0 = max(min(ci0 + a.cutoff, a.I0) - v.lo0, 0LL);
  v.w1 = max(min(ci1 + a.cutoff, a.I1) - v.lo1, 0LL);
  v.w2 = max(min(ci2 + a.cutoff, a.I2) - v.lo2, 0LL);
  return v;
}

// Part 2: re-score the window of a_t (snippets_a3.py:190-303; candidates in A -> 0), one wave per
// candidate; upper bounds where Q_yy is still only bounded.  2 + WIN_CAND waves: 0 and 1 compute the pick's
// own rows (row `round` of LQ and LS: every workgroup, the same values, so the same bits written to
// the workspace), the others one window candidate each — their right-hand sides and the substitution
// of rows 0 .. round-1 run WHILE the new rows are computed; after one barrier the last row.
constexpr int WIN_CAND = 2;  // window candidates per workgroup (1 / 3 / 4 / 6 / 14: DESIGN.md §4a)
constexpr int WIN_T = 64 * (2 + WIN_CAND);      // threads per workgroup

// The window kernel after its staging barrier: waves 0 and 1 the pick's new rows, the others one
// window candidate each (R: the rows in LDS or in the workspace).
template <int KIND, class R>
__device__ __forceinline__ void window_tail(const EArgs& a, const double* __restrict__ qdiag,
                                            double* cache, const unsigned char* sel,
                                            const ExactWS& w, int round, const long long* picks,
                                            const Window& v, const StagedPicks& sp, const R& L,
                                            RowsLds* lds) {
  DBG_DECL
  const int nr = round + 1;
  const int wave = threadIdx.x >> 6;
  DBG_T(0)
  DBG_T(1)
  if (wave < 2) {
    wave_new_row<KIND>(a, w, round, L, sp, lds);
    DBG_T(2)
    DBG_T(3)
    __syncthreads();
    DBG_T(4)
    DBG_T(5)
    if (blockIdx.x == 0) {
      DBG_END(3)
    }
    return;
  }
  const long long e = (long long)blockIdx.x * WIN_CAND + (wave - 2);
  const bool live = e < v.w0 * v.w1 * v.w2;
  const long long y = live ? ((v.lo0 + e / (v.w1 * v.w2)) * a.I1 + v.lo1 + (e / v.w2) % v.w1) *
                                     a.I2 + v.lo2 + e % v.w2
                           : 0;
  const bool picked = live && sel[y];
  Subst st{0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  double qyy = 0.0;
  bool ex = false;
  if (live && !picked) {
    st = subst_begin(wave_rescore_vals<KIND>(a, w, picks, nr, y, &sp));
    qyy = qdiag[y];
    ex = w.qexact[y] == 1;
    subst_rows(L, 0, round, round, st);  // rows of picks 0 .. round-1 (subst_all's first part)
  }
  __syncthreads();  // the new rows are in place
  if (!live) return;
  if (picked) {
    if ((threadIdx.x & 63) == 0) cache[y] = 0.0;
    return;
  }
  subst_last(L, round, st);
  const double d = rescore_delta<KIND>(a, qyy, ex, st);
  if ((threadIdx.x & 63) == 0) {
    cache[y] = d;
    w.lastA[y] = (unsigned char)(round + 1);
  }
}


// Part 3: refresh the block keys of the window rows (each (j0, j1) row is one contiguous i2 run),
// then their superblock keys.  The whole workgroup calls it (at >= 0: the window's centre).
__device__ void block_window_keys_rows(const EArgs& a, const double* cache,
                                       const unsigned char* sel, const ExactWS& w, long long nblk,
                                       const Window& v) {
  const int wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  const long long nrow = v.w0 * v.w1;
  for (long long rr = wave; rr < nrow; rr += nwave) {
    const long long y0 = ((v.lo0 + rr / v.w1) * a.I1 + v.lo1 + rr % v.w1) * a.I2 + v.lo2;
    const long long y1 = y0 + v.w2 - 1;
    for (long long b = y0 / EB; b <= y1 / EB; ++b) wave_block_key(cache, sel, a.n, b, w.bval, w.bidx);
  }
  __syncthreads();
  for (long long rr = wave; rr < nrow; rr += nwave) {
    const long long y0 = ((v.lo0 + rr / v.w1) * a.I1 + v.lo1 + rr % v.w1) * a.I2 + v.lo2;
    const long long y1 = y0 + v.w2 - 1;
    for (long long sb = y0 / EB / ESB; sb <= y1 / EB / ESB; ++sb)
      wave_super_key(w.bval, w.bidx, nblk, sb, w.sval, w.sidx);
  }
  __syncthreads();
}

// Inclusive prefix sum over the wave (lane order).
__device__ __forceinline__ int wave_incl_scan(int x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  return x;
}

constexpr int WK_LIST = 128;  // distinct blocks / superblocks of a window handled by the list form

// Part 3: refresh the block keys of the window rows (each (j0, j1) row is one contiguous i2 run),
// then their superblock keys.  The whole workgroup calls it (at >= 0: the window's centre).  Rows
// are increasing in y, so the blocks they touch form a sorted list with duplicates only between
// neighbouring rows: wave 0 builds the DISTINCT blocks and superblocks (one row per lane, an
// exclusive scan of the counts), then every block key is computed once — all of a wave's blocks'
// entries loaded before any key is reduced — and every superblock key once.  (Row by row, a block
// shared by two rows and a superblock shared by up to 36 were recomputed, each wave walking its
// rows with one dependent load / reduce / store chain per block: 17 us per round at 128^3.)
__device__ void block_window_keys(const EArgs& a, const double* cache, const unsigned char* sel,
                                  const ExactWS& w, long long nblk, long long at) {
  __shared__ long long s_blk[WK_LIST], s_sb[WK_LIST];
  __shared__ int s_nb, s_ns;
  const Window v = window_of(a, at);
  const long long nrow = v.w0 * v.w1;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwave = blockDim.x >> 6;
  if (nrow > 64 || v.w2 > EB) {
    block_window_keys_rows(a, cache, sel, w, nblk, v);
    return;
  }
  if (wave == 0) {
    long long blo = 0, bhi = -1;
    if (lane < nrow && v.w2 > 0) {
      const long long y0 = ((v.lo0 + lane / v.w1) * a.I1 + v.lo1 + lane % v.w1) * a.I2 + v.lo2;
      blo = y0 / EB;
      bhi = (y0 + v.w2 - 1) / EB;
    }
    // the last block of the rows before (rows increase, so it is the previous lane's)
    long long prev = __shfl_up(bhi, 1, 64);
    if (lane == 0) prev = -1;
    const long long own = max(blo, prev + 1);
    const int nbl = bhi >= own ? (int)(bhi - own + 1) : 0;
    const long long prev_sb = prev >= 0 ? prev / ESB : -1;
    const long long sb0 = max(own / ESB, prev_sb + 1);
    const int nsb_l = nbl > 0 && bhi / ESB >= sb0 ? (int)(bhi / ESB - sb0 + 1) : 0;
    const int ib = wave_incl_scan(nbl), is = wave_incl_scan(nsb_l);
    for (int q = 0; q < nbl; ++q)
      if (ib - nbl + q < WK_LIST) s_blk[ib - nbl + q] = own + q;
    for (int q = 0; q < nsb_l; ++q)
      if (is - nsb_l + q < WK_LIST) s_sb[is - nsb_l + q] = sb0 + q;
    if (lane == 63) {
      s_nb = ib;
      s_ns = is;
    }
  }
  __syncthreads();
  const int nb = s_nb, ns = s_ns;
  if (nb > 4 * nwave || ns > WK_LIST) {  // (a window of more blocks than the fast form holds)
    __syncthreads();
    block_window_keys_rows(a, cache, sel, w, nblk, v);
    return;
  }
  // blocks wave, wave + nwave, ...: at most 4 per wave
  {
    long long mine[4];
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = wave + q * nwave;
      mine[q] = j < nb ? s_blk[j] : 0;
      cnt += j < nb;
    }
    if (cnt > 0) wave_block_keys<4>(cache, sel, a.n, mine, cnt, w.bval, w.bidx);
  }
  __syncthreads();
  for (int j = wave; j < ns; j += nwave) wave_super_key(w.bval, w.bidx, nblk, s_sb[j], w.sval, w.sidx);
  __syncthreads();
}

__global__ __launch_bounds__(SEL_THREADS) void exact_window_keys_kernel(EArgs a, const double* cache,
                                                                        const unsigned char* sel,
                                                                        ExactWS w, long long nblk,
                                                                        int round,
                                                                        const long long* picks) {
  const long long at = picks[round];
  if (at < 0) return;
  const Window v = window_of(a, at);
  const int wave = threadIdx.x >> 6;
  const long long nrow = v.w0 * v.w1;
  for (long long rr = wave; rr < nrow; rr += SEL_THREADS / 64) {
    const long long y0 = ((v.lo0 + rr / v.w1) * a.I1 + v.lo1 + rr % v.w1) * a.I2 + v.lo2;
    const long long y1 = y0 + v.w2 - 1;
    for (long long b = y0 / EB; b <= y1 / EB; ++b) wave_block_key(cache, sel, a.n, b, w.bval, w.bidx);
  }
  __syncthreads();
  for (long long rr = wave; rr < nrow; rr += SEL_THREADS / 64) {
    const long long y0 = ((v.lo0 + rr / v.w1) * a.I1 + v.lo1 + rr % v.w1) * a.I2 + v.lo2;
    const long long y1 = y0 + v.w2 - 1;
    for (long long sb = y0 / EB / ESB; sb <= y1 / EB / ESB; ++sb)
      wave_super_key(w.bval, w.bidx, nblk, sb, w.sval, w.sidx);
  }
}

// The keys of the blocks a round changed — the window of the previous pick, which contains the
// pick itself (cutoff >= 1; its block is added explicitly otherwise) — recomputed with every
// global read issued up front: the superblock keys of the whole grid (for the arg-max) and the
// block keys of every superblock the window touches (for its superblock keys) are loaded into LDS
// while the window's cache entries are; the new block keys, superblock keys and the arg-max are
// then computed from LDS.  Returns false (nothing done) when the window exceeds the LDS lists;
// the caller then takes the global-memory path (block_window_keys + block_argmax).
constexpr int SK_MAXSB = 16;   // touched superblocks held in LDS
constexpr int SK_MAXNSB = 4096;  // superblocks of the grid held in LDS (n <= 2^28)

struct StepLds {
  double sval[SK_MAXNSB];
  long long sidx[SK_MAXNSB];
  double bval[SK_MAXSB][ESB];
  long long bidx[SK_MAXSB][ESB];
  long long blk[64];
  int bslot[64];  // the superblock slot (index into sb) of each listed block
  long long sb[SK_MAXSB];
  int nb, ns, ok;
};

__device__ bool block_window_keys_lds(const EArgs& a, const double* cache,
                                      const unsigned char* sel, const ExactWS& w, long long nblk,
                                      long long nsb, long long at, StepLds& L,
                                      unsigned long long* dt = nullptr) {
  // (dt: debug builds with VGPOSP_EXACT_DBG=2 stamp the phases here)
#define DBG_PT(k) \
  if (dt != nullptr && threadIdx.x == 0) dt[k] = __builtin_amdgcn_s_memrealtime();
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, nwave = blockDim.x >> 6;
  if (nsb > SK_MAXNSB) return false;
  // level 1: the distinct blocks / superblocks of the window (wave 0, ALU and LDS only); the
  // grid's superblock keys after it (their loads would stall wave 0's list behind them)
  if (wave == 0) {
    const Window v = window_of(a, at);
    const long long nrow = v.w0 * v.w1;
    const long long ab = at / EB;
    const bool fits = nrow <= 63 && v.w2 <= EB;
    long long blo = 0, bhi = -1;
    if (fits && lane < nrow && v.w2 > 0) {
      const long long y0 = ((v.lo0 + lane / v.w1) * a.I1 + v.lo1 + lane % v.w1) * a.I2 + v.lo2;
      blo = y0 / EB;
      bhi = (y0 + v.w2 - 1) / EB;
    }
    // the pick's own block, on lane 63 (the whole list when the window is empty: cutoff 0),
    // unless a row already covers it
    const bool covered = __ballot(lane < 63 && bhi >= 0 && ab >= blo && ab <= bhi) != 0;
    if (fits && lane == 63) {
      blo = ab;
      bhi = covered ? ab - 1 : ab;
    }
    // distinct blocks: rows increase with the lane, so duplicates sit between neighbours
    long long prev = __shfl_up(bhi, 1, 64);
    if (lane == 0) prev = -1;
    const long long own = lane == 63 ? blo : max(blo, prev + 1);
    const int nbl = bhi >= own ? (int)(bhi - own + 1) : 0;
    const int ib = wave_incl_scan(nbl);
    const int nbt = __builtin_amdgcn_readlane(ib, 63);
    const bool ok = fits && nbt >= 1 && nbt <= 64 && nbt <= 4 * nwave;
    if (ok)
      for (int q = 0; q < nbl; ++q) L.blk[ib - nbl + q] = own + q;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the distinct superblocks, lane q for listed block q: the list is increasing except its last
    // entry when that is the pick's block (not covered by a row), which joins an earlier entry's
    // superblock if one shares it
    int ns = 0;
    if (ok) {
      const long long bq = lane < nbt ? L.blk[lane] : -1;
      const long long sq = bq >= 0 ? bq / ESB : -1;
      long long sp = __shfl_up(sq, 1, 64);
      const bool pick_last = !covered;
      const long long spk = __shfl(sq, nbt - 1, 64);
      const unsigned long long same = __ballot(lane < nbt - 1 && sq == spk);
      bool isnew = lane < nbt && (lane == 0 || sp != sq);
      if (pick_last && lane == nbt - 1) isnew = same == 0;
      const int in = wave_incl_scan(isnew ? 1 : 0);
      ns = __builtin_amdgcn_readlane(in, 63);
      int slot = in - 1;
      if (pick_last && same != 0) {
        const int f = __builtin_ctzll(same);  // the first earlier entry in the pick's superblock
        const int fs = __shfl(in, f, 64) - 1;
        if (lane == nbt - 1) slot = fs;
      }
      if (isnew && in - 1 < SK_MAXSB) L.sb[in - 1] = sq;
      if (lane < nbt) L.bslot[lane] = slot;
    }
    if (lane == 0) {
      L.nb = nbt;
      L.ns = ns;
      L.ok = ok && ns <= SK_MAXSB;
    }
  }
  for (long long q = t; q < nsb; q += blockDim.x) {
    L.sval[q] = w.sval[q];
    L.sidx[q] = w.sidx[q];
  }
  __syncthreads();
  DBG_PT(1)
  if (!L.ok) return false;
  const int nb = L.nb, ns = L.ns;
  // level 2: the window blocks' entries (registers) — issued first, so that their round trip
  // overlaps the one of the touched superblocks' block keys, which go through LDS (the stores wait
  // on their loads)
  constexpr int PER = EB / 64;
  double c[4][PER];
  unsigned char sl[4][PER];
  long long mine[4];
  int mslot[4];
  int cnt = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = wave + q * nwave;
    mine[q] = j < nb ? L.blk[j] : -1;
    mslot[q] = j < nb ? L.bslot[j] : 0;
    cnt += j < nb;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const long long y = mine[q] >= 0 ? mine[q] * EB + e * 64 + lane : a.n;
      const long long yc = y < a.n ? y : a.n - 1;  // (unconditional loads, masked values)
      const double cv = cache[yc];
      const unsigned char sv = sel[yc];
      c[q][e] = y < a.n ? cv : 0.0;
      sl[q][e] = y < a.n ? sv : 1;
    }
  }
  for (int e = t; e < ns * ESB; e += blockDim.x) {
    const int q = e / ESB, j = e % ESB;
    const long long b = L.sb[q] * ESB + j;
    L.bval[q][j] = b < nblk ? w.bval[b] : 0.0;
    L.bidx[q][j] = b < nblk ? w.bidx[b] : -1;
  }
  __syncthreads();  // the LDS block keys are in place before the new ones overwrite them
  DBG_PT(2)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q >= cnt) break;
    Key k{0ull, 0ull};
#pragma unroll
    for (int e = 0; e < PER; ++e)
      key_take_max(k, key_enc(c[q][e], sl[q][e] ? -1 : mine[q] * EB + e * 64 + lane));
    k = wave_keymax(k);
    if (lane == 0) {
      const double kv = key_value(k);
      const long long ki = key_index(k);
      w.bval[mine[q]] = kv;
      w.bidx[mine[q]] = ki;
      L.bval[mslot[q]][mine[q] % ESB] = kv;
      L.bidx[mslot[q]][mine[q] % ESB] = ki;
    }
  }
  __syncthreads();
  DBG_PT(3)
  for (int q = wave; q < ns; q += nwave) {
    double v = L.bval[q][lane];
    long long idx = L.bidx[q][lane];
    wave_keymax(v, idx);
    if (lane == 0) {
      w.sval[L.sb[q]] = v;
      w.sidx[L.sb[q]] = idx;
      L.sval[L.sb[q]] = v;
      L.sidx[L.sb[q]] = idx;
    }
  }
  __syncthreads();
  DBG_PT(4)
#undef DBG_PT
  return true;
}

// Workgroup-wide arg-max over the superblock keys staged in LDS (block_argmax's reduction).
__device__ long long block_argmax_lds(const StepLds& L, long long nsb) {
  __shared__ double sv[SEL_THREADS / 64];
  __shared__ long long si[SEL_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double v = 0.0;
  long long idx = -1;
  for (long long s = t; s < nsb; s += SEL_THREADS) {
    if (L.sidx[s] >= 0 && key_gt(L.sval[s], L.sidx[s], v, idx)) {
      v = L.sval[s];
      idx = L.sidx[s];
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
    if (lane == 0) si[0] = idx;
  }
  __syncthreads();
  const long long r = si[0];
  __syncthreads();
  return r;
}

// One round of the bounded-lazy rounds, decided on the device (vgposp_exact_steps).  First the
// keys of the blocks the previous round changed (its pick and its window's re-scored entries),
// then the arg-max of the cache; if its Q_yy is exact (a refined candidate, its CG column in a
// slot) it is picked (marked selected, its cache entry 0; its keys are refreshed by the next
// round's kernel, the first reader — its window contains it) and, with `rows`, the pick's rows
// of chol(Q_AA) and chol(S_AA + eps I) are appended; otherwise the round STALLS: ctl[STALL] =
// round, and the B best cache entries that have no column yet become the pending refinement batch
// (rf_cand / rf_slot, ctl[NB]), each given a free slot or the oldest unpinned one — the host
// loop's rule (sparse_placement.ExactWindowGreedy.run_bounded, round 3).  Every later kernel of
// the issued rounds sees the stall (picks[round] stays -1, ctl[STALL] >= 0) and does nothing,
// until the host has run the refinement (exact_refine_end_kernel clears the stall) and re-issues
// the rounds from the stalled one.  One workgroup; a round is this kernel plus the window
// re-score (exact_window_kernel).  A stalled round refreshed the keys of round - 1's pick first,
// so the stall / refinement kernels that run next see current keys.
union StepSm {
  StepLds k;
  RowsLds r;
};

// The step of `round` by one workgroup of SEL_THREADS threads (exact_step_kernel, or the last
// workgroup of the previous round's window kernel).
template <int KIND>
__device__ __forceinline__ void step_body(const EArgs& ea, double* cache, unsigned char* sel,
                                          const ExactWS& w, long long nblk, long long nsb,
                                          int nslots, int round, int rows, long long* picks,
                                          double* pick_delta, StepSm& sm, int& s_slot) {
  DBG_DECL
  DBG_T(0)
  if (w.ctl[CTL_STALL] >= 0) return;  // an earlier round is waiting for a refinement
  const long long n = ea.n;
  long long a;
  const long long prev = round > 0 ? picks[round - 1] : -1;
#if VGPOSP_EXACT_DBG == 2
  unsigned long long* dtp = dbg_t;
#else
  unsigned long long* dtp = nullptr;
#endif
  if (prev >= 0 && block_window_keys_lds(ea, cache, sel, w, nblk, nsb, prev, sm.k, dtp)) {
#if VGPOSP_EXACT_DBG != 2
    DBG_T(1)
#endif
    a = block_argmax_lds(sm.k, nsb);
#if VGPOSP_EXACT_DBG == 2
    DBG_T(5)
    DBG_END(2)
    (void)0;
#endif
  } else {
    if (prev >= 0) {  // (a window too large for the LDS lists; the pick's own block as well)
      block_window_keys(ea, cache, sel, w, nblk, prev);
      if (threadIdx.x < 64) wave_refresh_keys(cache, sel, w, n, nblk, prev);
      __syncthreads();
    }
    DBG_T(1)
    a = block_argmax(w, nsb);
  }
  DBG_T(2)
  if (threadIdx.x == 0) s_slot = -1;
  __syncthreads();
  if (a >= 0)
    for (int i = threadIdx.x; i < nslots; i += SEL_THREADS)
      if (w.rl_cand[i] == a) s_slot = i;
  __syncthreads();
  DBG_T(3)
  const int slot = s_slot;
  if (a < 0 || slot >= 0) {  // pick (no candidate left: picks[round] = -1, nothing changes)
    if (threadIdx.x == 0) {
      picks[round] = a;
      if (pick_delta) pick_delta[round] = a >= 0 ? cache[a] : 0.0;
      if (a >= 0) {
        w.slot_of_round[round] = slot;
        w.rl_pin[slot] = 1;
        w.ctl[CTL_UNPICKED] -= 1;
        sel[a] = 1;
        cache[a] = 0.0;
      }
    }
    __syncthreads();
    DBG_T(4)
    if (a >= 0 && rows) block_factor_rows<KIND>(ea, w, round, picks, sm.r);
    DBG_T(5)
    DBG_END_STEP()
    return;
  }
  // stall: the batch is chosen by exact_stall_kernel, which the host launches first thing in
  // the refinement (vgposp_exact_refine_pending)
  if (threadIdx.x == 0) w.ctl[CTL_STALL] = round;
}

template <int KIND>
__global__ __launch_bounds__(SEL_THREADS) void exact_step_kernel(EArgs ea, double* cache,
                                                                 unsigned char* sel, ExactWS w,
                                                                 long long nblk, long long nsb,
                                                                 int nslots, int round, int B,
                                                                 int rows, long long* picks,
                                                                 double* pick_delta) {
  __shared__ int s_slot;
  __shared__ StepSm sm;
  (void)B;
  step_body<KIND>(ea, cache, sel, w, nblk, nsb, nslots, round, rows, picks, pick_delta, sm, s_slot);
}

template <int KIND>
__global__ __launch_bounds__(WIN_T) void exact_window_kernel(EArgs a, const double* __restrict__ qdiag,
                                                             double* cache, const unsigned char* sel,
                                                             ExactWS w, int round,
                                                             const long long* picks) {
  __shared__ RowsLds sm;
  __shared__ StagedPicks sp;
  const long long at = picks[round];
  if (at < 0) return;
  const Window v = window_of(a, at);
  const int nr = round + 1;
  stage_picks(a, w, picks, nr, sp);
  if (nr * (nr + 1) <= ROWS_LDS) {
    const LRows L = stage_rows(w, round, sm);
    __syncthreads();
    window_tail<KIND>(a, qdiag, cache, sel, w, round, picks, v, sp, L, &sm);
  } else {
    __syncthreads();
    window_tail<KIND>(a, qdiag, cache, sel, w, round, picks, v, sp, global_rows(w), nullptr);
  }
}

// The refinement batch of a stalled round: the B best entries without a column, each given a
// free slot or the oldest unpinned one (the host loop's rule, ExactWindowGreedy.run_bounded of
// round 3).  One workgroup.
__global__ __launch_bounds__(SEL_THREADS) void exact_stall_kernel(double* cache, unsigned char* sel,
                                                                  long long n, ExactWS w,
                                                                  long long nblk, long long nsb,
                                                                  int nslots, int B) {
  __shared__ long long top[CG_B + 1];
  __shared__ long long s_todo[CG_B];
  DBG_DECL
  DBG_T(0)
  if (w.ctl[CTL_STALL] < 0) return;
  const long long a = block_argmax(w, nsb);
#if VGPOSP_EXACT_DBG != 3
  DBG_T(1)
#endif
  // stall: the B best entries without a column become the refinement batch.  The slot table is
  // staged in LDS and ranked in parallel (a first version walked it with thread 0's dependent
  // global loads: 750 us per stall at B = 32): free slots are taken first, lowest index first,
  // then the unpinned ones, oldest refinement first — the candidates in the batch have no column,
  // so no slot of theirs can be recycled.
#if VGPOSP_EXACT_DBG == 3
  DBG_T(0)
  block_topb_entries(cache, sel, n, w, nblk, nsb, B, top, dbg_t);
  DBG_T(5)
  DBG_END(1)
#else
  block_topb_entries(cache, sel, n, w, nblk, nsb, B, top);
#endif
  DBG_T(2)
  __shared__ long long s_cand[EX_SLOTS_MAX];
  __shared__ int s_age[EX_SLOTS_MAX], s_inv_free[EX_SLOTS_MAX], s_inv_old[EX_SLOTS_MAX];
  __shared__ unsigned char s_pin[EX_SLOTS_MAX];
  __shared__ int s_has[CG_B], s_nfree, s_nold;
  __shared__ unsigned char s_qx[CG_B + 1];  // qexact of the top entries and of the arg-max
  const int t = threadIdx.x;
  const int ntop = (int)top[0];
  if (t < nslots) {
    s_cand[t] = w.rl_cand[t];
    s_age[t] = w.rl_age[t];
    s_pin[t] = w.rl_pin[t];
  }
  if (t < CG_B) s_has[t] = 0;
  // (loaded in parallel here: thread 0's serial loop below would otherwise wait on one dependent
  // byte load per entry — its stores may alias them)
  if (t < ntop) s_qx[t] = w.qexact[top[1 + t]];
  if (t == CG_B && a >= 0) s_qx[CG_B] = w.qexact[a];
  if (t == 0) s_nfree = s_nold = 0;
  __syncthreads();
  DBG_T(3)
  for (int e = t; e < nslots * ntop; e += SEL_THREADS) {
    const int i = e / ntop, b = e % ntop;
    if (s_cand[i] >= 0 && s_cand[i] == top[1 + b]) s_has[b] = 1;
  }
  if (t < nslots) {
    const bool fr = s_cand[t] < 0, old = !fr && !s_pin[t];
    int rank = 0;
#pragma unroll 8
    for (int i = 0; i < nslots; ++i) {
      if (fr) rank += s_cand[i] < 0 && i < t;
      else if (old) rank += s_cand[i] >= 0 && !s_pin[i] && (s_age[i] < s_age[t] || (s_age[i] == s_age[t] && i < t));
    }
    if (fr) {
      s_inv_free[rank] = t;
      atomicAdd(&s_nfree, 1);
    } else if (old) {
      s_inv_old[rank] = t;
      atomicAdd(&s_nold, 1);
    }
  }
  __syncthreads();
  DBG_T(4)
  if (t < 64) {
    // without a column: a candidate still on its K_lo bound is tightened (K_hi bound, cheap); one
    // already tightened (or exact but recycled), and the arg-max itself, gets its CG column (the
    // arg-max would stall the next event on its own otherwise).  Wave 0, lane b for top entry b:
    // the two lists keep the entries' order (prefix counts), slot j goes to the j-th column.
    const int lane = t;
    const bool live = lane < ntop && !s_has[lane];
    const long long y = lane < ntop ? top[1 + lane] : -1;
    const bool tight = live && s_qx[lane] == 0 && y != a;
    const bool col = live && !tight;
    const unsigned long long mt = __ballot(tight), mc = __ballot(col);
    const unsigned long long below = (1ull << lane) - 1ull;
    int ntight = __popcll(mt), nt = __popcll(mc);
    if (tight) w.rt_cand[__popcll(mt & below)] = y;
    if (col) s_todo[__popcll(mc & below)] = y;
    if (nt == 0 && ntight == 0) {  // (wave-uniform)
      if (s_qx[CG_B] == 0) {
        if (lane == 0) w.rt_cand[0] = a;
        ntight = 1;
      } else {
        if (lane == 0) s_todo[0] = a;
        nt = 1;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nfree = s_nfree, nold = s_nold;
    const int nb = min(nt, nfree + nold), recycled = nb - min(nb, nfree);
    const int age = w.ctl[CTL_AGE];
    if (lane < nb) {
      // free slots first; then the unpinned ones (their candidates lose their columns: bounded again)
      const int slot_j = lane < nfree ? s_inv_free[lane] : s_inv_old[lane - nfree];
      const long long yj = s_todo[lane];
      w.rl_cand[slot_j] = yj;
      w.rl_age[slot_j] = age + lane;
      w.rf_cand[lane] = yj;
      w.rf_slot[lane] = slot_j;
    } else if (lane < CG_B) {
      w.rf_cand[lane] = -1;
      w.rf_slot[lane] = -1;
    }
    if (lane == 0) {
      w.ctl[CTL_NT] = ntight;
      w.ctl[CTL_AGE] = age + nb;
      w.ctl[CTL_UNPICKED] -= recycled;
      w.ctl[CTL_NB] = nb;
    }
  }
  DBG_T(5)
#if VGPOSP_EXACT_DBG != 3
  DBG_END(1)
#endif
}

}  // namespace vgposp

using namespace vgposp;

namespace {

#define VGPOSP_EXACT_CHECK_COMMON()                                                          \
  VG_CHECK_ARG(kind >= VGPOSP_KERNEL_EQ && kind <= VGPOSP_KERNEL_MATERN52, 1);             \
  VG_CHECK_ARG(X != nullptr, 2);                                                          \
  VG_CHECK_ARG(I0 >= 1 && I1 >= 1 && I2 >= 1 && I0 * I1 * I2 < (1LL << 31), 3);           \
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

template <class F>
int dispatch_kind(int kind, F&& f) {
  switch (kind) {
    case VGPOSP_KERNEL_EQ: return f(std::integral_constant<int, VGPOSP_KERNEL_EQ>{});
    case VGPOSP_KERNEL_MATERN12: return f(std::integral_constant<int, VGPOSP_KERNEL_MATERN12>{});
    case VGPOSP_KERNEL_MATERN32: return f(std::integral_constant<int, VGPOSP_KERNEL_MATERN32>{});
    default: return f(std::integral_constant<int, VGPOSP_KERNEL_MATERN52>{});
  }
}

template <int KIND>
int exact_prepare_t(const EArgs& a, const double* qdiag, double* cache, unsigned char* sel,
                    const ExactWS& w, int flags, hipStream_t s) {
  const long long n = a.n;
  const long long nblk = ceil_div(n, EB), nsb = ceil_div(nblk, ESB);
  const bool bounded = (flags & 1) != 0;
  VG_CHECK_ARG(n < (1LL << 31), 3);  // (coef_row's 32-bit grid coordinates)
  VG_HIP(vg_memset(sel, 0, n, s));
  VG_HIP(vg_memset(w.lastA, 0, n, s));
  // 0: on the K_lo bound, to be tightened first (flags & 2: a second bound level); 2: final bound
  VG_HIP(vg_memset(w.qexact, bounded ? ((flags & 2) ? 0 : 2) : 1, n, s));
  if (!bounded) {
    hipLaunchKernelGGL(exact_coef_kernel<KIND>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                       a, w.coef);
    VG_LAUNCH_CHECK();
  }
  {
    ProfScope ps("exact_score", s, 0.0, 16.0 * n);
    hipLaunchKernelGGL(exact_score_kernel<KIND>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                       a, qdiag, w.qexact, cache);
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

// cg_iters CG iterations for the nb columns centers[j] -> slots[j] (device arrays), from a
// fresh start, batched over blockIdx.y.
int exact_cg_run(const EArgs& a, const ExactWS& w, int nb, const int* slots,
                 const long long* centers, int radius, int cg_iters, double cg_tol,
                 hipStream_t s) {
  const long long bv = w.b0 * w.b1 * w.b2;
  const int m = a.m1 + 1;
  ProfScope ps("exact_cg", s, 0.0, (double)nb * cg_iters * 8.0 * bv * (m + 9));
  const double tol2 = cg_tol * cg_tol;
  // the 7-point stencil (face neighbours only): walk the Manhattan ball, not its bounding cube
  const bool oct = a.m1 == 6 && radius == 1;  // (the 6 offsets of squared distance 1)
  // ~8 elements per thread (one per thread had 800 short workgroups per column, 42 us a batch)
  const dim3 sg((unsigned)std::min<long long>(ceil_div(bv, 256 * 8), 1024), (unsigned)nb);
  if (oct)
    hipLaunchKernelGGL(exact_cg_start_kernel<true>, sg, dim3(256), 0, s, w, a.I0, a.I1, a.I2, slots,
                       centers);
  else
    hipLaunchKernelGGL(exact_cg_start_kernel<false>, sg, dim3(256), 0, s, w, a.I0, a.I1, a.I2, slots,
                       centers);
  VG_LAUNCH_CHECK();
  unsigned prev = 1;
  for (int it = 0; it < cg_iters; ++it) {
    // the unclipped active region bounds the launch: a grid that grows with the iterate's support
    const long long side = std::min<long long>(2LL * (it + 1) * radius + 1, 2 * w.H + 1);
    const long long R = std::min<long long>(it + 1, w.H);
    const unsigned blocks = (unsigned)std::min<long long>(
        CG_BLOCKS, oct ? ceil_div(2 * R * R + 2 * R + 1, (long long)(CG_T / 64 * CG_RPW))
                       : ceil_div(side * side * side, (long long)CG_T));
    if (oct) {
      hipLaunchKernelGGL(exact_cg_a_kernel<true>, dim3(blocks * (unsigned)nb), dim3(CG_T), 0, s, w,
                         a.I0, a.I1, a.I2, a.offs, a.m1, radius, slots, centers, it, (int)prev,
                         tol2, nb);
      VG_LAUNCH_CHECK();
      hipLaunchKernelGGL(exact_cg_b_kernel<true>, dim3(blocks * (unsigned)nb), dim3(CG_T), 0, s, w,
                         a.I0, a.I1, a.I2, radius, slots, centers, it, nb);
    } else {
      hipLaunchKernelGGL(exact_cg_a_kernel<false>, dim3(blocks * (unsigned)nb), dim3(CG_T), 0, s, w,
                         a.I0, a.I1, a.I2, a.offs, a.m1, radius, slots, centers, it, (int)prev,
                         tol2, nb);
      VG_LAUNCH_CHECK();
      hipLaunchKernelGGL(exact_cg_b_kernel<false>, dim3(blocks * (unsigned)nb), dim3(CG_T), 0, s, w,
                         a.I0, a.I1, a.I2, radius, slots, centers, it, nb);
    }
    VG_LAUNCH_CHECK();
    prev = blocks;
  }
  return 0;
}

template <int KIND>
int exact_update_t(const EArgs& a, const double* qdiag, double* cache, unsigned char* sel,
                   const ExactWS& w, int round, const long long* picks, hipStream_t s) {
  const long long nblk = ceil_div(a.n, EB);
  ProfScope ps("exact_update", s, 0.0, 0.0);
  const long long side = 2LL * a.cutoff;
  const long long nw = side * side * side;
  if (nw <= 0) {  // (otherwise the window kernel computes the pick's factor rows)
    hipLaunchKernelGGL(exact_rows_kernel<KIND>, dim3(1), dim3(128), 0, s, a, w, round, picks);
    VG_LAUNCH_CHECK();
  }
  if (nw > 0) {
    hipLaunchKernelGGL(exact_window_kernel<KIND>, dim3((unsigned)ceil_div(nw, WIN_CAND)), dim3(WIN_T), 0, s,
                       a, qdiag, cache, sel, w, round, picks);
    VG_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(exact_window_keys_kernel, dim3(1), dim3(SEL_THREADS), 0, s, a, cache, sel, w,
                     nblk, round, picks);
  VG_LAUNCH_CHECK();
  return 0;
}

template <int KIND>
int exact_round_t(const EArgs& a, const double* qdiag, double* cache, unsigned char* sel,
                  const ExactWS& w, int round, int last, long long* picks, double* pick_delta,
                  int radius, int cg_iters, double cg_tol, hipStream_t s) {
  const long long n = a.n;
  const long long nblk = ceil_div(n, EB), nsb = ceil_div(nblk, ESB);
  {
    ProfScope ps("exact_select", s, 0.0, 16.0 * nsb);
    hipLaunchKernelGGL(exact_select_kernel, dim3(1), dim3(SEL_THREADS), 0, s, cache, sel, a.I0, a.I1,
                       a.I2, w, nblk, nsb, round, picks, pick_delta);
    VG_LAUNCH_CHECK();
  }
  if (last) return 0;
  // the pick's column into slot `round` (exact_select_kernel wrote slot_of_round[round] = round)
  if (int rc = exact_cg_run(a, w, 1, w.slot_of_round + round, picks + round, radius, cg_iters,
                            cg_tol, s))
    return rc;
  return exact_update_t<KIND>(a, qdiag, cache, sel, w, round, picks, s);
}

template <int KIND>
int exact_refine_t(const EArgs& a, double* qdiag, double* cache, unsigned char* sel,
                   const ExactWS& w, int nb, const long long* cands, const int* slots,
                   const long long* picks, int radius, int cg_iters, double cg_tol, hipStream_t s,
                   int resume = 0) {
  const long long nblk = ceil_div(a.n, EB);
  if (int rc = exact_cg_run(a, w, nb, slots, cands, radius, cg_iters, cg_tol, s)) return rc;
  hipLaunchKernelGGL(exact_refine_end_kernel<KIND>, dim3(1), dim3(SEL_THREADS), 0, s, a, qdiag, cache, sel, w,
                     nblk, nb, slots, cands, picks, resume);
  VG_LAUNCH_CHECK();
  return 0;
}

}  // namespace

#define VGPOSP_EXACT_PARAMS                                                                      \
  int kind, const double *X, int64_t I0, int64_t I1, int64_t I2, double amp, double ls,          \
      double diag_shift, double jitter, double threshold, const int *offsets, int m,             \
      const double *tau, int ntau, int kmax, int cutoff, int radius, int cg_iters,               \
      const double *qdiag, double *cache, uint8_t *selected, void *ws, size_t ws_bytes

#define VGPOSP_EXACT_PROLOGUE(NAME)                                                              \
  clear_error();                                                                                 \
  VGPOSP_EXACT_CHECK_COMMON();                                                                   \
  const ExactWS w = exact_layout(ws, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters);           \
  if (ws_bytes < w.bytes) {                                                                      \
    set_error(NAME ": workspace %zu < %zu bytes", ws_bytes, w.bytes);                            \
    return VGPOSP_E_WS;                                                                          \
  }                                                                                              \
  const EArgs a = make_eargs(X, I0, I1, I2, amp, ls, diag_shift, jitter, threshold, offsets, m, \
                             tau, ntau, kmax, cutoff);                                           \
  hipStream_t s = as_stream(stream)

#if VGPOSP_EXACT_DBG
extern "C" int vgposp_exact_dbg(unsigned long long* out) {  // 64 x 8 records, then reset
  hipMemcpyFromSymbol(out, HIP_SYMBOL(vgposp::g_exact_dbg), sizeof(vgposp::g_exact_dbg));
  const unsigned z = 0;
  hipMemcpyToSymbol(HIP_SYMBOL(vgposp::g_exact_dbg_n), &z, sizeof(z));
  return 0;
}
#endif

extern "C" size_t vgposp_exact_workspace_bytes(int64_t I0, int64_t I1, int64_t I2, int m, int kmax,
                                               int radius, int cg_iters) {
  if (I0 <= 0 || I1 <= 0 || I2 <= 0 || m <= 0 || kmax <= 0 || radius < 1 || cg_iters < 1) return 0;
  return exact_layout(nullptr, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters).bytes;
}

extern "C" int vgposp_exact_prepare(VGPOSP_EXACT_PARAMS, int flags, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_prepare");
  VG_CHECK_ARG(flags == 0 || flags == 1 || flags == 3, 24);
  return dispatch_kind(kind, [&](auto K) {
    return exact_prepare_t<decltype(K)::value>(a, qdiag, cache, selected, w, flags, s);
  });
}

extern "C" int vgposp_exact_round(VGPOSP_EXACT_PARAMS, int round, int last, int64_t* picks,
                                  double* pick_delta, double cg_tol, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_round");
  VG_CHECK_ARG(round >= 0 && round < kmax, 24);
  VG_CHECK_ARG(picks != nullptr, 26);
  VG_CHECK_ARG(cg_tol >= 0.0, 28);
  long long* pk = reinterpret_cast<long long*>(picks);
  return dispatch_kind(kind, [&](auto K) {
    return exact_round_t<decltype(K)::value>(a, qdiag, cache, selected, w, round, last, pk,
                                             pick_delta, radius, cg_iters, cg_tol, s);
  });
}

extern "C" int vgposp_exact_coef(VGPOSP_EXACT_PARAMS, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_coef");
  const long long n = a.n;
  VG_CHECK_ARG(n < (1LL << 31), 3);  // (coef_row's 32-bit grid coordinates)
  const int rc = dispatch_kind(kind, [&](auto K) {
    if (coef_stride(m) == 8)
      hipLaunchKernelGGL(exact_coef8_kernel<decltype(K)::value>, dim3((unsigned)ceil_div(n, 256)),
                         dim3(256), 0, s, a, w.coef);
    else
      hipLaunchKernelGGL(exact_coef_kernel<decltype(K)::value>, dim3((unsigned)ceil_div(n, 256)),
                         dim3(256), 0, s, a, w.coef);
    VG_LAUNCH_CHECK();
    return 0;
  });
  if (rc) return rc;
  const unsigned blocks = (unsigned)std::min<long long>(CG_BLOCKS, ceil_div(n, 256));
  hipLaunchKernelGGL(exact_gersh_kernel, dim3(blocks), dim3(256), 0, s, w.coef, n, m, w.gersh);
  VG_LAUNCH_CHECK();
  hipLaunchKernelGGL(exact_gersh_final_kernel, dim3(1), dim3(64), 0, s, w.gersh, (int)blocks);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_exact_bounds(VGPOSP_EXACT_PARAMS, const int* tab_off, const int* tab_nb,
                                   const int* tab_cnt, int T, int K, double hi_scale, double mu,
                                   int64_t c0, int64_t c1, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_bounds");
  VG_CHECK_ARG(tab_off != nullptr, 24);
  VG_CHECK_ARG(m == 1 || tab_nb != nullptr, 25);
  VG_CHECK_ARG(tab_cnt != nullptr, 26);
  VG_CHECK_ARG(T >= 1 && T <= BND_TMAX && (int64_t)T * (m - 1) <= BND_NBMAX, 27);
  VG_CHECK_ARG(K >= 1 && K <= 4 * BND_SMAX, 28);
  VG_CHECK_ARG(hi_scale >= 1.0, 29);
  VG_CHECK_ARG(mu >= 0.0, 30);
  VG_CHECK_ARG(c0 >= 0 && c0 <= c1 && c1 <= a.n, 31);
  VG_CHECK_ARG(a.n < (1LL << 31), 3);
  if (c1 == c0) return 0;
  ProfScope ps("exact_bounds", s, 0.0, 0.0);
  const long long waves = c1 - c0;
  const unsigned blocks =
      (unsigned)(8 * std::min<long long>(ceil_div(ceil_div(waves, BND_WAVES), 8LL),
                                         BND_GRID / 8));
  double* out = const_cast<double*>(qdiag);
  const long long lc0 = c0, lc1 = c1;
#define VG_BOUNDS_REG(SMV)                                                                     \
  if (T <= 64 * SMV) {                                                                           \
    hipLaunchKernelGGL((exact_bounds_reg_kernel<SMV, 6>), dim3(blocks), dim3(BND_T), 0, s, w.coef, \
                       a.I0, a.I1, a.I2, tab_off, tab_nb, tab_cnt, T, K, hi_scale, mu, lc0, lc1,   \
                       out);                                                                      \
    VG_LAUNCH_CHECK();                                                                           \
    return 0;                                                                                    \
  }
  if (a.m1 == 6 && T <= 64 && BND_G > 1) {  // K <= 3: G candidates per wave
    constexpr int G = BND_G;
    // at most 16,384 workgroups: each wave then walks ~16 candidate pairs and the per-workgroup
    // table staging and per-wave address setup are amortised (65,536: 0.84 ms per 128^3 pass,
    // 16,384: 0.76, 8,192: 0.77; profiles/r5_c4_ab.jsonl)
    const unsigned gblocks =
        (unsigned)(8 * std::min<long long>(ceil_div(ceil_div(waves, BND_WAVES * G), 8LL),
                                           BND_GRP_GRID / 8));
    hipLaunchKernelGGL(exact_bounds_grp_kernel<G>, dim3(gblocks), dim3(BND_T), 0, s, w.coef, a.I0,
                       a.I1, a.I2, tab_off, tab_nb, tab_cnt, T, K, hi_scale, mu, lc0, lc1, out,
                       fast_div_for((unsigned)(a.I1 * a.I2)), fast_div_for((unsigned)a.I2));
    VG_LAUNCH_CHECK();
    return 0;
  }
  if (a.m1 == 6) {  // the 7-point taper support of the reference's beta = 4
    VG_BOUNDS_REG(1)
    VG_BOUNDS_REG(2)
    VG_BOUNDS_REG(3)
    VG_BOUNDS_REG(4)
    VG_BOUNDS_REG(6)
    VG_BOUNDS_REG(9)
  }
#undef VG_BOUNDS_REG
  hipLaunchKernelGGL(exact_bounds_kernel, dim3(blocks), dim3(BND_T), 0, s, w.coef, a.I0, a.I1, a.I2,
                     a.m1, tab_off, tab_nb, tab_cnt, T, K, hi_scale, mu, lc0, lc1, out);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_exact_steps_reset(VGPOSP_EXACT_PARAMS, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_steps_reset");
  (void)a;
  hipLaunchKernelGGL(exact_steps_reset_kernel, dim3(1), dim3(256), 0, s, w, exact_slots(kmax),
                     kmax);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_exact_steps(VGPOSP_EXACT_PARAMS, int round0, int round1, int k, int batch,
                                  int64_t* picks, double* pick_delta, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_steps");
  VG_CHECK_ARG(k >= 1 && k <= kmax, 26);
  VG_CHECK_ARG(round0 >= 0 && round0 <= round1 && round1 <= k, 24);
  VG_CHECK_ARG(batch >= 1 && batch <= CG_B, 27);
  VG_CHECK_ARG(picks != nullptr, 28);
  const long long nblk = ceil_div(a.n, EB), nsb = ceil_div(nblk, ESB);
  long long* pk = reinterpret_cast<long long*>(picks);
  const long long side = 2LL * a.cutoff;
  const long long nw = side * side * side;
  return dispatch_kind(kind, [&](auto K) {
    constexpr int KD = decltype(K)::value;
    for (int r = round0; r < round1; ++r) {
      const bool more = r + 1 < k;  // the last pick needs neither factor rows nor a window
      {
        ProfScope ps("exact_select", s, 0.0, 16.0 * nsb);
        // (the factor rows of pick r: in the window kernel, here only when there is no window)
        hipLaunchKernelGGL(exact_step_kernel<KD>, dim3(1), dim3(SEL_THREADS), 0, s, a, cache,
                           selected, w, nblk, nsb, exact_slots(kmax), r, batch,
                           (int)(more && nw <= 0), pk, pick_delta);
        VG_LAUNCH_CHECK();
      }
      if (more && nw > 0) {  // the window of pick r (no-op when the round stalled: picks[r] = -1)
        ProfScope ps("exact_update", s, 0.0, 0.0);
        hipLaunchKernelGGL(exact_window_kernel<KD>, dim3((unsigned)ceil_div(nw, WIN_CAND)), dim3(WIN_T), 0, s,
                           a, qdiag, cache, selected, w, r, pk);
        VG_LAUNCH_CHECK();
      }
    }
    // if a round stalled: choose its batch now, so ONE read of the control block tells the host
    // what to run (no-op otherwise)
    ProfScope ps("exact_stall", s, 0.0, 0.0);
    hipLaunchKernelGGL(exact_stall_kernel, dim3(1), dim3(SEL_THREADS), 0, s, cache, selected, a.n, w,
                       nblk, nsb, exact_slots(kmax), batch);
    VG_LAUNCH_CHECK();
    return 0;
  });
}

extern "C" int vgposp_exact_refine_pending(VGPOSP_EXACT_PARAMS, int batch, const int64_t* picks,
                                           double cg_tol, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_refine_pending");
  VG_CHECK_ARG(batch >= 1 && batch <= CG_B, 24);
  VG_CHECK_ARG(picks != nullptr, 25);
  VG_CHECK_ARG(cg_tol >= 0.0, 26);
  const long long* pk = reinterpret_cast<const long long*>(picks);
  return dispatch_kind(kind, [&](auto K) {
    return exact_refine_t<decltype(K)::value>(a, const_cast<double*>(qdiag), cache, selected, w,
                                              batch, w.rf_cand, w.rf_slot, pk, radius, cg_iters,
                                              cg_tol, s, 1);
  });
}

extern "C" int vgposp_exact_update(VGPOSP_EXACT_PARAMS, int round, const int64_t* picks,
                                   void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_update");
  VG_CHECK_ARG(round >= 0 && round < kmax, 24);
  VG_CHECK_ARG(picks != nullptr, 25);
  const long long* pk = reinterpret_cast<const long long*>(picks);
  return dispatch_kind(kind, [&](auto K) {
    return exact_update_t<decltype(K)::value>(a, qdiag, cache, selected, w, round, pk, s);
  });
}

extern "C" int vgposp_exact_buffers(void* ws, int64_t I0, int64_t I1, int64_t I2, int m, int kmax,
                                    int radius, int cg_iters, double** qcols, int64_t** boxlo,
                                    int** cgstate, int** slot_of_round, int64_t** cand,
                                    double** gersh) {
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  const ExactWS w = exact_layout(ws, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters);
  if (qcols) *qcols = w.Qcols;
  if (boxlo) *boxlo = reinterpret_cast<int64_t*>(w.boxlo);
  if (cgstate) *cgstate = w.cgstate;
  if (slot_of_round) *slot_of_round = w.slot_of_round;
  if (cand) *cand = reinterpret_cast<int64_t*>(w.cand);
  if (gersh) *gersh = w.gersh;
  return 0;
}

extern "C" int vgposp_exact_tighten_pending(VGPOSP_EXACT_PARAMS, const int* tab_off,
                                            const int* tab_nb, const int* tab_cnt, int T, int K,
                                            double hi_scale, double mu, const int64_t* picks,
                                            void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_tighten_pending");
  VG_CHECK_ARG(tab_off != nullptr && tab_nb != nullptr && tab_cnt != nullptr, 24);
  VG_CHECK_ARG(T >= 1 && T <= BND_TMAX && (int64_t)T * (m - 1) <= BND_NBMAX, 27);
  VG_CHECK_ARG(K >= 1 && K <= 4 * BND_SMAX, 28);
  VG_CHECK_ARG(hi_scale >= 1.0, 29);
  VG_CHECK_ARG(mu >= 0.0, 30);
  VG_CHECK_ARG(picks != nullptr, 31);
  VG_CHECK_ARG(a.m1 == 6, 12);  // the register bounds kernel (the 7-point taper)
  VG_CHECK_ARG(a.n < (1LL << 31), 3);
  const long long nblk = ceil_div(a.n, EB);
  double* out = const_cast<double*>(qdiag);
  const unsigned blocks = (unsigned)ceil_div(CG_B, BND_WAVES);
  {
    ProfScope ps("exact_tighten", s, 0.0, 0.0);
#define VG_TIGHT_REG(SMV)                                                                        \
  if (T <= 64 * SMV) {                                                                           \
    hipLaunchKernelGGL((exact_bounds_reg_kernel<SMV, 6, true>), dim3(blocks), dim3(BND_T), 0, s,   \
                       w.coef, a.I0, a.I1, a.I2, tab_off, tab_nb, tab_cnt, T, K, hi_scale, mu,    \
                       0LL, 0LL, out, w.rt_cand, w.ctl + CTL_NT);                                 \
  } else
    VG_TIGHT_REG(4) VG_TIGHT_REG(6) VG_TIGHT_REG(9) VG_TIGHT_REG(14) {
      set_error("vgposp_exact_tighten_pending: reach table of %d nodes", T);
      return 27;
    }
#undef VG_TIGHT_REG
    VG_LAUNCH_CHECK();
  }
  return dispatch_kind(kind, [&](auto KK) {
    hipLaunchKernelGGL(exact_tighten_end_kernel<decltype(KK)::value>, dim3(1), dim3(SEL_THREADS), 0, s,
                       a, qdiag, cache, selected, w, nblk,
                       reinterpret_cast<const long long*>(picks));
    VG_LAUNCH_CHECK();
    return 0;
  });
}

extern "C" int vgposp_exact_pretighten(VGPOSP_EXACT_PARAMS, const int* tab_off,
                                       const int* tab_nb, const int* tab_cnt, int T, int K,
                                       double hi_scale, double mu, int64_t M, void* stream) {
  VGPOSP_EXACT_PROLOGUE("vgposp_exact_pretighten");
  VG_CHECK_ARG(tab_off != nullptr && tab_nb != nullptr && tab_cnt != nullptr, 24);
  VG_CHECK_ARG(T >= 1 && T <= BND_TMAX && (int64_t)T * (m - 1) <= BND_NBMAX, 27);
  VG_CHECK_ARG(K >= 1 && K <= 4 * BND_SMAX, 28);
  VG_CHECK_ARG(hi_scale >= 1.0, 29);
  VG_CHECK_ARG(mu >= 0.0, 30);
  VG_CHECK_ARG(M >= 1 && M <= PT_MAX / 2, 31);
  VG_CHECK_ARG(a.m1 == 6, 12);  // the register bounds kernel (the 7-point taper)
  VG_CHECK_ARG(a.n < (1LL << 31), 3);
  const long long n = a.n, nblk = ceil_div(n, EB), nsb = ceil_div(nblk, ESB);
  // (512 workgroups: each merges its 4,096-bin histogram into the global one with atomics)
  const unsigned sweep = (unsigned)std::min<long long>(ceil_div(n, 256), 512);
  double* out = const_cast<double*>(qdiag);
  ProfScope ps("exact_pretighten", s, 0.0, 0.0);
  VG_HIP(vg_memset(w.pt_hist, 0, 4 * (size_t)PT_BINS, s));
  hipLaunchKernelGGL(exact_pt_init_kernel, dim3(1), dim3(64), 0, s, w.pt_state, (long long)M);
  VG_LAUNCH_CHECK();
  for (int pass = 0; pass < PT_PASSES; ++pass) {
    hipLaunchKernelGGL(exact_pt_hist_kernel, dim3(sweep), dim3(256), 0, s, cache, w.qexact, n,
                       w.pt_state, pass, w.pt_hist);
    VG_LAUNCH_CHECK();
    hipLaunchKernelGGL(exact_pt_pick_kernel, dim3(1), dim3(64), 0, s, w.pt_state, pass, w.pt_hist);
    VG_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(exact_pt_list_kernel, dim3(sweep), dim3(256), 0, s, cache, w.qexact, n,
                     w.pt_state, w.pt_list, w.pt_count);
  VG_LAUNCH_CHECK();
  hipLaunchKernelGGL(exact_pt_count_kernel, dim3(1), dim3(64), 0, s, w.pt_state, w.pt_count,
                     w.ctl);
  VG_LAUNCH_CHECK();
  const unsigned blocks = (unsigned)std::min<long long>(ceil_div(M + 4096, BND_WAVES), 2048);
#define VG_PT_REG(SMV)                                                                           \
  if (T <= 64 * SMV) {                                                                           \
    hipLaunchKernelGGL((exact_bounds_reg_kernel<SMV, 6, true>), dim3(blocks), dim3(BND_T), 0, s,   \
                       w.coef, a.I0, a.I1, a.I2, tab_off, tab_nb, tab_cnt, T, K, hi_scale, mu,    \
                       0LL, 0LL, out, w.pt_list, w.pt_count);                                     \
  } else
  VG_PT_REG(4) VG_PT_REG(6) VG_PT_REG(9) VG_PT_REG(14) {
    set_error("vgposp_exact_pretighten: reach table of %d nodes", T);
    return 27;
  }
#undef VG_PT_REG
  VG_LAUNCH_CHECK();
  return dispatch_kind(kind, [&](auto KK) {
    hipLaunchKernelGGL(exact_pt_score_kernel<decltype(KK)::value>,
                       dim3((unsigned)ceil_div(PT_MAX, 256)), dim3(256), 0, s, a, qdiag, w.qexact,
                       cache, w.pt_list, w.pt_count);
    VG_LAUNCH_CHECK();
    hipLaunchKernelGGL(exact_block_keys_kernel, dim3((unsigned)ceil_div(nblk, 4)), dim3(256), 0, s,
                       cache, selected, n, w.bval, w.bidx, nblk);
    VG_LAUNCH_CHECK();
    hipLaunchKernelGGL(exact_super_keys_kernel, dim3((unsigned)ceil_div(nsb, 4)), dim3(256), 0, s,
                       w.bval, w.bidx, nblk, w.sval, w.sidx, nsb);
    VG_LAUNCH_CHECK();
    return 0;
  });
}

extern "C" int vgposp_exact_ctl(void* ws, int64_t I0, int64_t I1, int64_t I2, int m, int kmax,
                                int radius, int cg_iters, int** ctl) {
  clear_error();
  VG_CHECK_ARG(ws != nullptr, 1);
  VG_CHECK_ARG(ctl != nullptr, 9);
  *ctl = exact_layout(ws, I0, I1, I2, m, kmax, (int64_t)radius * cg_iters).ctl;
  return 0;
}
