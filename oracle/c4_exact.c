// TEST INFRASTRUCTURE (never shipped, never called by vgposp_amd): a CPU restatement in plain C of
// config C4's exact algorithm 3 — snippets_a3.sparse_placement_algorithm_3 (snippets_a3.py:43-364)
// on the beta-decay tapered covariance of main_architecture_2_sampledistribution.py:355-421 — in
// the bounded-lazy form of vgposp_amd/csrc/exact_greedy.hip, so that the GPU picks can be checked
// against a CPU run at 128^3, where no dense algorithm 3 fits (Sigma would be 35 TB).
//
//   nom_y = s_yy - s_yA (S_AA + eps I)^-1 s_Ay                       (tf_nominator, eps = jitter)
//   den_y = 1 / P_yy - eps,  P_yy = Q_yy - Q_yA Q_AA^-1 Q_Ay,  Q = (S + eps I)^-1   (tf_denominator)
//   delta = 0 when |nom| or |den| < thr, else nom / den                   (snippets_a2.py:480)
//
// Q_yy is bracketed by K CG steps from e_y (g_K <= Q_yy <= hi_scale g_K); the cache holds upper
// bounds of the cached deltas; an arg-max on a bracketed candidate computes its CG column (Q_cc
// exact to rounding) and re-scores its entry with the A of its last window re-score; picks are
// taken only on exact entries, so they are the reference algorithm's arg-maxes (lowest index on
// ties, placement_algorithm2.py:24-50).  The stopping rules, iteration counts and the Krylov box
// are the GPU's; summation orders differ (sequential here), so values agree to rounding.
//
// Build: oracle/Makefile (gcc -O3 -fopenmp); bound by oracle/c4_exact.py (ctypes).
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

// OpenMP threads the bounds loop runs on.
int c4o_threads(void) { return omp_get_max_threads(); }
// the OpenMP team size of the next runs (the CPU baseline times it at OMP_NUM_THREADS and at
// every CPU of the host)
void c4o_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}

typedef struct {
  const double* X;
  long long I0, I1, I2, n;
  int kind;  // 0 EQ, 1 Matern 1/2, 2 Matern 3/2, 3 Matern 5/2
  double tla, inv_ls, inv_ls2, shift, jitter, thr;
  const int* offs;
  int m1;
  const double* tau;
  int ntau;
} Prob;

static double kfun(const Prob* p, double d2) {
  if (p->kind == 0) return exp(p->tla - 0.5 * d2 * p->inv_ls2);
  const double r = sqrt(d2) * p->inv_ls;
  if (p->kind == 1) return exp(p->tla - r);
  if (p->kind == 2) {
    const double s = 1.7320508075688772 * r;
    return (1.0 + s) * exp(p->tla - s);
  }
  const double s = 2.23606797749979 * r;
  return (1.0 + s + s * s * (1.0 / 3.0)) * exp(p->tla - s);
}

static double sigma_diag(const Prob* p) { return p->tau[0] * (kfun(p, 0.0) + p->shift); }

static double sigma_off(const Prob* p, long long i, long long j) {
  const long long I12 = p->I1 * p->I2;
  const long long e0 = i / I12 - j / I12, e1 = (i / p->I2) % p->I1 - (j / p->I2) % p->I1,
                  e2 = i % p->I2 - j % p->I2;
  const long long d2i = e0 * e0 + e1 * e1 + e2 * e2;
  if (d2i >= p->ntau || p->tau[d2i] == 0.0) return 0.0;
  const double d0 = p->X[3 * i] - p->X[3 * j], d1 = p->X[3 * i + 1] - p->X[3 * j + 1],
               d2 = p->X[3 * i + 2] - p->X[3 * j + 2];
  return p->tau[d2i] * kfun(p, d0 * d0 + d1 * d1 + d2 * d2);
}

static Prob make_prob(const double* X, long long I0, long long I1, long long I2, int kind,
                      double amp, double ls, double shift, double jitter, double thr,
                      const int* offs, int m1, const double* tau, int ntau) {
  Prob p;
  p.X = X;
  p.I0 = I0;
  p.I1 = I1;
  p.I2 = I2;
  p.n = I0 * I1 * I2;
  p.kind = kind;
  p.tla = 2.0 * log(amp);
  p.inv_ls = 1.0 / ls;
  p.inv_ls2 = 1.0 / (ls * ls);
  p.shift = shift;
  p.jitter = jitter;
  p.thr = thr;
  p.offs = offs;
  p.m1 = m1;
  p.tau = tau;
  p.ntau = ntau;
  return p;
}

// coef[i][0] = S_ii + eps, coef[i][1 + o] = S(i, i + off_o) (0 outside the grid); lam = the
// Gershgorin bounds [min_i c_ii - sum |c_ij|, max_i c_ii + sum |c_ij|].
int c4o_coef(const double* X, long long I0, long long I1, long long I2, int kind, double amp,
             double ls, double shift, double jitter, const int* offs, int m1, const double* tau,
             int ntau, double* coef, double* lam) {
  const Prob p = make_prob(X, I0, I1, I2, kind, amp, ls, shift, jitter, 0.0, offs, m1, tau, ntau);
  const int m = m1 + 1;
  double lo = INFINITY, hi = -INFINITY;
#pragma omp parallel for reduction(min : lo) reduction(max : hi) schedule(static)
  for (long long i = 0; i < p.n; ++i) {
    double* c = coef + i * m;
    c[0] = sigma_diag(&p) + jitter;
    const long long i0 = i / (I1 * I2), i1 = (i / I2) % I1, i2 = i % I2;
    double s = 0.0;
    for (int o = 0; o < m1; ++o) {
      const long long j0 = i0 + offs[3 * o], j1 = i1 + offs[3 * o + 1], j2 = i2 + offs[3 * o + 2];
      double v = 0.0;
      if (j0 >= 0 && j0 < I0 && j1 >= 0 && j1 < I1 && j2 >= 0 && j2 < I2)
        v = sigma_off(&p, i, (j0 * I1 + j1) * I2 + j2);
      c[1 + o] = v;
      s += fabs(v);
    }
    if (c[0] - s < lo) lo = c[0] - s;
    if (c[0] + s > hi) hi = c[0] + s;
  }
  lam[0] = lo;
  lam[1] = hi;
  return 0;
}

typedef struct {
  long long lo[3];
  double* x;  // box values
} Column;

typedef struct {
  Prob p;
  const double* coef;
  int m;
  long long H, b0, b1, b2;
  int srad, cg_iters;
  double tol2;
} Ctx;

// CG on S x = e_c over the Krylov box of c (half-width H, clipped into the grid), the GPU's
// iteration count and stopping rule; the active cube of iteration it is within (it + 1) srad.
static void cg_column(const Ctx* C, long long c, Column* col, double* r, double* pa, double* pb,
                      double* q) {
  const Prob* p = &C->p;
  const long long I1 = p->I1, I2 = p->I2;
  const long long a0 = c / (I1 * I2), a1 = (c / I2) % I1, a2 = c % I2;
  long long lo[3] = {a0 - C->H, a1 - C->H, a2 - C->H};
  const long long bd[3] = {C->b0, C->b1, C->b2}, Id[3] = {p->I0, p->I1, p->I2};
  for (int d = 0; d < 3; ++d) {
    if (lo[d] < 0) lo[d] = 0;
    if (lo[d] > Id[d] - bd[d]) lo[d] = Id[d] - bd[d];
    col->lo[d] = lo[d];
  }
  const long long bv = C->b0 * C->b1 * C->b2;
  memset(r, 0, 8 * bv);
  memset(pa, 0, 8 * bv);
  memset(pb, 0, 8 * bv);
  memset(col->x, 0, 8 * bv);
  r[((a0 - lo[0]) * C->b1 + (a1 - lo[1])) * C->b2 + (a2 - lo[2])] = 1.0;
  double rr = 1.0, rr_prev = 1.0;
  for (int it = 0; it < C->cg_iters; ++it) {
    if (rr <= C->tol2) break;
    const double beta = it == 0 ? 0.0 : rr / rr_prev;
    double* pold = (it & 1) ? pa : pb;
    double* pnew = (it & 1) ? pb : pa;
    long long rad = (long long)(it + 1) * C->srad;
    if (rad > C->H) rad = C->H;
    long long c0[3], e[3];
    const long long a[3] = {a0, a1, a2};
    for (int d = 0; d < 3; ++d) {
      c0[d] = a[d] - rad > lo[d] ? a[d] - rad : lo[d];
      const long long c1 = a[d] + rad < lo[d] + bd[d] - 1 ? a[d] + rad : lo[d] + bd[d] - 1;
      e[d] = c1 - c0[d] + 1;
    }
    double pq = 0.0;
    for (long long g0 = c0[0]; g0 < c0[0] + e[0]; ++g0)
      for (long long g1 = c0[1]; g1 < c0[1] + e[1]; ++g1)
        for (long long g2 = c0[2]; g2 < c0[2] + e[2]; ++g2) {
          const long long l = ((g0 - lo[0]) * C->b1 + (g1 - lo[1])) * C->b2 + (g2 - lo[2]);
          const double pi = it == 0 ? r[l] : beta * pold[l] + r[l];
          const double* cf = C->coef + ((g0 * I1 + g1) * I2 + g2) * C->m;
          double s = cf[0] * pi;
          for (int o = 0; o < p->m1; ++o) {
            const double cv = cf[1 + o];
            if (cv == 0.0) continue;
            const long long j0 = g0 + p->offs[3 * o] - lo[0], j1 = g1 + p->offs[3 * o + 1] - lo[1],
                            j2 = g2 + p->offs[3 * o + 2] - lo[2];
            if (j0 < 0 || j0 >= C->b0 || j1 < 0 || j1 >= C->b1 || j2 < 0 || j2 >= C->b2) continue;
            const long long j = (j0 * C->b1 + j1) * C->b2 + j2;
            const double pj = it == 0 ? r[j] : beta * pold[j] + r[j];
            s += cv * pj;
          }
          pnew[l] = pi;
          q[l] = s;
          pq += pi * s;
        }
    const double alpha = rr / pq;
    double rn = 0.0;
    for (long long g0 = c0[0]; g0 < c0[0] + e[0]; ++g0)
      for (long long g1 = c0[1]; g1 < c0[1] + e[1]; ++g1)
        for (long long g2 = c0[2]; g2 < c0[2] + e[2]; ++g2) {
          const long long l = ((g0 - lo[0]) * C->b1 + (g1 - lo[1])) * C->b2 + (g2 - lo[2]);
          col->x[l] += alpha * pnew[l];
          r[l] -= alpha * q[l];
          rn += r[l] * r[l];
        }
    rr_prev = rr;
    rr = rn;
  }
}

static double col_at(const Ctx* C, const Column* col, long long y) {
  const long long I1 = C->p.I1, I2 = C->p.I2;
  const long long l0 = y / (I1 * I2) - col->lo[0], l1 = (y / I2) % I1 - col->lo[1],
                  l2 = y % I2 - col->lo[2];
  if (l0 < 0 || l0 >= C->b0 || l1 < 0 || l1 >= C->b1 || l2 < 0 || l2 >= C->b2) return 0.0;
  return col->x[(l0 * C->b1 + l1) * C->b2 + l2];
}

static double delta_from(double nom, double P, int exact, double eps, double thr) {
  const double den = 1.0 / P - eps;
  if (exact) return (fabs(nom) < thr || fabs(den) < thr) ? 0.0 : nom / den;
  if (fabs(nom) < thr) return 0.0;
  return nom / (den > thr ? den : thr);
}

// The cached delta of y given the first nA picks (rows of LS / LQ, kmax stride).
static double rescore(const Ctx* C, const long long* picks, Column* const* pcol, int nA,
                      const double* LS, const double* LQ, int km, long long y, double qyy,
                      int exact, double* zs, double* zq) {
  double ns = 0.0, nq = 0.0;
  for (int r = 0; r < nA; ++r) {
    double vs = sigma_off(&C->p, picks[r], y), vq = col_at(C, pcol[r], y);
    for (int s = 0; s < r; ++s) {
      vs -= LS[r * km + s] * zs[s];
      vq -= LQ[r * km + s] * zq[s];
    }
    zs[r] = vs / LS[r * km + r];
    zq[r] = vq / LQ[r * km + r];
    ns += zs[r] * zs[r];
    nq += zq[r] * zq[r];
  }
  return delta_from(sigma_diag(&C->p) - ns, qyy - nq, exact, C->p.jitter, C->p.thr);
}

// The whole run.  tab_off [T][3] / tab_nb [T][m1] / tab_cnt [K + 1]: the reach table of
// sparse_placement.reach_table(offsets, K); hi_scale = (1 + margin) / (1 - 4 rho^2K).
// Outputs: picks [k] (-1 past the last candidate), deltas [k], stats [2] = (refinements, rounds).
int c4o_run(const double* X, long long I0, long long I1, long long I2, int kind, double amp,
            double ls, double shift, double jitter, double thr, const int* offs, int m1,
            const double* tau, int ntau, const double* coef, const int* tab_off,
            const int* tab_nb, const int* tab_cnt, int T, int K, double hi_scale, int cg_iters,
            double cg_tol, int k, int cutoff, long long* picks, double* deltas, long long* stats) {
  Ctx C;
  C.p = make_prob(X, I0, I1, I2, kind, amp, ls, shift, jitter, thr, offs, m1, tau, ntau);
  C.coef = coef;
  C.m = m1 + 1;
  int srad = 1;
  for (int o = 0; o < 3 * m1; ++o) srad = abs(offs[o]) > srad ? abs(offs[o]) : srad;
  C.srad = srad;
  C.cg_iters = cg_iters;
  C.tol2 = cg_tol * cg_tol;
  C.H = (long long)srad * cg_iters;
  C.b0 = 2 * C.H + 1 < I0 ? 2 * C.H + 1 : I0;
  C.b1 = 2 * C.H + 1 < I1 ? 2 * C.H + 1 : I1;
  C.b2 = 2 * C.H + 1 < I2 ? 2 * C.H + 1 : I2;
  const long long n = C.p.n, bv = C.b0 * C.b1 * C.b2;
  double* qd = (double*)malloc(8 * n);
  double* cache = (double*)malloc(8 * n);
  unsigned char* exact = (unsigned char*)calloc(n, 1);
  unsigned char* sel = (unsigned char*)calloc(n, 1);
  int* lastA = (int*)calloc(n, sizeof(int));
  int* colid = (int*)malloc(sizeof(int) * n);
  const int maxcols = (int)(n < 64LL * k + 4096 ? n : 64LL * k + 4096);
  Column* cols = (Column*)calloc(maxcols, sizeof(Column));
  Column** pcol = (Column**)calloc(k > 0 ? k : 1, sizeof(Column*));
  double* LS = (double*)calloc((size_t)k * k + 1, 8);
  double* LQ = (double*)calloc((size_t)k * k + 1, 8);
  double *r = (double*)malloc(8 * bv), *pa = (double*)malloc(8 * bv), *pb = (double*)malloc(8 * bv),
         *q = (double*)malloc(8 * bv);
  double* zs = (double*)malloc(8 * (k + 1));
  double* zq = (double*)malloc(8 * (k + 1));
  for (long long i = 0; i < n; ++i) colid[i] = -1;
  const double syy = sigma_diag(&C.p);
  // brackets of every Q_yy: K CG steps from e_y on the reach table around y
#pragma omp parallel
  {
    double* vr = (double*)malloc(8 * T);
    double* vp = (double*)malloc(8 * (T + 1));
    double* vq = (double*)malloc(8 * T);
    long long* gi = (long long*)malloc(8 * T);
#pragma omp for schedule(static)
    for (long long y = 0; y < n; ++y) {
      const long long y0 = y / (I1 * I2), y1 = (y / I2) % I1, y2 = y % I2;
      for (int j = 0; j < T; ++j) {
        const long long g0 = y0 + tab_off[3 * j], g1 = y1 + tab_off[3 * j + 1],
                        g2 = y2 + tab_off[3 * j + 2];
        gi[j] = (g0 >= 0 && g0 < I0 && g1 >= 0 && g1 < I1 && g2 >= 0 && g2 < I2)
                    ? (g0 * I1 + g1) * I2 + g2
                    : -1;
        vr[j] = j == 0 ? 1.0 : 0.0;
        vp[j] = vr[j];
      }
      vp[T] = 0.0;
      double rr = 1.0, g = 0.0;
      for (int it = 0; it < K; ++it) {
        const int cnt = tab_cnt[it + 1];
        double pq = 0.0;
        for (int j = 0; j < cnt; ++j) {
          double acc = 0.0;
          if (gi[j] >= 0) {
            const double* c = coef + gi[j] * C.m;
            acc = c[0] * vp[j];
            for (int o = 0; o < m1; ++o) {
              const int jn = tab_nb[j * m1 + o];
              if (jn >= 0) acc += c[1 + o] * vp[jn];
            }
          }
          vq[j] = acc;
          pq += vp[j] * acc;
        }
        const double alpha = rr / pq;
        g += alpha * rr;
        if (it + 1 == K) break;
        double rn = 0.0;
        for (int j = 0; j < cnt; ++j) {
          vr[j] -= alpha * vq[j];
          rn += vr[j] * vr[j];
        }
        const double beta = rn / rr;
        rr = rn;
        for (int j = 0; j < cnt; ++j) vp[j] = vr[j] + beta * vp[j];
      }
      qd[y] = g * hi_scale;
      cache[y] = delta_from(syy, qd[y], 0, jitter, thr);
    }
    free(vr);
    free(vp);
    free(vq);
    free(gi);
  }
  long long refinements = 0;
  int ncols = 0, rounds = 0;
  for (int t = 0; t < k; ++t) {
    long long c = -1;
    for (;;) {
      double best = 0.0;
      c = -1;
      for (long long y = 0; y < n; ++y) {
        if (sel[y]) continue;
        const double v = cache[y];
        if (c < 0 || v > best) {  // strict: the lowest index wins ties
          best = v;
          c = y;
        }
      }
      if (c < 0 || colid[c] >= 0) break;
      if (ncols == maxcols) {  // out of column storage: give up (the caller sees stats)
        stats[0] = refinements;
        stats[1] = -1;
        return 1;
      }
      cols[ncols].x = (double*)malloc(8 * bv);
      cg_column(&C, c, &cols[ncols], r, pa, pb, q);
      colid[c] = ncols++;
      const double qcc = col_at(&C, &cols[colid[c]], c);
      qd[c] = qcc;
      exact[c] = 1;
      cache[c] = rescore(&C, picks, pcol, lastA[c], LS, LQ, k, c, qcc, 1, zs, zq);
      ++refinements;
    }
    if (c < 0) {
      for (int u = t; u < k; ++u) {
        picks[u] = -1;
        deltas[u] = 0.0;
      }
      break;
    }
    picks[t] = c;
    deltas[t] = cache[c];
    pcol[t] = &cols[colid[c]];
    sel[c] = 1;
    cache[c] = 0.0;
    ++rounds;
    if (t == k - 1) break;
    // rows t of LQ = chol(Q_AA) and LS = chol(S_AA + eps I)
    for (int rr_ = 0; rr_ <= t; ++rr_) {
      const long long ar = picks[rr_];
      double vq = col_at(&C, pcol[t], ar);
      double vs = rr_ == t ? syy + jitter : sigma_off(&C.p, c, ar);
      for (int s = 0; s < rr_; ++s) {
        vq -= LQ[t * k + s] * LQ[rr_ * k + s];
        vs -= LS[t * k + s] * LS[rr_ * k + s];
      }
      if (rr_ == t) {
        LQ[t * k + t] = sqrt(vq);
        LS[t * k + t] = sqrt(vs);
      } else {
        LQ[t * k + rr_] = vq / LQ[rr_ * k + rr_];
        LS[t * k + rr_] = vs / LS[rr_ * k + rr_];
      }
    }
    // the window [i - cutoff, i + cutoff) per axis (snippets_a3.py:190-303)
    const long long ci[3] = {c / (I1 * I2), (c / I2) % I1, c % I2}, Id[3] = {I0, I1, I2};
    long long wlo[3], whi[3];
    for (int d = 0; d < 3; ++d) {
      wlo[d] = ci[d] - cutoff > 0 ? ci[d] - cutoff : 0;
      whi[d] = ci[d] + cutoff < Id[d] ? ci[d] + cutoff : Id[d];
    }
    for (long long j0 = wlo[0]; j0 < whi[0]; ++j0)
      for (long long j1 = wlo[1]; j1 < whi[1]; ++j1)
        for (long long j2 = wlo[2]; j2 < whi[2]; ++j2) {
          const long long y = (j0 * I1 + j1) * I2 + j2;
          if (sel[y]) {
            cache[y] = 0.0;
            continue;
          }
          cache[y] = rescore(&C, picks, pcol, t + 1, LS, LQ, k, y, qd[y], exact[y], zs, zq);
          lastA[y] = t + 1;
        }
  }
  stats[0] = refinements;
  stats[1] = rounds;
  for (int i = 0; i < ncols; ++i) free(cols[i].x);
  free(cols);
  free(pcol);
  free(LS);
  free(LQ);
  free(r);
  free(pa);
  free(pb);
  free(q);
  free(zs);
  free(zq);
  free(qd);
  free(cache);
  free(exact);
  free(sel);
  free(lastA);
  free(colid);
  return 0;
}
