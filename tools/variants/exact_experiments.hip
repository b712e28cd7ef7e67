// A/B VARIANTS, NOT BUILT: measured-slower C4 kernels moved out of vgposp_amd/csrc/exact_greedy.hip
// (round 5 hygiene).  Kept for the record of what was measured; DESIGN.md §4a cites the numbers.
//
// exact_bounds_tile_kernel: the all-candidate bounds with each 4^3 tile's coefficient rows (and a
// 3-node halo) staged in LDS.  Bit-identical bounds, 1.81 ms against the register kernel's 1.70 ms
// per 128^3 pass (profiles/r4_c4_bounds_tile.jsonl).  Its launch lived in vgposp_exact_bounds:
//
// #ifndef VGPOSP_BND_TILE  // (A/B: 1 = the tiled kernel for T <= 64; measured slower, see there)
// #define VGPOSP_BND_TILE 0
// #endif
//   if (VGPOSP_BND_TILE && a.m1 == 6 && T <= 64) {
//     // the tiles of the grid planes y0 that [c0, c1) touches
//     const long long plane = a.I1 * a.I2;
//     const long long TD1 = ceil_div(a.I1, (long long)BT_E), TD2 = ceil_div(a.I2, (long long)BT_E);
//     const long long lo = c0 / plane / BT_E * TD1 * TD2, hi = ((c1 - 1) / plane / BT_E + 1) * TD1 * TD2;
//     const long long per_xcd = ceil_div(hi - lo, 8LL);
//     hipLaunchKernelGGL(exact_bounds_tile_kernel<6>, dim3((unsigned)(8 * per_xcd)), dim3(BT_T), 0, s,
//                        w.coef, a.I0, a.I1, a.I2, tab_off, tab_nb, tab_cnt, T, K, hi_scale, mu, lc0,
//                        lc1, out, (int)lo, (int)hi, (int)per_xcd);
//     VG_LAUNCH_CHECK();
//     return 0;
//   }

// The all-candidate bounds for K <= BT_H steps on the 7-point stencil (one reach-table slot per
// lane, T <= 64), tiled: a workgroup takes a BT_E^3 tile of candidates and stages the coefficient
// rows of the tile and its BT_H halo (BT_B^3 = 1,000 rows, 56 KB as seven planes) into LDS once,
// with neighbouring rows on neighbouring lanes; a candidate's 63 rows are then LDS reads, not 63
// scattered 64-byte global loads (15.6 staged rows per candidate against 63 loaded ones).  The CG
// is exactly exact_bounds_reg_kernel's (bounds_cg, the same coefficients in the same order), so
// the bounds are bit-identical.  A table offset outside the halo (a stencil with longer reach)
// reads its row from global memory, as the register kernel does.
// A/B only (-DVGPOSP_BND_TILE=1, profiles/r4_c4_bounds_tile.jsonl): bounds bit-identical, but the
// 128^3 K = 3 pass takes 1.81 ms against the register kernel's 1.70.  The coefficient loads were
// not the bound: a candidate is ~500 wave instructions of CG (the six gathers, FMAs, two wave
// sums and three fp64 divisions per step), and the 61 KB of LDS halves the waves per SIMD.
constexpr int BT_E = 4, BT_H = 3, BT_B = BT_E + 2 * BT_H, BT_ROWS = BT_B * BT_B * BT_B;
constexpr int BT_T = 512, BT_WAVES = BT_T / 64;

template <int M1>
__global__ __launch_bounds__(BT_T) void exact_bounds_tile_kernel(
    const double* __restrict__ coef, long long I0, long long I1, long long I2,
    const int* __restrict__ tab_off, const int* __restrict__ tab_nb,
    const int* __restrict__ tab_cnt, int T, int K, double hi_scale, double mu, long long c0,
    long long c1, double* __restrict__ qhi, int tile_lo, int tile_hi, int per_xcd) {
  constexpr int M = M1 + 1;
  __shared__ double cl[M][BT_ROWS];
  __shared__ double plds[BT_WAVES][64 + 1];
  __shared__ short nbl[64 * M1];
  __shared__ int cntl[4 * BND_SMAX + 1];
  // XCD-aware: XCD x (= blockIdx.x mod 8) takes its own contiguous run of tiles, so the halos
  // neighbouring tiles share meet in the same L2
  const int tile = tile_lo + (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
  if (tile >= tile_hi) return;  // (whole workgroup)
  const int I0i = (int)I0, I1i = (int)I1, I2i = (int)I2;
  const int TD1 = (I1i + BT_E - 1) / BT_E, TD2 = (I2i + BT_E - 1) / BT_E;
  const int t0 = tile / (TD1 * TD2) * BT_E, t1 = tile / TD2 % TD1 * BT_E, t2 = tile % TD2 * BT_E;
  for (int i = threadIdx.x; i < 64 * M1; i += BT_T) {
    const int v = i < T * M1 ? tab_nb[i] : -1;
    nbl[i] = (short)(v >= 0 ? v : 64);
  }
  for (int i = threadIdx.x; i <= K; i += BT_T) cntl[i] = tab_cnt[i];
  for (int b = threadIdx.x; b < BT_ROWS; b += BT_T) {
    const int g0 = t0 - BT_H + b / (BT_B * BT_B), g1 = t1 - BT_H + b / BT_B % BT_B,
              g2 = t2 - BT_H + b % BT_B;
    int gi = -1;
    if ((unsigned)g0 < (unsigned)I0i && (unsigned)g1 < (unsigned)I1i && (unsigned)g2 < (unsigned)I2i)
      gi = (g0 * I1i + g1) * I2i + g2;
    double row[M];
    load_coef_row<M>(coef, gi, row);
#pragma unroll
    for (int o = 0; o < M; ++o) cl[o][b] = row[o];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* pl = plds[wave];
  if (lane == 0) pl[64] = 0.0;
  __syncthreads();
  constexpr int NP = (M1 + 1) / 2;
  unsigned nbo[1][NP];
#pragma unroll
  for (int o = 0; o < NP; ++o) {
    const unsigned lo = 8u * (unsigned)nbl[lane * M1 + 2 * o];
    const unsigned hi = 2 * o + 1 < M1 ? 8u * (unsigned)nbl[lane * M1 + 2 * o + 1] : 0u;
    nbo[0][o] = lo | (hi << 16);
  }
  // the lane's node: its offset in the staged box (inbox) or, outside the halo, its grid offset
  int o0 = 0, o1 = 0, o2 = 0;
  const bool valid = lane < T;
  if (valid) o0 = tab_off[3 * lane], o1 = tab_off[3 * lane + 1], o2 = tab_off[3 * lane + 2];
  const bool inbox = valid && abs(o0) <= BT_H && abs(o1) <= BT_H && abs(o2) <= BT_H;
  const int dob = (o0 * BT_B + o1) * BT_B + o2;
  for (int lc = wave; lc < BT_E * BT_E * BT_E; lc += BT_WAVES) {
    const int l0 = lc / (BT_E * BT_E), l1 = lc / BT_E % BT_E, l2 = lc % BT_E;
    const int y0 = t0 + l0, y1 = t1 + l1, y2 = t2 + l2;
    if (y0 >= I0i || y1 >= I1i || y2 >= I2i) continue;  // (whole wave)
    const long long y = ((long long)y0 * I1i + y1) * I2i + y2;
    if (y < c0 || y >= c1) continue;
    double c[1][M];
    if (inbox) {
      const int b = ((l0 + BT_H) * BT_B + (l1 + BT_H)) * BT_B + (l2 + BT_H) + dob;
#pragma unroll
      for (int o = 0; o < M; ++o) c[0][o] = cl[o][b];
    } else {
      int gi = -1;
      const int g0 = y0 + o0, g1 = y1 + o1, g2 = y2 + o2;
      if (valid && (unsigned)g0 < (unsigned)I0i && (unsigned)g1 < (unsigned)I1i &&
          (unsigned)g2 < (unsigned)I2i)
        gi = (g0 * I1i + g1) * I2i + g2;
      load_coef_row<M>(coef, gi, c[0]);
    }
    const double ub = bounds_cg<1, M1>(c, nbo, pl, cntl, K, hi_scale, mu, lane);
    if (lane == 0) qhi[y] = ub;
  }
}

// Round 0 (snippets_a3.py:77-124): A empty, nom = s_yy, denom = 1 / Q_yy - eps (an upper bound of
// the delta where qexact[y] = 0).

// exact_cg_wg_kernel (round 5): the whole CG solve of a column in ONE workgroup of 1,024 threads
// (part A / part B as workgroup phases, their sums workgroup reductions): one launch per batch
// instead of 2 per iteration.  Parity green (75 C4 GPU tests), but one CU per column cannot
// stream the column's late iterations: exact_cg 1.46 -> 4.0 ms per 128^3 run
// (profiles/r5_c4_ab.jsonl, call k).  Constants and launch it used:
//
// constexpr int CG_WG = 1024;
//   hipLaunchKernelGGL(exact_cg_wg_kernel<true>, dim3((unsigned)nb), dim3(CG_WG), 0, s, w, a.I0,
//                      a.I1, a.I2, a.offs, a.m1, radius, slots, centers, cg_iters, tol2);
//
// // The whole CG solve of column j = blockIdx.x in ONE workgroup of CG_WG threads: iteration it's
// // part A (p_it on the fly, q = (S + eps I) p_it, p.q) and part B (x, r, |r|^2) are the per-phase
// // kernels' node arithmetic, their sums workgroup reductions in a fixed order (deterministic), and
// // the barrier inside each reduction orders the phases.  No launch per phase: the batch's columns
// // run side by side on CG_B CUs for all iterations.  The same stopping rule and state as the
// // per-phase kernels (state[0] = 1, state[1] = it when |r_it|^2 <= tol2 at the top of iteration it).
// template <bool OCT>
// __global__ __launch_bounds__(CG_WG) void exact_cg_wg_kernel(ExactWS w, long long I0, long long I1,
//                                                            long long I2, const int* offs, int m1,
//                                                            int srad, const int* slots,
//                                                            const long long* centers, int cg_iters,
//                                                            double tol2) {
//   __shared__ double red[CG_WG / 64];
//   const int j = blockIdx.x;
//   const CGCol cc = cg_col(w, j);
//   if (cc.state[0]) return;  // no candidate in this column of the batch
//   const int slot = slots[j];
//   const long long a = centers[j];
//   double* x = w.Qcols + (size_t)slot * (w.b0 * w.b1 * w.b2);
//   const int m = m1 + 1;
//   const int t = threadIdx.x, lane = t & 63;
//   auto wg_sum = [&](double v) {
//     v = wave_sum(v);
//     if (lane == 0) red[t >> 6] = v;
//     __syncthreads();
//     double tot = 0.0;
// #pragma unroll
//     for (int i = 0; i < CG_WG / 64; ++i) tot += red[i];
//     __syncthreads();
//     return tot;
//   };
//   double rr = cc.rr[0], rr_prev = rr;
//   for (int it = 0; it < cg_iters; ++it) {
//     if (rr <= tol2) {
//       if (t == 0) {
//         cc.state[0] = 1;
//         cc.state[1] = it;
//       }
//       return;
//     }
//     const double beta = it == 0 ? 0.0 : rr / rr_prev;
//     const double* pold = (it & 1) ? cc.p0 : cc.p1;
//     double* pnew = (it & 1) ? cc.p1 : cc.p0;
//     const ActiveCube q = active_cube(w, I1, I2, slot, a, it, srad);
//     double acc = 0.0;
//     auto node_a = [&](long long g0, long long g1, long long g2) {
//       const long long l = ((g0 - q.lo0) * w.b1 + (g1 - q.lo1)) * w.b2 + (g2 - q.lo2);
//       const double pi = it == 0 ? cc.r[l] : fma(beta, pold[l], cc.r[l]);
//       const double* c = w.coef + ((g0 * I1 + g1) * I2 + g2) * coef_stride(m);
//       double s = c[0] * pi;
//       for (int o = 0; o < m1; ++o) {
//         const double cv = c[1 + o];
//         if (cv == 0.0) continue;
//         const long long j0 = g0 + offs[3 * o] - q.lo0, j1 = g1 + offs[3 * o + 1] - q.lo1,
//                         j2 = g2 + offs[3 * o + 2] - q.lo2;
//         if (j0 < 0 || j0 >= w.b0 || j1 < 0 || j1 >= w.b1 || j2 < 0 || j2 >= w.b2) continue;
//         const long long jj = (j0 * w.b1 + j1) * w.b2 + j2;
//         const double pj = it == 0 ? cc.r[jj] : fma(beta, pold[jj], cc.r[jj]);
//         s = fma(cv, pj, s);
//       }
//       pnew[l] = pi;
//       cc.q[l] = s;
//       acc = fma(pi, s, acc);
//     };
//     cg_walk<OCT>(w, q, I0, I1, I2, a, it, t, CG_WG, node_a);
//     const double alpha = rr / wg_sum(acc);
//     acc = 0.0;
//     auto node_b = [&](long long g0, long long g1, long long g2) {
//       const long long l = ((g0 - q.lo0) * w.b1 + (g1 - q.lo1)) * w.b2 + (g2 - q.lo2);
//       x[l] = fma(alpha, pnew[l], x[l]);
//       const double ri = fma(-alpha, cc.q[l], cc.r[l]);
//       cc.r[l] = ri;
//       acc = fma(ri, ri, acc);
//     };
//     cg_walk<OCT>(w, q, I0, I1, I2, a, it, t, CG_WG, node_b);
//     rr_prev = rr;
//     rr = wg_sum(acc);
//     if (t == 0) cc.rr[it + 1] = rr;
//   }
// }

// exact_window_kernel<KIND, STEP = true> (round 5): round r's window kernel at 14 candidates per
// 1,024-thread workgroup whose LAST workgroup (a ticket in ctl[8] after a device-scope fence)
// runs round r + 1's step (step_body, exact_step_kernel's code): one launch per round.  Parity
// green (75 C4 GPU tests), but slower (profiles/r5_c4_ab.jsonl, call m): the 16-wave window
// workgroups alone cost 0.69 -> 0.98 ms per run, the fences and the ticket another 0.14 ms
// (4.04 -> 4.64 ms).  The host loop skipped the standalone step of a round whose step had run
// in the previous window launch.
//
// struct WinSm {
//   RowsLds r;
// };
//
// // STEP: the last workgroup to finish (a ticket in ctl[CTL_TICKET], after a device-scope fence of
// // every workgroup's stores) then runs round + 1's step (step_body) — one launch per round instead
// // of two.  The step's arithmetic is exact_step_kernel's.
// template <int KIND, bool STEP>
// __global__ __launch_bounds__(WIN_T) void exact_window_kernel(EArgs a, const double* __restrict__ qdiag,
//                                                              double* cache, unsigned char* sel,
//                                                              ExactWS w, int round, long long* picks,
//                                                              long long nblk, long long nsb,
//                                                              int nslots, double* pick_delta) {
//   __shared__ typename std::conditional<STEP, StepSm, WinSm>::type sm;
//   __shared__ StagedPicks sp;
//   __shared__ int s_slot, s_last;
//   const long long at = picks[round];
//   if (at < 0) {  // stalled (the step returns at once) or nothing left to pick
//     if constexpr (STEP) {
//       if (blockIdx.x == 0)
//         step_body<KIND>(a, cache, sel, w, nblk, nsb, nslots, round + 1, 0, picks, pick_delta, sm,
//                         s_slot);
//     }
//     return;
//   }
//   const Window v = window_of(a, at);
//   const int nr = round + 1;
//   stage_picks(a, w, picks, nr, sp);
//   if (nr * (nr + 1) <= ROWS_LDS) {
//     const LRows L = stage_rows(w, round, sm.r);
//     __syncthreads();
//     window_tail<KIND>(a, qdiag, cache, sel, w, round, picks, v, sp, L, &sm.r);
//   } else {
//     __syncthreads();
//     window_tail<KIND>(a, qdiag, cache, sel, w, round, picks, v, sp, global_rows(w), nullptr);
//   }
//   if constexpr (STEP) {
//     __threadfence();
//     __syncthreads();
//     if (threadIdx.x == 0) s_last = atomicAdd(w.ctl + CTL_TICKET, 1) == (int)gridDim.x - 1;
//     __syncthreads();
//     if (!s_last) return;
//     __threadfence();
//     if (threadIdx.x == 0) w.ctl[CTL_TICKET] = 0;
//     step_body<KIND>(a, cache, sel, w, nblk, nsb, nslots, round + 1, 0, picks, pick_delta, sm,
//                     s_slot);
//   } else {
//     (void)nblk, (void)nsb, (void)nslots, (void)pick_delta, (void)s_slot, (void)s_last;
//   }
// }

// exact_cg_ab_kernel (round 5): the 7-point CG with one launch per iteration — part B of
// iteration it - 1 and part A of it together, |r_it|^2 from the recurrence
// |r - alpha q|^2 = |r|^2 - 2 alpha r.q + alpha^2 q.q (r and q double-buffered by parity, the
// partials by parity).  WRONG in floating point: the recurrence loses |r|^2 to cancellation once
// the residual is small, beta goes astray and the solve diverges (GPU: column errors ~1e4 on a
// 12 x 11 x 10 grid; the same in numpy: plain CG converges in 24 iterations to 7e-16, the
// recurrence form reaches |r|^2 = 2e9 at the 31-iteration cap).  The stable one-reduction form
// (Chronopoulos-Gear: r.r and w.r by direct sums, w = A r) moves ~30 % more bytes per iteration
// and was slower in round 3.  Not built.
//
// // The 7-point CG with ONE launch per iteration (A/B build VGPOSP_CG_AB=1).  Launch it does, on the
// // walk of radius it + 1: part B of iteration it - 1 at every node (x += alpha p_{it-1},
// // r_it = r_{it-1} - alpha q_{it-1}) and part A of iteration it (p_it = r_it + beta p_{it-1}, formed
// // on the fly at the neighbours from their r_{it-1}, q_{it-1}, p_{it-1}; q_it = (S + eps I) p_it),
// // with the partials of p.q, r.q and q.q.  |r_it|^2 comes from the recurrence
// // |r_{it-1} - alpha q|^2 = |r_{it-1}|^2 - 2 alpha r.q + alpha^2 q.q (no separate |r|^2 pass), so beta
// // and the stopping test are known at the top of the launch.  r and q alternate between two
// // buffers by parity (a node's neighbours still read iteration it - 1's values).  last: the closing
// // launch (it = cg_iters) that applies part B only.  Per element the same fmas as the two-launch
// // kernels; alpha, beta and the stopping test differ by rounding (the recurrence for |r|^2).
// __global__ __launch_bounds__(CG_T) void exact_cg_ab_kernel(ExactWS w, long long I0, long long I1,
//                                                            long long I2, const int* offs,
//                                                            const int* slots,
//                                                            const long long* centers, int it,
//                                                            int np_prev, double tol2, int last) {
//   __shared__ double red[CG_T / 64];
//   const CGCol cc = cg_col(w, blockIdx.y);
//   // converged in an EARLIER launch: state[2 + parity] is written only by block 0 of a launch of
//   // that parity and read only by the next launch (so no block reads a flag its own launch sets)
//   const int cur = it & 1, prv = cur ^ 1;
//   if (centers[blockIdx.y] < 0) return;
//   if (it > 0 && cc.state[2 + prv]) {
//     if (blockIdx.x == 0 && threadIdx.x == 0) cc.state[2 + cur] = 1;
//     return;
//   }
//   double alpha = 0.0, beta = 0.0, rr = cc.rr[0];
//   bool done = last != 0;
//   if (it > 0) {
//     // the previous launch's partials (parity it - 1; this launch writes the other set)
//     const int op = (it - 1) & 1;
//     const double pq = sum_partials(op ? cc.part_rr : cc.part_pq, np_prev, red);
//     const double rq = sum_partials(cc.part_rq + op * CG_BLOCKS, np_prev, red);
//     const double qq = sum_partials(cc.part_qq + op * CG_BLOCKS, np_prev, red);
//     const double rp = cc.rr[it - 1];
//     alpha = rp / pq;
//     rr = fma(alpha, fma(alpha, qq, -2.0 * rq), rp);
//     beta = rr / rp;
//     if (blockIdx.x == 0 && threadIdx.x == 0) cc.rr[it] = rr;
//     if (rr <= tol2) {
//       done = true;
//       if (blockIdx.x == 0 && threadIdx.x == 0) {
//         cc.state[0] = 1;
//         cc.state[1] = it;
//         cc.state[2 + cur] = 1;
//       }
//     }
//   }
//   const int o = prv, nw = cur;
//   const double* ro = o ? cc.r1 : cc.r;
//   const double* qo = o ? cc.q1 : cc.q;
//   const double* po = o ? cc.p1 : cc.p0;
//   double* rn = nw ? cc.r1 : cc.r;
//   double* qn = nw ? cc.q1 : cc.q;
//   double* pn = nw ? cc.p1 : cc.p0;
//   const int slot = slots[blockIdx.y];
//   double* x = w.Qcols + (size_t)slot * (w.b0 * w.b1 * w.b2);
//   const ActiveCube q = active_cube(w, I1, I2, slot, centers[blockIdx.y], it, 1);
//   int od[6][3];
//   long long dl[6];
// #pragma unroll
//   for (int k = 0; k < 6; ++k) {
//     od[k][0] = offs[3 * k];
//     od[k][1] = offs[3 * k + 1];
//     od[k][2] = offs[3 * k + 2];
//     dl[k] = ((long long)od[k][0] * w.b1 + od[k][1]) * w.b2 + od[k][2];
//   }
//   double apq = 0.0, arq = 0.0, aqq = 0.0;
//   auto node = [&](long long g0, long long g1, long long g2) {
//     const long long j0 = g0 - q.lo0, j1 = g1 - q.lo1, j2 = g2 - q.lo2;
//     const long long l = (j0 * w.b1 + j1) * w.b2 + j2;
//     if (it == 0) {  // r_0 = e_c in place, p_0 = r_0
//       const double* c = w.coef + ((g0 * I1 + g1) * I2 + g2) * coef_stride(7);
//       double cv[7], rv[7];
//       bool in[7];
//       in[0] = true;
// #pragma unroll
//       for (int k = 0; k < 6; ++k) {
//         const long long k0 = j0 + od[k][0], k1 = j1 + od[k][1], k2 = j2 + od[k][2];
//         in[1 + k] = k0 >= 0 && k0 < w.b0 && k1 >= 0 && k1 < w.b1 && k2 >= 0 && k2 < w.b2;
//       }
// #pragma unroll
//       for (int k = 0; k < 7; ++k) {
//         cv[k] = c[k];
//         rv[k] = cc.r[k == 0 ? l : (in[k] ? l + dl[k - 1] : l)];
//       }
//       double sq = cv[0] * rv[0];
// #pragma unroll
//       for (int k = 1; k < 7; ++k) sq = fma(cv[k], in[k] ? rv[k] : 0.0, sq);
//       pn[l] = rv[0];
//       qn[l] = sq;
//       apq = fma(rv[0], sq, apq);
//       arq = fma(rv[0], sq, arq);
//       aqq = fma(sq, sq, aqq);
//       return;
//     }
//     const double r_own = fma(-alpha, qo[l], ro[l]);
//     const double p_old = po[l];
//     x[l] = fma(alpha, p_old, x[l]);
//     rn[l] = r_own;
//     if (done) return;
//     const double* c = w.coef + ((g0 * I1 + g1) * I2 + g2) * coef_stride(7);
//     double cv[7], rv[7], qv[7], pv[7];
//     bool in[7];
//     in[0] = true;
// #pragma unroll
//     for (int k = 0; k < 6; ++k) {
//       const long long k0 = j0 + od[k][0], k1 = j1 + od[k][1], k2 = j2 + od[k][2];
//       in[1 + k] = k0 >= 0 && k0 < w.b0 && k1 >= 0 && k1 < w.b1 && k2 >= 0 && k2 < w.b2;
//     }
// #pragma unroll
//     for (int k = 0; k < 7; ++k) cv[k] = c[k];
// #pragma unroll
//     for (int k = 1; k < 7; ++k) {
//       const long long jj = in[k] ? l + dl[k - 1] : l;
//       rv[k] = ro[jj];
//       qv[k] = qo[jj];
//       pv[k] = po[jj];
//     }
//     const double pi = fma(beta, p_old, r_own);
//     double sq = cv[0] * pi;
// #pragma unroll
//     for (int k = 1; k < 7; ++k) {
//       const double pj = fma(beta, pv[k], fma(-alpha, qv[k], rv[k]));
//       sq = fma(cv[k], in[k] ? pj : 0.0, sq);
//     }
//     pn[l] = pi;
//     qn[l] = sq;
//     apq = fma(pi, sq, apq);
//     arq = fma(r_own, sq, arq);
//     aqq = fma(sq, sq, aqq);
//   };
//   cg_walk<true>(w, q, I0, I1, I2, centers[blockIdx.y], min(it, last ? it - 1 : it),
//                 (long long)blockIdx.x * CG_T + threadIdx.x, (long long)gridDim.x * CG_T, node);
//   if (done) return;
//   block_partial(apq, nw ? cc.part_rr : cc.part_pq, red);
//   __syncthreads();  // (red is reused: thread 0 has read it)
//   block_partial(arq, cc.part_rq + nw * CG_BLOCKS, red);
//   __syncthreads();
//   block_partial(aqq, cc.part_qq + nw * CG_BLOCKS, red);
// }
