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
