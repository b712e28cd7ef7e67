// Local-kernel greedy MI placement (config C4: 128^3 = 2,097,152 candidates), never forming Sigma.
//
// The reference's answer to large N is its algorithm 3 (snippets_a3.py:43-364) on the beta-decay
// tapered covariance (main_architecture_2_sampledistribution.py:355-421):
//   s(u, v) = g(|i_u - i_v|) (K(x_u, x_v) + shift [u == v]),  g(d) = exp(-(beta d)^2 / (2 pi)),
//   g < 0.01 -> 0,
// with the epsilon-local deltas its comments name (snippets_a3.py:63, :182-186): conditioning is
// restricted to the taper support N(y) of each candidate,
//   nom_y   = s_yy - s_yB (S_BB + eps I)^-1 s_By,  B = A ∩ N(y)
//   denom_y = s_yy - s_yB (S_BB + eps I)^-1 s_By,  B = N(y) \ A
// (eps = 1e-6, snippets_a2.py:161-163; delta = 0 below 1e-7, :480).  A pick y* then changes only
// the deltas of N(y*), and the reference's window re-score keeps the cache exact.
//
// One candidate = one m x m SPD matrix (its neighbours in C order, y last, excluded neighbours as
// identity rows) whose last Schur complement is the conditional variance.  MM = 8/16/32/64 lanes
// hold one candidate, one matrix ROW per lane (64 / MM candidates per wave64): the entries are
// computed on the fly from X (K is never stored), and the elimination broadcasts column j of the
// trailing matrix lane by lane (v_readlane for one candidate per wave, ds_bpermute for several).
// Everything per candidate stays in VGPRs.
//
// Arg-max: one (value, index) key per 256-entry block of the cache.  After a pick, only the blocks
// its window touched are refreshed (they follow from the pick's grid coordinates), then the block
// keys are reduced: a round reads a few KB, not the 16 MB cache.  Keys order by value, ties by
// LOWER index (placement_algorithm2.py:24-50).
//
// Single rank, small supports (m <= 16, the reference's beta = 4): the whole k-round loop runs in
// ONE persistent workgroup (pick -> window re-score -> block refresh -> arg-max), so a round costs
// no launch at all.  Otherwise (and for the candidate-sharded path, which all-gathers the keys
// between arg-max and pick) a round is a select kernel and a pick+window kernel.
#include <cmath>

#include "common.h"
#include "psd.h"

namespace vgposp {

constexpr int SEL_T = 1024;   // threads of the select kernel
constexpr int ROUNDS_T = 512; // threads of the persistent rounds kernel
constexpr int MAXBLK = 8192;  // block keys held in LDS by the rounds kernel (128 KiB)
constexpr int SBF = 64;       // blocks per superblock

// Two-level arg-max keys: block keys (value, index) over lblk cache entries each, superblock keys
// over SBF blocks.  lblk is the smallest power of two >= 256 with <= MAXBLK blocks per slab.
static int64_t block_len(int64_t nloc) {
  int64_t l = 256;
  while (ceil_div(nloc, l) > MAXBLK) l *= 2;
  return l;
}

struct LocalWS {
  double* bval;      // [nblk]
  long long* bidx;   // [nblk]
  double* sval;      // [nsb]
  long long* sidx;   // [nsb]
  size_t bytes;
};

static size_t lalign(size_t x) { return (x + 255) & ~(size_t)255; }

static LocalWS local_layout(void* base, int64_t nloc) {
  LocalWS w{};
  nloc = std::max<int64_t>(nloc, 1);
  const int64_t nblk = ceil_div(nloc, block_len(nloc)), nsb = ceil_div(nblk, SBF);
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t b) {
    char* r = p ? p + off : nullptr;
    off += lalign(b);
    return r;
  };
  w.bval = (double*)take(nblk * 8);
  w.bidx = (long long*)take(nblk * 8);
  w.sval = (double*)take(nsb * 8);
  w.sidx = (long long*)take(nsb * 8);
  w.bytes = off;
  return w;
}

struct ScoreArgs {
  const double* X;
  long long I0, I1, I2;
  double two_log_amp, inv_ls, inv_ls2, shift, jitter, thr;
  const int* offs;   // [m-1][3]
  int m;
  const double* tau;
  int ntau;
  unsigned char* sel;
  long long c0, c1;
  int cutoff;
  double* cache;
  int* info;
  double* bval;
  long long* bidx;
  double* sval;
  long long* sidx;
  long long lblk, nblk, nsb;
};

// Window [i_d - cutoff, i_d + cutoff) per axis around flat index c (snippets_a3.py:190-303).
struct Win {
  long long lo0, lo1, lo2, w0, w1, w2;
};

__device__ __forceinline__ Win window_of(const ScoreArgs& a, long long c) {
  Win w;
  const long long ci0 = c / (a.I1 * a.I2), ci1 = (c / a.I2) % a.I1, ci2 = c % a.I2;
  w.lo0 = max(ci0 - a.cutoff, 0LL);
  w.lo1 = max(ci1 - a.cutoff, 0LL);
  w.lo2 = max(ci2 - a.cutoff, 0LL);
  w.w0 = max(min(ci0 + a.cutoff, a.I0) - w.lo0, 0LL);
  w.w1 = max(min(ci1 + a.cutoff, a.I1) - w.lo1, 0LL);
  w.w2 = max(min(ci2 + a.cutoff, a.I2) - w.lo2, 0LL);
  return w;
}

// Memory phases inside one workgroup.  __syncthreads() carries workgroup-scope release/acquire,
// which is all the one-workgroup kernels need (their waves share the CU's L1).  An agent-scope
// __threadfence() would be wrong here: on gfx950 it writes back and invalidates this XCD's L2,
// and every later load in the kernel would miss (the select kernel: 35 -> 17 us per round).
__device__ __forceinline__ void sync_phase() { __syncthreads(); }

template <int MM>
__device__ __forceinline__ double bcast(double v, int base, int l) {
  if constexpr (MM == 64) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
  } else {
    return __shfl(v, base + l, 64);
  }
}

template <int MM>
__device__ __forceinline__ int bcast_i(int v, int base, int l) {
  if constexpr (MM == 64) return __builtin_amdgcn_readlane(v, l);
  else return __shfl(v, base + l, 64);
}

// Build this lane's row of the candidate matrix for one pass (inc: this row takes part) and run the
// elimination.  Returns the last Schur complement (meaningful on the y lane, r == MM - 1).
template <int KIND, int MM>
__device__ __forceinline__ double schur_pass(const ScoreArgs& a, int base, int r, bool inc, double x0,
                                             double x1, double x2, int o0, int o1, int o2,
                                             double kdiag, bool isy, bool& bad) {
  double row[MM];
  const int incl = inc ? 1 : 0;
#pragma unroll
  for (int l = 0; l < MM; ++l) {
    const double y0 = bcast<MM>(x0, base, l);
    const double y1 = bcast<MM>(x1, base, l);
    const double y2 = bcast<MM>(x2, base, l);
    const int il = bcast_i<MM>(incl, base, l);
    double v = 0.0;
    if (l == MM - 1 || l < a.m - 1) {
      // offset of row l: the table entry, or 0 for the y row
      const int p0 = (l == MM - 1) ? 0 : a.offs[3 * l + 0];
      const int p1 = (l == MM - 1) ? 0 : a.offs[3 * l + 1];
      const int p2 = (l == MM - 1) ? 0 : a.offs[3 * l + 2];
      const int e0 = o0 - p0, e1 = o1 - p1, e2 = o2 - p2;
      const int d2i = e0 * e0 + e1 * e1 + e2 * e2;
      if (l < r && inc && il && d2i < a.ntau) {
        const double t = a.tau[d2i];
        if (t != 0.0) {
          const double dx0 = x0 - y0, dx1 = x1 - y1, dx2 = x2 - y2;
          const double d2 = dx0 * dx0 + dx1 * dx1 + dx2 * dx2;
          v = t * kfun<KIND>(d2, a.two_log_amp, a.inv_ls, a.inv_ls2);
        }
      }
    }
    if (l == r) v = inc ? (kdiag + a.shift + (isy ? 0.0 : a.jitter)) : 1.0;
    row[l] = v;
  }
  // right-looking elimination of columns 0 .. MM-2; lane r keeps row r of the trailing matrix
#pragma unroll
  for (int j = 0; j < MM - 1; ++j) {
    const double pj = bcast<MM>(row[j], base, j);
    bad |= (r == j) && !(pj > 0.0);
    const double f = row[j] / pj;
#pragma unroll
    for (int l = j + 1; l < MM; ++l) {
      const double alj = bcast<MM>(row[j], base, l);
      row[l] = fma(-f, alj, row[l]);
    }
  }
  return row[MM - 1];
}

// Score candidate y of this lane group (all 64 lanes of the wave must call this together).
// ystar >= 0 is treated as selected in addition to the mask (a pick whose mask byte another
// workgroup may not have written yet).  Writes cache[y - c0] on the group's y lane.
template <int KIND, int MM>
__device__ __forceinline__ void score_group(const ScoreArgs& a, long long y, bool active,
                                            long long ystar) {
  const int lane = threadIdx.x & 63;
  const int r = lane % MM;
  const int base = lane - r;
  const bool ysel = active && (y == ystar || a.sel[y]);
  const bool live = active && !ysel;   // scored candidate (a selected one just gets 0)

  // this lane's row: neighbour r (r < m - 1) or y itself (r == MM - 1); others are padding
  const bool isy = (r == MM - 1);
  int o0 = 0, o1 = 0, o2 = 0;
  bool valid = false;
  long long u = 0;
  if (live) {
    const long long i0 = y / (a.I1 * a.I2), i1 = (y / a.I2) % a.I1, i2 = y % a.I2;
    if (isy) {
      valid = true;
      u = y;
    } else if (r < a.m - 1) {
      o0 = a.offs[3 * r];
      o1 = a.offs[3 * r + 1];
      o2 = a.offs[3 * r + 2];
      const long long j0 = i0 + o0, j1 = i1 + o1, j2 = i2 + o2;
      valid = j0 >= 0 && j0 < a.I0 && j1 >= 0 && j1 < a.I1 && j2 >= 0 && j2 < a.I2;
      u = valid ? (j0 * a.I1 + j1) * a.I2 + j2 : 0;
    }
  }
  double x0 = 0.0, x1 = 0.0, x2 = 0.0;
  if (valid) {
    x0 = a.X[3 * u];
    x1 = a.X[3 * u + 1];
    x2 = a.X[3 * u + 2];
  }
  const bool insel = valid && !isy && (u == ystar || a.sel[u]);
  const double kdiag = kfun<KIND>(0.0, a.two_log_amp, a.inv_ls, a.inv_ls2);
  bool bad = false;

  // denominator: y given the unselected neighbours
  const double den = schur_pass<KIND, MM>(a, base, r, isy ? live : (valid && !insel), x0, x1, x2,
                                         o0, o1, o2, kdiag, isy, bad);
  // nominator: y given the selected neighbours (only waves that have one need the pass)
  double nom = kdiag + a.shift;
  if (__any(insel)) {
    nom = schur_pass<KIND, MM>(a, base, r, isy ? live : insel, x0, x1, x2, o0, o1, o2, kdiag, isy,
                               bad);
  }
  if (isy && live && !(den > 0.0 && nom > 0.0)) bad = true;
  if (isy && active) {
    double d = 0.0;
    if (live) {
      const bool small = fabs(nom) < a.thr || fabs(den) < a.thr;   // snippets_a2.py:480
      d = small ? 0.0 : nom / den;
    }
    a.cache[y - a.c0] = d;
  }
  if (bad && live) atomicOr(a.info, 1);
}

// m <= 8 (the reference's beta = 4 gives the 7-point stencil): one candidate per LANE, its whole
// matrix in registers, no cross-lane traffic.  Row 7 is y; rows m-1 .. 6 are identity padding and
// are skipped (eliminating them is an exact no-op), so the arithmetic is the lane-group path's.
template <int KIND>
__device__ __forceinline__ double schur_thread(const ScoreArgs& a, const double (&px)[8],
                                               const double (&py)[8], const double (&pz)[8],
                                               unsigned inc, double kdiag, bool& bad) {
  double G[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i == 7 || i < a.m - 1) {
      const bool ii = (inc >> i) & 1u;
      const int q0 = (i == 7) ? 0 : a.offs[3 * i], q1 = (i == 7) ? 0 : a.offs[3 * i + 1],
                q2 = (i == 7) ? 0 : a.offs[3 * i + 2];
#pragma unroll
      for (int l = 0; l < i; ++l) {
        double v = 0.0;
        if (l < a.m - 1) {
          const int e0 = q0 - a.offs[3 * l], e1 = q1 - a.offs[3 * l + 1], e2 = q2 - a.offs[3 * l + 2];
          const int d2i = e0 * e0 + e1 * e1 + e2 * e2;
          if (ii && ((inc >> l) & 1u) && d2i < a.ntau) {
            const double t = a.tau[d2i];
            if (t != 0.0) {
              const double dx0 = px[i] - px[l], dx1 = py[i] - py[l], dx2 = pz[i] - pz[l];
              v = t * kfun<KIND>(dx0 * dx0 + dx1 * dx1 + dx2 * dx2, a.two_log_amp, a.inv_ls,
                                 a.inv_ls2);
            }
          }
        }
        G[i][l] = v;
      }
      G[i][i] = ii ? (kdiag + a.shift + (i == 7 ? 0.0 : a.jitter)) : 1.0;
    }
  }
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    if (j < a.m - 1) {
      const double pj = G[j][j];
      bad |= !(pj > 0.0);
#pragma unroll
      for (int i = j + 1; i < 8; ++i) {
        if (i == 7 || i < a.m - 1) {
          const double f = G[i][j] / pj;
#pragma unroll
          for (int l = j + 1; l <= i; ++l) {
            if (l == 7 || l < a.m - 1) G[i][l] = fma(-f, G[l][j], G[i][l]);
          }
        }
      }
    }
  }
  return G[7][7];
}

template <int KIND>
__device__ __forceinline__ void score_thread(const ScoreArgs& a, long long y, bool active,
                                             long long ystar, double* stv = nullptr,
                                             long long* sti = nullptr, int slot = 0) {
  // stv / sti (LDS, optional): the (delta, index) written, index -1 when nothing was scored
  if (sti) sti[slot] = -1;
  if (!active) return;
  const long long i0 = y / (a.I1 * a.I2), i1 = (y / a.I2) % a.I1, i2 = y % a.I2;
  // neighbour indices first (no memory), then every load issued unconditionally (invalid rows read
  // y's own entries) so the 8 points and mask bytes arrive in one memory round
  long long uu[8];
  unsigned valid = 1u << 7;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uu[r] = y;
    if (r < a.m - 1) {
      const long long j0 = i0 + a.offs[3 * r], j1 = i1 + a.offs[3 * r + 1],
                      j2 = i2 + a.offs[3 * r + 2];
      if (j0 >= 0 && j0 < a.I0 && j1 >= 0 && j1 < a.I1 && j2 >= 0 && j2 < a.I2) {
        uu[r] = (j0 * a.I1 + j1) * a.I2 + j2;
        valid |= 1u << r;
      }
    }
  }
  uu[7] = y;
  double px[8], py[8], pz[8];
  unsigned char sb[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    px[r] = a.X[3 * uu[r]];
    py[r] = a.X[3 * uu[r] + 1];
    pz[r] = a.X[3 * uu[r] + 2];
    sb[r] = a.sel[uu[r]];
  }
  if (y == ystar || sb[7]) {   // a selected candidate just gets 0
    a.cache[y - a.c0] = 0.0;
    return;
  }
  if (stv) stv[slot] = 0.0;
  unsigned insel = 0;
#pragma unroll
  for (int r = 0; r < 7; ++r)
    if (((valid >> r) & 1u) && (sb[r] || uu[r] == ystar)) insel |= 1u << r;
  const double kdiag = kfun<KIND>(0.0, a.two_log_amp, a.inv_ls, a.inv_ls2);
  bool bad = false;
  const double den = schur_thread<KIND>(a, px, py, pz, valid & ~insel, kdiag, bad);
  const double nom = insel ? schur_thread<KIND>(a, px, py, pz, insel | (1u << 7), kdiag, bad)
                           : kdiag + a.shift;
  if (!(den > 0.0 && nom > 0.0)) bad = true;
  const bool small = fabs(nom) < a.thr || fabs(den) < a.thr;   // snippets_a2.py:480
  const double d = small ? 0.0 : nom / den;
  a.cache[y - a.c0] = d;
  if (sti) {
    stv[slot] = d;
    sti[slot] = y;
  }
  if (bad) atomicOr(a.info, 1);
}

// One lane group (MM > 8) or one lane (MM == 8) per candidate.
template <int KIND, int MM>
__device__ __forceinline__ void score_one(const ScoreArgs& a, long long y, bool active,
                                          long long ystar) {
  if constexpr (MM == 8) score_thread<KIND>(a, y, active, ystar);
  else score_group<KIND, MM>(a, y, active, ystar);
}

template <int MM>
__host__ __device__ constexpr int per_wave() {
  return MM == 8 ? 64 : 64 / MM;
}
__device__ __forceinline__ int slot_in_wave(int mm) {
  return mm == 8 ? (threadIdx.x & 63) : (threadIdx.x & 63) / mm;
}

// Candidate of window slot s around pick c (y = -1 past the end); active = inside the slab.
__device__ __forceinline__ long long window_slot(const ScoreArgs& a, const Win& w, long long s,
                                                 bool& active) {
  active = false;
  if (s >= w.w0 * w.w1 * w.w2) return -1;
  const long long s0 = s / (w.w1 * w.w2), s1 = (s / w.w2) % w.w1, s2 = s % w.w2;
  const long long y = ((w.lo0 + s0) * a.I1 + w.lo1 + s1) * a.I2 + w.lo2 + s2;
  active = y >= a.c0 && y < a.c1;
  return y;
}

// Best of the gathered keys.
__device__ __forceinline__ void best_key(const long long* keys, int nkeys, double& v, long long& i) {
  v = 0.0;
  i = -1;
  for (int q = 0; q < nkeys; ++q) {
    const double kv = __longlong_as_double(keys[2 * q]);
    const long long ki = keys[2 * q + 1];
    if (key_gt(kv, ki, v, i)) {
      v = kv;
      i = ki;
    }
  }
}

// Record pick i of round rnd: mask byte, picks / pick_delta, cache[i] = 0 on the owner
// (snippets_a3.py:162-168).
__device__ __forceinline__ void apply_pick(const ScoreArgs& a, long long i, double v, int rnd,
                                           long long* picks, double* pick_delta) {
  picks[rnd] = i;
  if (pick_delta) pick_delta[rnd] = v;
  if (i >= 0) {
    a.sel[i] = 1;
    if (i >= a.c0 && i < a.c1) a.cache[i - a.c0] = 0.0;
  }
}

// Key of block b: one wave over its lblk cache entries, 4 x 64 entries per memory round (all
// loads issued before any is consumed).
__device__ __forceinline__ void block_key(const ScoreArgs& a, long long b, double& v, long long& i) {
  const int lane = threadIdx.x & 63;
  const long long nloc = a.c1 - a.c0;
  v = 0.0;
  i = -1;
  for (long long q = 0; q < a.lblk; q += 256) {
    unsigned char sb[4];
    double cv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const long long e = b * a.lblk + q + 64 * t + lane;
      const bool in = e < nloc;
      sb[t] = in ? a.sel[a.c0 + (in ? e : 0)] : 1;
      cv[t] = in ? a.cache[in ? e : 0] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const long long e = b * a.lblk + q + 64 * t + lane;
      if (!sb[t] && key_gt(cv[t], a.c0 + e, v, i)) {
        v = cv[t];
        i = a.c0 + e;
      }
    }
  }
  wave_keymax(v, i);
}

// Key of superblock sb: one wave over its block keys (from `bv/bi`, global or LDS).
__device__ __forceinline__ void super_key(const ScoreArgs& a, const double* bv, const long long* bi,
                                          long long sb, double& v, long long& i) {
  const long long b = sb * SBF + (threadIdx.x & 63);
  v = 0.0;
  i = -1;
  if (b < a.nblk) {
    v = bv[b];
    i = bi[b];
  }
  wave_keymax(v, i);
}

// The distinct blocks the pick p and its window [i_d - cutoff, i_d + cutoff) touched, collected
// into an LDS list (a workgroup call; `bits` is an LDS bitmap over the blocks, clear on entry and
// on exit).  One thread per window row segment (plus one for the pick itself).
constexpr int TOUCH_MAX = 1024;

// Phase timestamps of the persistent rounds kernel (wall clock, 100 MHz) for rounds 1..7, in a
// -DVGPOSP_LOCAL_TIMING build only (tools/bench_c4.py reads them through
// vgposp_local_debug_times, which is not part of the ABI).
#ifdef VGPOSP_LOCAL_TIMING
__device__ long long g_local_t[8][8];
#define VG_T(r, ph) \
  if (threadIdx.x == 0 && (r) > 0 && (r) < 8) g_local_t[r][ph] = wall_clock64()
#else
#define VG_T(r, ph)
#endif

__device__ int collect_touched(const ScoreArgs& a, long long p, int* list, int* cnt,
                               unsigned* bits) {
  if (threadIdx.x == 0) *cnt = 0;
  __syncthreads();
  const Win w = window_of(a, p);
  const long long rows = w.w0 * w.w1;
  for (long long q = threadIdx.x; q <= rows; q += blockDim.x) {
    long long s, e;
    if (q == rows) {   // the pick itself (its window is empty when cutoff = 0)
      s = p;
      e = p + 1;
    } else {
      const long long j0 = w.lo0 + q / w.w1, j1 = w.lo1 + q % w.w1;
      s = (j0 * a.I1 + j1) * a.I2 + w.lo2;
      e = s + w.w2;
    }
    s = max(s, a.c0);
    e = min(e, a.c1);
    if (s >= e) continue;
    for (long long b = (s - a.c0) / a.lblk; b <= (e - 1 - a.c0) / a.lblk; ++b) {
      const unsigned m = 1u << (b & 31);
      if (!(atomicOr(&bits[b >> 5], m) & m)) {
        const int slot = atomicAdd(cnt, 1);
        if (slot < TOUCH_MAX) list[slot] = (int)b;
      }
    }
  }
  __syncthreads();
  const int n = min(*cnt, TOUCH_MAX);
  for (int q = threadIdx.x; q < n; q += blockDim.x) bits[list[q] >> 5] = 0u;
  __syncthreads();
  return n;
}

__device__ __forceinline__ bool in_window(const ScoreArgs& a, const Win& w, long long e) {
  const long long e0 = e / (a.I1 * a.I2), e1 = (e / a.I2) % a.I1, e2 = e % a.I2;
  return e0 >= w.lo0 && e0 < w.lo0 + w.w0 && e1 >= w.lo1 && e1 < w.lo1 + w.w1 && e2 >= w.lo2 &&
         e2 < w.lo2 + w.w2;
}

// New key of a block the pick p and its window touched (one wave).  Only window entries changed:
// unless the old best was one of them (or p), the new key is the old one combined with the
// re-scored entries inside the block, which are recent writes; otherwise the block is re-read.
__device__ void touched_key(const ScoreArgs& a, long long p, long long b, double ov, long long oi,
                            double& v, long long& i) {
  const Win w = window_of(a, p);
  if (oi < 0 || oi == p || in_window(a, w, oi)) {
    block_key(a, b, v, i);
    return;
  }
  v = ov;
  i = oi;
  const long long lo = a.c0 + b * a.lblk, hi = min(lo + a.lblk, a.c1);
  const long long rows = w.w0 * w.w1;
  for (long long q = threadIdx.x & 63; q < rows; q += 64) {
    const long long j0 = w.lo0 + q / w.w1, j1 = w.lo1 + q % w.w1;
    const long long s = max((j0 * a.I1 + j1) * a.I2 + w.lo2, lo);
    const long long e = min((j0 * a.I1 + j1) * a.I2 + w.lo2 + w.w2, hi);
    for (long long x0 = s; x0 < e; x0 += 8) {
      unsigned char sb[8];
      double cv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const long long x = min(x0 + t, e - 1);
        sb[t] = a.sel[x];
        cv[t] = a.cache[x - a.c0];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (x0 + t < e && !sb[t] && key_gt(cv[t], x0 + t, v, i)) {
          v = cv[t];
          i = x0 + t;
        }
    }
  }
  wave_keymax(v, i);
}

// Distinct superblocks of the touched-block list (a workgroup call; sbits clear on entry/exit).
__device__ int collect_supers(const int* list, int n, int* slist, int* scnt, unsigned* sbits) {
  if (threadIdx.x == 0) *scnt = 0;
  __syncthreads();
  for (int q = threadIdx.x; q < n; q += blockDim.x) {
    const int sb = list[q] / SBF;
    const unsigned m = 1u << (sb & 31);
    if (!(atomicOr(&sbits[sb >> 5], m) & m)) slist[atomicAdd(scnt, 1)] = sb;
  }
  __syncthreads();
  const int ns = *scnt;
  for (int q = threadIdx.x; q < ns; q += blockDim.x) sbits[slist[q] >> 5] = 0u;
  __syncthreads();
  return ns;
}

__device__ __forceinline__ void wg_reduce_key(double& v, long long& i, double* sv, long long* si) {
  wave_keymax(v, i);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = v;
    si[w] = i;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int nw = blockDim.x >> 6;
    v = threadIdx.x < nw ? sv[threadIdx.x] : 0.0;
    i = threadIdx.x < nw ? si[threadIdx.x] : -1;
    wave_keymax(v, i);
  }
  __syncthreads();
}

// Reduce n keys (global or LDS); the result is valid on thread 0.
__device__ __forceinline__ void reduce_keys(const double* kv, const long long* ki, long long n,
                                            double& v, long long& i, double* sv, long long* si) {
  v = 0.0;
  i = -1;
  for (long long b = threadIdx.x; b < n; b += blockDim.x) {
    if (key_gt(kv[b], ki[b], v, i)) {
      v = kv[b];
      i = ki[b];
    }
  }
  wg_reduce_key(v, i, sv, si);
}

// ---- kernels ---------------------------------------------------------------------------------

// Round 0: score every candidate of the slab.
template <int KIND, int MM>
__global__ __launch_bounds__(256) void local_score_kernel(ScoreArgs a) {
  constexpr int G = per_wave<MM>();
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long y = a.c0 + wave * G + slot_in_wave(MM);
  score_one<KIND, MM>(a, y, y < a.c1, -1);
}

// All block and superblock keys (after the full pass): one workgroup per superblock.
__global__ __launch_bounds__(256) void local_blockmax_kernel(ScoreArgs a) {
  __shared__ double bv[SBF];
  __shared__ long long bi[SBF];
  const long long sb = blockIdx.x;
  const int wave = threadIdx.x >> 6;
  for (int q = wave; q < SBF; q += 4) {
    const long long b = sb * SBF + q;
    double v = 0.0;
    long long i = -1;
    if (b < a.nblk) block_key(a, b, v, i);
    if ((threadIdx.x & 63) == 0) {
      bv[q] = v;
      bi[q] = i;
      if (b < a.nblk) {
        a.bval[b] = v;
        a.bidx[b] = i;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    double v = bv[threadIdx.x];
    long long i = bi[threadIdx.x];
    wave_keymax(v, i);
    if (threadIdx.x == 0) {
      a.sval[sb] = v;
      a.sidx[sb] = i;
    }
  }
}

// Arg-max of the slab after round rnd - 1's pick + window (rnd = 0: after the full pass):
// refresh the touched blocks, then their superblocks, then reduce the superblock keys.
__global__ __launch_bounds__(SEL_T) void local_select_kernel(ScoreArgs a, const long long* picks,
                                                             int rnd, long long* key_out) {
  __shared__ double sv[SEL_T / 64];
  __shared__ long long si[SEL_T / 64];
  __shared__ int list[TOUCH_MAX];
  __shared__ int slist[MAXBLK / SBF];
  __shared__ int cnt, scnt;
  __shared__ unsigned bits[MAXBLK / 32];
  __shared__ unsigned sbits[MAXBLK / SBF / 32];
  const int wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  if (rnd > 0 && picks[rnd - 1] >= 0) {
    for (int q = threadIdx.x; q < MAXBLK / 32; q += blockDim.x) bits[q] = 0u;
    if (threadIdx.x < MAXBLK / SBF / 32) sbits[threadIdx.x] = 0u;
    __syncthreads();
    const long long p = picks[rnd - 1];
    const int n = collect_touched(a, p, list, &cnt, bits);
    for (int q = wave; q < n; q += nwave) {
      const long long b = list[q];
      double v;
      long long i;
      touched_key(a, p, b, a.bval[b], a.bidx[b], v, i);
      if ((threadIdx.x & 63) == 0) {
        a.bval[b] = v;
        a.bidx[b] = i;
      }
    }
    sync_phase();
    const int ns = collect_supers(list, n, slist, &scnt, sbits);
    for (int q = wave; q < ns; q += nwave) {
      double v;
      long long i;
      super_key(a, a.bval, a.bidx, slist[q], v, i);
      if ((threadIdx.x & 63) == 0) {
        a.sval[slist[q]] = v;
        a.sidx[slist[q]] = i;
      }
    }
    sync_phase();
  }
  double v;
  long long i;
  reduce_keys(a.sval, a.sidx, a.nsb, v, i, sv, si);
  if (threadIdx.x == 0) {
    key_out[0] = __double_as_longlong(v);
    key_out[1] = i;
  }
}

// Pick of round rnd from the gathered keys (every workgroup derives it; workgroup 0 records it),
// then the window re-score around it unless do_window = 0.
template <int KIND, int MM>
__global__ __launch_bounds__(256) void local_pick_window_kernel(ScoreArgs a, const long long* keys,
                                                                int nkeys, int rnd, int do_window,
                                                                long long* picks,
                                                                double* pick_delta) {
  constexpr int G = per_wave<MM>();
  double v;
  long long ys;
  best_key(keys, nkeys, v, ys);
  if (blockIdx.x == 0 && threadIdx.x == 0) apply_pick(a, ys, v, rnd, picks, pick_delta);
  if (!do_window || ys < 0) return;
  const Win w = window_of(a, ys);
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  bool active;
  const long long y = window_slot(a, w, wave * G + slot_in_wave(MM), active);
  score_one<KIND, MM>(a, y, active, ys);
}

// Single rank, m <= 8, cutoff <= RW_MAX: the whole loop in one workgroup.  Rounds 0 .. k-1 of
// arg-max -> pick -> window re-score, with the block / superblock keys, the taper tables and the
// re-scored window entries resident in LDS: a touched block's key is the old one combined with the
// staged window entries (no memory traffic) unless its old best was re-scored, and only those
// blocks (usually just the pick's) are re-read.
constexpr int RW_MAX = 5;
constexpr int STAGE = 8 * RW_MAX * RW_MAX * RW_MAX;

template <int KIND>
__global__ __launch_bounds__(ROUNDS_T) void local_rounds_kernel(ScoreArgs a, int k, long long* picks,
                                                                double* pick_delta) {
  __shared__ double lbv[MAXBLK];
  __shared__ long long lbi[MAXBLK];
  __shared__ double lsv[MAXBLK / SBF];
  __shared__ long long lsi[MAXBLK / SBF];
  __shared__ double stv[STAGE];
  __shared__ long long sti[STAGE];
  __shared__ int soffs[3 * 7];
  __shared__ double stau[64];
  __shared__ long long s_pick;
  __shared__ int list[TOUCH_MAX];
  __shared__ int flist[TOUCH_MAX];
  __shared__ int slist[MAXBLK / SBF];
  __shared__ int cnt, scnt, fcnt;
  __shared__ unsigned bits[MAXBLK / 32];
  __shared__ unsigned sbits[MAXBLK / SBF / 32];
  const int wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  for (int q = threadIdx.x; q < MAXBLK / 32; q += blockDim.x) bits[q] = 0u;
  if (threadIdx.x < MAXBLK / SBF / 32) sbits[threadIdx.x] = 0u;
  if (threadIdx.x < 3 * (a.m - 1)) soffs[threadIdx.x] = a.offs[threadIdx.x];
  if (threadIdx.x < a.ntau && threadIdx.x < 64) stau[threadIdx.x] = a.tau[threadIdx.x];
  for (long long b = threadIdx.x; b < a.nblk; b += blockDim.x) {
    lbv[b] = a.bval[b];
    lbi[b] = a.bidx[b];
  }
  for (long long b = threadIdx.x; b < a.nsb; b += blockDim.x) {
    lsv[b] = a.sval[b];
    lsi[b] = a.sidx[b];
  }
  __syncthreads();
  ScoreArgs la = a;   // taper tables from LDS
  la.offs = soffs;
  la.tau = stau;
  la.ntau = min(a.ntau, 64);
  long long nw = 0;
  for (int rnd = 0; rnd < k; ++rnd) {
    VG_T(rnd, 0);
    if (rnd > 0) {
      const long long p = s_pick;
      const Win w = window_of(a, p);
      const int n = collect_touched(a, p, list, &cnt, bits);
      if (threadIdx.x == 0) fcnt = 0;
      __syncthreads();
      VG_T(rnd, 1);
      for (int q = wave; q < n; q += nwave) {   // one wave per touched block
        const long long b = list[q];
        double v = lbv[b];
        long long i = lbi[b];
        if (i < 0 || i == p || in_window(a, w, i)) {
          if ((threadIdx.x & 63) == 0) flist[atomicAdd(&fcnt, 1)] = (int)b;   // re-read it
        } else {
          const long long lo = a.c0 + b * a.lblk, hi = min(lo + a.lblk, a.c1);
          for (long long s = threadIdx.x & 63; s < nw; s += 64) {
            const long long si = sti[s];
            const double sv = stv[s];
            if (si >= lo && si < hi && key_gt(sv, si, v, i)) {
              v = sv;
              i = si;
            }
          }
          wave_keymax(v, i);
          if ((threadIdx.x & 63) == 0) {
            lbv[b] = v;
            lbi[b] = i;
          }
        }
      }
      __syncthreads();
      for (int q = wave; q < fcnt; q += nwave) {
        double v;
        long long i;
        block_key(a, flist[q], v, i);
        if ((threadIdx.x & 63) == 0) {
          lbv[flist[q]] = v;
          lbi[flist[q]] = i;
        }
      }
      __syncthreads();
      VG_T(rnd, 2);
      const int ns = collect_supers(list, n, slist, &scnt, sbits);
      for (int q = wave; q < ns; q += nwave) {
        double v;
        long long i;
        super_key(a, lbv, lbi, slist[q], v, i);
        if ((threadIdx.x & 63) == 0) {
          lsv[slist[q]] = v;
          lsi[slist[q]] = i;
        }
      }
      __syncthreads();
    }
    double v;
    long long ys;
    VG_T(rnd, 3);
    if (wave == 0) {   // one wave reduces the superblock keys (no barrier inside)
      v = 0.0;
      ys = -1;
      for (long long b = threadIdx.x; b < a.nsb; b += 64)
        if (key_gt(lsv[b], lsi[b], v, ys)) {
          v = lsv[b];
          ys = lsi[b];
        }
      wave_keymax(v, ys);
    }
    VG_T(rnd, 4);
    if (threadIdx.x == 0) {
      apply_pick(a, ys, v, rnd, picks, pick_delta);
      s_pick = ys;
    }
    sync_phase();
    VG_T(rnd, 5);
    ys = s_pick;
    if (ys < 0) break;   // nothing left to pick (k > N)
    if (rnd == k - 1) break;
    const Win w = window_of(a, ys);
    nw = w.w0 * w.w1 * w.w2;
    for (long long s0 = 0; s0 < nw; s0 += blockDim.x) {
      bool active;
      const long long slot = s0 + threadIdx.x;
      const long long y = window_slot(a, w, slot, active);
      if (slot < nw) score_thread<KIND>(la, y, active, ys, stv, sti, (int)slot);
    }
    VG_T(rnd, 6);
    sync_phase();
    VG_T(rnd, 7);
  }
}

template <int KIND, int MM>
static void launch_full(const ScoreArgs& a, hipStream_t s) {
  constexpr int G = per_wave<MM>();
  const long long blocks = ceil_div(ceil_div(a.c1 - a.c0, G), 4);
  hipLaunchKernelGGL((local_score_kernel<KIND, MM>), dim3((unsigned)blocks), dim3(256), 0, s, a);
}

template <int KIND, int MM>
static void launch_pick_window(const ScoreArgs& a, const long long* keys, int nkeys, int rnd,
                               int do_window, long long* picks, double* pick_delta, hipStream_t s) {
  constexpr int G = per_wave<MM>();
  const long long nw = (long long)(2 * a.cutoff) * (2 * a.cutoff) * (2 * a.cutoff);
  const long long blocks = do_window ? std::max<long long>(1, ceil_div(ceil_div(nw, G), 4)) : 1;
  hipLaunchKernelGGL((local_pick_window_kernel<KIND, MM>), dim3((unsigned)blocks), dim3(256), 0, s,
                     a, keys, nkeys, rnd, do_window, picks, pick_delta);
}

template <int KIND>
static void launch_rounds(const ScoreArgs& a, int k, long long* picks, double* pick_delta,
                          hipStream_t s) {
  hipLaunchKernelGGL((local_rounds_kernel<KIND>), dim3(1), dim3(ROUNDS_T), 0, s, a, k, picks,
                     pick_delta);
}

// Dispatch on the kernel family and the lane-group width.
template <template <int, int> class F, typename... Args>
static void dispatch(int kind, int m, Args... args) {
#define VG_MM(KIND)                                  \
  if (m <= 8) F<KIND, 8>::run(args...);              \
  else if (m <= 16) F<KIND, 16>::run(args...);       \
  else if (m <= 32) F<KIND, 32>::run(args...);       \
  else F<KIND, 64>::run(args...);
  switch (kind) {
    case VGPOSP_KERNEL_EQ: { VG_MM(VGPOSP_KERNEL_EQ) } break;
    case VGPOSP_KERNEL_MATERN12: { VG_MM(VGPOSP_KERNEL_MATERN12) } break;
    case VGPOSP_KERNEL_MATERN32: { VG_MM(VGPOSP_KERNEL_MATERN32) } break;
    default: { VG_MM(VGPOSP_KERNEL_MATERN52) } break;
  }
#undef VG_MM
}

template <int KIND, int MM>
struct FullF {
  static void run(const ScoreArgs& a, hipStream_t s) { launch_full<KIND, MM>(a, s); }
};
template <int KIND, int MM>
struct PickWindowF {
  static void run(const ScoreArgs& a, const long long* keys, int nkeys, int rnd, int do_window,
                  long long* picks, double* pick_delta, hipStream_t s) {
    launch_pick_window<KIND, MM>(a, keys, nkeys, rnd, do_window, picks, pick_delta, s);
  }
};
template <int KIND, int MM>
struct RoundsF {
  static void run(const ScoreArgs& a, int k, long long* picks, double* pick_delta, hipStream_t s) {
    if constexpr (MM == 8) launch_rounds<KIND>(a, k, picks, pick_delta, s);
  }
};

static int make_args(ScoreArgs& a, int kind, const double* X, int64_t I0, int64_t I1, int64_t I2,
                     double amp, double ls, double diag_shift, double jitter, double threshold,
                     const int* offsets, int m, const double* tau, int ntau, uint8_t* selected,
                     int64_t c0, int64_t c1, int cutoff, double* cache, int* info, void* ws,
                     size_t ws_bytes) {
  VG_CHECK_ARG(kind >= 0 && kind <= 3, 1);
  VG_CHECK_ARG(X != nullptr, 2);
  VG_CHECK_ARG(I0 > 0 && I1 > 0 && I2 > 0, 3);
  VG_CHECK_ARG(amp > 0.0, 6);
  VG_CHECK_ARG(ls > 0.0, 7);
  VG_CHECK_ARG(m >= 1 && m <= 64 && (m == 1 || offsets != nullptr), 12);
  VG_CHECK_ARG(tau != nullptr && ntau >= 1, 13);
  VG_CHECK_ARG(selected != nullptr, 15);
  VG_CHECK_ARG(c0 >= 0 && c1 > c0 && c1 <= I0 * I1 * I2, 17);
  VG_CHECK_ARG(cutoff >= 0 && 4LL * cutoff * cutoff < TOUCH_MAX / 2, 18);
  VG_CHECK_ARG(cache != nullptr, 19);
  VG_CHECK_ARG(info != nullptr, 20);
  LocalWS w = local_layout(ws, c1 - c0);
  if (!ws || ws_bytes < w.bytes) {
    set_error("local greedy: workspace %zu < %zu bytes", ws_bytes, w.bytes);
    return VGPOSP_E_WS;
  }
  a = ScoreArgs{};
  a.X = X;
  a.I0 = I0;
  a.I1 = I1;
  a.I2 = I2;
  a.two_log_amp = 2.0 * std::log(amp);
  a.inv_ls = 1.0 / ls;
  a.inv_ls2 = 1.0 / (ls * ls);
  a.shift = diag_shift;
  a.jitter = jitter;
  a.thr = threshold;
  a.offs = offsets;
  a.m = m;
  a.tau = tau;
  a.ntau = ntau;
  a.sel = selected;
  a.c0 = c0;
  a.c1 = c1;
  a.cutoff = cutoff;
  a.cache = cache;
  a.info = info;
  a.bval = w.bval;
  a.bidx = w.bidx;
  a.sval = w.sval;
  a.sidx = w.sidx;
  a.lblk = block_len(c1 - c0);
  a.nblk = ceil_div(c1 - c0, a.lblk);
  a.nsb = ceil_div(a.nblk, SBF);
  return 0;
}

static int full_pass(const ScoreArgs& a, int kind, hipStream_t s) {
  {
    ProfScope ps("local_score", s, 0.0, 8.0 * (double)(a.c1 - a.c0));
    dispatch<FullF>(kind, a.m, a, s);
    VG_LAUNCH_CHECK();
  }
  ProfScope ps("local_blockmax", s, 0.0, 9.0 * (double)(a.c1 - a.c0));
  hipLaunchKernelGGL(local_blockmax_kernel, dim3((unsigned)a.nsb), dim3(256), 0, s, a);
  VG_LAUNCH_CHECK();
  return 0;
}

}  // namespace vgposp

using namespace vgposp;

#define VG_LOCAL_ARGS                                                                         \
  int kind, const double *X, int64_t I0, int64_t I1, int64_t I2, double amp, double ls,       \
      double diag_shift, double jitter, double threshold, const int *offsets, int m,          \
      const double *tau, int ntau, uint8_t *selected, int64_t c0, int64_t c1, int cutoff,     \
      double *cache, int *info, void *ws, size_t ws_bytes
#define VG_LOCAL_PASS                                                                          \
  kind, X, I0, I1, I2, amp, ls, diag_shift, jitter, threshold, offsets, m, tau, ntau, selected, \
      c0, c1, cutoff, cache, info, ws, ws_bytes

extern "C" size_t vgposp_local_workspace_bytes(int64_t n_local) {
  return local_layout(nullptr, n_local).bytes;
}

extern "C" int vgposp_local_score(VG_LOCAL_ARGS, void* stream) {
  clear_error();
  ScoreArgs a;
  if (int rc = make_args(a, VG_LOCAL_PASS)) return rc;
  return full_pass(a, kind, as_stream(stream));
}

extern "C" int vgposp_local_select(VG_LOCAL_ARGS, const int64_t* picks, int round, int64_t* key_out,
                                   void* stream) {
  clear_error();
  ScoreArgs a;
  if (int rc = make_args(a, VG_LOCAL_PASS)) return rc;
  VG_CHECK_ARG(round == 0 || picks != nullptr, 23);
  VG_CHECK_ARG(round >= 0, 24);
  VG_CHECK_ARG(key_out != nullptr, 25);
  hipStream_t s = as_stream(stream);
  ProfScope ps("local_select", s, 0.0, 0.0);
  hipLaunchKernelGGL(local_select_kernel, dim3(1), dim3(SEL_T), 0, s, a,
                     reinterpret_cast<const long long*>(picks), round,
                     reinterpret_cast<long long*>(key_out));
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_local_pick(VG_LOCAL_ARGS, const int64_t* keys, int nkeys, int round,
                                 int do_window, int64_t* picks, double* pick_delta, void* stream) {
  clear_error();
  ScoreArgs a;
  if (int rc = make_args(a, VG_LOCAL_PASS)) return rc;
  VG_CHECK_ARG(keys != nullptr, 23);
  VG_CHECK_ARG(nkeys >= 1, 24);
  VG_CHECK_ARG(round >= 0, 25);
  VG_CHECK_ARG(picks != nullptr, 27);
  hipStream_t s = as_stream(stream);
  ProfScope ps(do_window ? "local_window" : "local_pick", s, 0.0, 0.0);
  dispatch<PickWindowF>(kind, m, a, reinterpret_cast<const long long*>(keys), nkeys, round,
                        do_window, reinterpret_cast<long long*>(picks), pick_delta, s);
  VG_LAUNCH_CHECK();
  return 0;
}

extern "C" int vgposp_local_run(VG_LOCAL_ARGS, int k, int64_t* picks, double* pick_delta,
                                int64_t* keys, void* stream) {
  clear_error();
  ScoreArgs a;
  if (int rc = make_args(a, VG_LOCAL_PASS)) return rc;
  VG_CHECK_ARG(k >= 1, 23);
  VG_CHECK_ARG(picks != nullptr, 24);
  VG_CHECK_ARG(keys != nullptr, 26);
  hipStream_t s = as_stream(stream);
  if (int rc = full_pass(a, kind, s)) return rc;
  if (m <= 8 && cutoff <= RW_MAX && ceil_div(c1 - c0, 256) <= MAXBLK) {
    ProfScope ps("local_rounds", s, 0.0, 0.0);
    dispatch<RoundsF>(kind, m, a, k, reinterpret_cast<long long*>(picks), pick_delta, s);
    VG_LAUNCH_CHECK();
    return 0;
  }
  for (int r = 0; r < k; ++r) {
    if (int rc = vgposp_local_select(VG_LOCAL_PASS, picks, r, keys, stream)) return rc;
    if (int rc = vgposp_local_pick(VG_LOCAL_PASS, keys, 1, r, r < k - 1, picks, pick_delta, stream))
      return rc;
  }
  return 0;
}

#ifdef VGPOSP_LOCAL_TIMING
extern "C" int vgposp_local_debug_times(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_local_t), sizeof(g_local_t)) == hipSuccess ? 0 : -1;
}
#endif
