// VARIANT (round 6): the product gemm.hip with 8-deep K-tiles in a 4-stage LDS ring (same
// 64 KiB per workgroup, two workgroups per CU); generated from gemm.hip, see DESIGN.md §4.
// fp64 GEMM on CDNA4 matrix cores (v_mfma_f64_16x16x4f64), the dense contraction behind the
// Cholesky trailing update, the fused block Gauss-Jordan inverse and C^-1 = M^T M formation.
//
//   C = alpha * op(A) * op(B) + beta * C        (row-major, fp64)
//
// Three kernels share the 128x128x16 tile geometry (4 waves in a 2x2 grid, 64x64 = 4x4 MFMA
// fragments per wave):
//   gemm_glds_kernel (default)  LDS-DMA staging (global_load_lds), 2-stage ring, 2 WG per CU,
//                               XOR-swizzled lane-linear LDS images; described above the kernel.
//   gemm_rs_kernel (opt-in)     one wave per SIMD, register-staged, 256 AGPR accumulators.
//   gemm_ref_kernel (fallback)  odd sizes / unaligned operands: register staging into padded
//                               images, bank-conflict-free for the fragment reads (lane l reads
//                               row l&15, k = l>>4):
//     KC image [row][k] with a row pitch of 18 doubles   (operand stored k-contiguous)
//     MC image [k][row] with a row pitch of 144 doubles  (operand stored row-contiguous)
// No operand ever needs an explicit transpose in HBM.
#include <algorithm>
#include <atomic>
#include <type_traits>

#include "common.h"

namespace vgposp {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef unsigned int v2u32_t __attribute__((ext_vector_type(2)));

constexpr int GBM = 128;
constexpr int GBN = 128;
constexpr int GBK = 16;
constexpr int KC_PITCH = GBK + 2;    // 18 doubles
constexpr int MC_PITCH = GBM + 16;   // 144 doubles
constexpr int TILE_ELEMS = GBM * KC_PITCH;  // == GBK * MC_PITCH == 2304 doubles
static_assert(GBM * KC_PITCH == GBK * MC_PITCH, "LDS images must be the same size");

struct GemmParams {
  int64_t m, n, k;
  double alpha, beta;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  double* C;
  int64_t ldc;
  int uplo_c, tri_a, tri_b;
  // split-K: nsplit > 1 launches nblk * nsplit workgroups; split z covers K range
  // [z * kchunk, (z + 1) * kchunk) and writes alpha * partial to part + z * m * n (ld n)
  int nsplit, nblk;
  int64_t kchunk;
  double* part;
  // batch (grid.y of the fast kernel, grid.z of the reference kernel): element b reads
  // A + b sA, B + b sB and writes C + b sC (split-K partials at part + b sP)
  int64_t sA, sB, sC, sP;
  // device abort flag (a failed pivot of the enclosing factorization): non-zero -> the launch
  // does nothing (vgposp_greedy_init's early stop without a host synchronisation)
  const int* abort;
};

// Set by a factorization for the GEMMs it launches from this thread (gemm_abort_scope).
thread_local const int* tl_gemm_abort = nullptr;

// Stage one operand tile (128 rows of the M/N dimension x 16 of K) into registers.
//   KC: stored[row][k] (row = M/N index), MC: stored[k][row].
// tri: the stored matrix is lower triangular (entries with column > row read as 0).
template <bool KC>
__device__ __forceinline__ void load_tile(const double* __restrict__ base, int64_t ld, int64_t r0,
                                          int64_t k0, int64_t R, int64_t K, bool tri, bool vec,
                                          double2 (&reg)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int e = t + 256 * it;
    int64_t gr, gk;
    if (KC) {
      gr = r0 + (e >> 3);
      gk = k0 + (e & 7) * 2;
    } else {
      gk = k0 + (e >> 6);
      gr = r0 + (e & 63) * 2;
    }
    double2 v = make_double2(0.0, 0.0);
    if (KC) {
      // elements (gr, gk) and (gr, gk+1) of stored[row][k]
      const double* p = base + gr * ld + gk;
      if (gr < R) {
        if (vec && gk + 1 < K) {
          v = *reinterpret_cast<const double2*>(p);
        } else {
          if (gk < K) v.x = p[0];
          if (gk + 1 < K) v.y = p[1];
        }
        if (tri) {
          if (gk > gr) v.x = 0.0;
          if (gk + 1 > gr) v.y = 0.0;
        }
      }
    } else {
      // elements (gk, gr) and (gk, gr+1) of stored[k][row]
      const double* p = base + gk * ld + gr;
      if (gk < K) {
        if (vec && gr + 1 < R) {
          v = *reinterpret_cast<const double2*>(p);
        } else {
          if (gr < R) v.x = p[0];
          if (gr + 1 < R) v.y = p[1];
        }
        if (tri) {
          if (gr > gk) v.x = 0.0;
          if (gr + 1 > gk) v.y = 0.0;
        }
      }
    }
    reg[it] = v;
  }
}

template <bool KC>
__device__ __forceinline__ void store_tile(double* lds, const double2 (&reg)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int e = t + 256 * it;
    int off;
    if (KC) off = (e >> 3) * KC_PITCH + (e & 7) * 2;
    else off = (e >> 6) * MC_PITCH + (e & 63) * 2;
    *reinterpret_cast<double2*>(lds + off) = reg[it];
  }
}

// Fragment read: element (row, k) of the staged tile.
template <bool KC>
__device__ __forceinline__ double frag(const double* lds, int row, int k) {
  return KC ? lds[row * KC_PITCH + k] : lds[k * MC_PITCH + row];
}

// TA: A stored k x m (A^T used).  TB: B stored n x k (B^T used).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_ref_kernel(GemmParams p, int vec_a, int vec_b) {
  if (p.abort != nullptr && *p.abort != 0) return;
  constexpr bool A_KC = !TA;  // A[m][k] is k-contiguous
  constexpr bool B_KC = TB;   // B[n][k] is k-contiguous
  __shared__ double smem[2 * 2 * TILE_ELEMS];  // [buf][A|B][tile]

  const int64_t m0 = (int64_t)blockIdx.y * GBM;
  const int64_t n0 = (int64_t)blockIdx.x * GBN;
  if (p.uplo_c == VGPOSP_LOWER && n0 > m0 + GBM - 1) return;  // tile entirely above diagonal
  p.A += blockIdx.z * p.sA;
  p.B += blockIdx.z * p.sB;
  p.C += blockIdx.z * p.sC;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;

  // K range that can contribute (triangular operands have zero blocks).
  int64_t kbeg = 0, kend = p.k;
  if (p.tri_a) {
    if (TA) kbeg = m0;               // stored A[k][i], zero for i > k  -> k >= i >= m0
    else kend = min(kend, m0 + GBM); // stored A[i][k], zero for k > i  -> k <= i < m0+GBM
  }
  if (p.tri_b) {
    if (TB) kend = min(kend, n0 + GBN);  // stored B[j][k], zero for k > j
    else kbeg = max(kbeg, n0);           // stored B[k][j], zero for j > k
  }
  kbeg = (kbeg / GBK) * GBK;

  dbl4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  const bool va = vec_a != 0, vb = vec_b != 0;
  double2 ra[4], rb[4];
  int buf = 0;
  if (kbeg < kend) {
    load_tile<A_KC>(p.A, p.lda, m0, kbeg, p.m, p.k, p.tri_a != 0, va, ra);
    load_tile<B_KC>(p.B, p.ldb, n0, kbeg, p.n, p.k, p.tri_b != 0, vb, rb);
    store_tile<A_KC>(smem, ra);
    store_tile<B_KC>(smem + TILE_ELEMS, rb);
  }
  __syncthreads();

  for (int64_t k0 = kbeg; k0 < kend; k0 += GBK) {
    const bool more = k0 + GBK < kend;
    if (more) {
      load_tile<A_KC>(p.A, p.lda, m0, k0 + GBK, p.m, p.k, p.tri_a != 0, va, ra);
      load_tile<B_KC>(p.B, p.ldb, n0, k0 + GBK, p.n, p.k, p.tri_b != 0, vb, rb);
    }
    const double* As = smem + buf * 2 * TILE_ELEMS;
    const double* Bs = As + TILE_ELEMS;
#pragma unroll
    for (int ks = 0; ks < GBK / 4; ++ks) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag<A_KC>(As, wm * 64 + i * 16 + fr, ks * 4 + fk);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag<B_KC>(Bs, wn * 64 + j * 16 + fr, ks * 4 + fk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      double* Ad = smem + (buf ^ 1) * 2 * TILE_ELEMS;
      store_tile<A_KC>(Ad, ra);
      store_tile<B_KC>(Ad + TILE_ELEMS, rb);
    }
    __syncthreads();
    buf ^= 1;
  }

  // Epilogue.  f64 MFMA C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg.
  const bool lower = p.uplo_c == VGPOSP_LOWER;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t col = n0 + wn * 64 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + fk + 4 * r;
        if (row < p.m && col < p.n && (!lower || col <= row)) {
          double* c = p.C + row * p.ldc + col;
          double v = p.alpha * acc[i][j][r];
          if (p.beta != 0.0) v += p.beta * *c;
          *c = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fast path: operands streamed HBM -> LDS with global_load_lds_dwordx4 (no VGPR staging) through
// a STAGES-deep ring, counted vmcnt waits and raw barriers, so STAGES-1 K-tiles are in flight
// while one is multiplied.  Two stages (64 KiB of LDS) let two workgroups share a CU, i.e. two
// waves per SIMD: one wave's barrier / LDS-latency bubbles are filled by the other's MFMAs.
// Measured on 8192^3 NT: 4 stages x 1 WG/CU 57 TF/s, 3 x 1 61, 2 x 1 62, 2 x 2 69 TF/s.  The LDS images are lane-linear (as glds requires) and the XOR swizzle
// is applied on the per-lane SOURCE address and on the fragment read (conflict-free reads):
//   KC image [128 rows][16 k]:  slot (r, pair p) holds pair p ^ ((r & 15) >> 1)
//   MC image [16 k][128 cols]:  slot (k, pair p) holds pair p ^ ((k & 1) << 3)
// Out-of-range rows / columns / k are CLAMPED to valid addresses (every load is in bounds); the
// duplicated data is discarded at the store (rows, columns) or masked at the fragment read (k,
// triangular operands).  Requires even m, n, k, ld and 16-byte aligned bases (else gemm_ref).
// Workgroups are remapped XCD-aware (contiguous tile ranges per XCD) and, for a lower-triangular
// C, only tiles on or below the diagonal are launched.
constexpr int STAGES = 4;      // VARIANT bk8: 4-stage ring of 8-deep K-tiles
constexpr int GBKF = 8;        // fast kernel's K-tile depth
constexpr int GEMM_GROUP = 4;  // row tiles per XCD band (1, 2, 8, 16 measured: DESIGN.md §4)
constexpr int GEMM_OCC = 2;    // workgroups per CU (the launch bound)
// 2-stage ring: the next K-tile's pieces spread over the first SPREAD2 k-slices, after each
// slice's fragment reads (0 = all issued right after the barrier)
constexpr int SPREAD2 = 2;
constexpr int OPND_ELEMS = GBM * GBKF;       // 1024 doubles = 8 KiB per operand per stage

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One 1-KiB wave-instruction ("piece" i = 0..15) of a 128-row x 16-k operand tile.
template <bool KC>
__device__ __forceinline__ void glds_piece(const double* base, int64_t ld, int64_t r0, int64_t k0,
                                           int64_t R, int64_t K, double* dst, int i, int lane) {
  {
    const double* src;
    if (KC) {
      const int row = 16 * i + (lane >> 2);
      const int kp = (lane & 3) ^ ((row >> 2) & 3);
      const int64_t gr = min(r0 + row, R - 1);
      const int64_t gk = min(k0 + 2 * kp, K - 2);
      src = base + gr * ld + gk;
    } else {
      const int p = lane ^ ((i & 1) << 3);
      const int64_t gk = min(k0 + i, K - 1);
      const int64_t gc = min(r0 + 2 * p, R - 2);
      src = base + gk * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(dst + i * 128), 16, 0, 0);
  }
}

template <bool KC>
__device__ __forceinline__ int frag_off(int row, int k) {
  if (KC) return row * 8 + 2 * ((k >> 1) ^ ((row >> 2) & 3)) + (k & 1);
  return k * 128 + 2 * ((row >> 1) ^ ((k & 1) << 3)) + (row & 1);
}

__device__ __forceinline__ int tri_root(int64_t id) {
  int64_t t = (int64_t)((sqrt(8.0 * (double)id + 1.0) - 1.0) * 0.5);
  while ((t + 1) * (t + 2) / 2 <= id) ++t;
  while (t * (t + 1) / 2 > id) --t;
  return (int)t;
}

// Tile configuration: 128x128 tiles, 4 waves of 64x64 (4x4 fragments), a STAGES-deep ring, 2
// workgroups per CU.  (The 256x128 configurations measured against it live in
// tools/variants/gemm_experiments.hip.)
template <int CFG> struct GemmCfg {
  static_assert(CFG == 1, "only the 128x128 configuration is built into the library");
  static constexpr int NSUB = 1;              // 128-row A sub-tiles
  static constexpr int NW = 4;                // waves
  static constexpr int FI = 4;                // 16-row fragments per wave
  static constexpr int NST = STAGES;          // ring depth
  static constexpr int OCC = GEMM_OCC;  // workgroups per CU (launch bound)
};

// LDS of one workgroup of the fast kernel (doubles): the STAGES-deep ring of A sub-tiles | B.
template <int CFG>
constexpr int glds_smem_elems() {
  return GemmCfg<CFG>::NST * (GemmCfg<CFG>::NSUB + 1) * OPND_ELEMS;
}

// One workgroup of the fast kernel: workgroup `bid` of the launch's `nwg` for this problem, batch
// element bz, LDS ring at smem (the kernel's own __shared__ array).
template <bool TA, bool TB, bool TRIA, bool TRIB, int CFG>
__device__ __forceinline__ void gemm_glds_body(const GemmParams& p, int tiles_m, int tiles_n,
                                               const int bid, const int nwg, const int64_t bz,
                                               double* smem) {
  if (p.abort != nullptr && *p.abort != 0) return;
  constexpr bool A_KC = !TA;
  constexpr bool B_KC = TB;
  constexpr int NSUB = GemmCfg<CFG>::NSUB, NW = GemmCfg<CFG>::NW, FI = GemmCfg<CFG>::FI;
  constexpr int NST = GemmCfg<CFG>::NST;
  constexpr int TBM = GBM * NSUB;                      // rows per tile
  constexpr int WROWS = 16 * FI;                       // rows per wave
  constexpr int SE = (NSUB + 1) * OPND_ELEMS;          // doubles per stage: A subs | B
  constexpr int PO = 8 / NW;                           // pieces per operand per wave
  constexpr int PPW = PO * (NSUB + 1);                 // pieces per wave per stage (8, 12 or 6)
#ifdef VGPOSP_BK8_NOSPREAD
  constexpr bool SPREAD = false;
#else
  constexpr bool SPREAD = NST >= 3 || SPREAD2 > 0;     // next-tile loads between the MFMAs
#endif
  constexpr bool A_IL = false, B_IL = false;  // plain fragment order
  static_assert(NST * SE == glds_smem_elems<CFG>(), "LDS ring size");

  // Tile order.  Uniform-K launches: XCD-aware bijective remap (each XCD walks a contiguous range
  // of tiles, so neighbours share A rows / B columns in its L2).  A lower-triangular A (K range
  // grows with the row tile) must NOT hand contiguous ranges to XCDs — one XCD would get every
  // long tile — so it keeps the round-robin dispatch and walks row groups longest first.
  int wg = bid;
  if (!TRIA) {
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  }
  int zsplit = 0;
  if (p.nsplit > 1) {
    zsplit = wg / p.nblk;
    wg -= zsplit * p.nblk;
  }
  int ti, tj;
  if (p.uplo_c == VGPOSP_LOWER) {
    ti = tri_root(wg);
    tj = wg - ti * (ti + 1) / 2;
  } else {
    constexpr int GROUP = GEMM_GROUP;  // row tiles per group: neighbours share A rows and B columns
    const int per_group = GROUP * tiles_n;
    const int g = wg / per_group, first = g * GROUP;
    const int gsize = min(GROUP, tiles_m - first);
    const int local = wg - g * per_group;
    ti = first + local % gsize;
    tj = local / gsize;
    if (TRIA && !TA) ti = tiles_m - 1 - ti;  // longest K ranges first
  }
  const int64_t m0 = (int64_t)ti * TBM, n0 = (int64_t)tj * GBN;
  const double* const gA = p.A + bz * p.sA;
  const double* const gB = p.B + bz * p.sB;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;

  // K range that can contribute when an operand is stored lower triangular.
  int64_t kbeg = 0, kend = p.k;
  if (TRIA) {
    if (TA) kbeg = max(kbeg, m0);        // stored A[k][i], zero for i > k
    else kend = min(kend, m0 + TBM);     // stored A[i][k], zero for k > i
  }
  if (TRIB) {
    if (TB) kend = min(kend, n0 + GBN);  // stored B[j][k], zero for k > j
    else kbeg = max(kbeg, n0);           // stored B[k][j], zero for j > k
  }
  if (p.nsplit > 1) {
    kbeg = max(kbeg, (int64_t)zsplit * p.kchunk);
    kend = min(kend, (int64_t)(zsplit + 1) * p.kchunk);
  }
  kbeg = (kbeg / GBKF) * GBKF;
  if (kend < kbeg) kend = kbeg;
  const int T = (int)((kend - kbeg + GBKF - 1) / GBKF);
  const bool partial_last = ((kend - kbeg) % GBKF) != 0;

  dbl4 acc[FI][4];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  // stage layout: [A sub-tile 0 | ... | A sub-tile NSUB-1 | B].  Every wave issues PO pieces of
  // each operand, with no branches (measured: splitting the waves into A-loaders and B-loaders
  // cost 10% on 8192^3).  Piece q (0 .. PPW-1) of this wave for K-tile t: q / PO = operand.
  auto issue_piece = [&](int t, int q) {
    double* st = smem + (t % NST) * SE;
    const int64_t k0 = kbeg + (int64_t)t * GBKF;
    const int op = q / PO, j = wave * PO + q % PO;
    if (op < NSUB)
      glds_piece<A_KC>(gA, p.lda, m0 + GBM * op, k0, p.m, p.k, st + op * OPND_ELEMS, j, lane);
    else
      glds_piece<B_KC>(gB, p.ldb, n0, k0, p.n, p.k, st + NSUB * OPND_ELEMS, j, lane);
  };
  auto issue = [&](int t) {
#pragma unroll
    for (int q = 0; q < PPW; ++q) issue_piece(t, q);
  };

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < T) issue(s);

  for (int t = 0; t < T; ++t) {
    const int after = min(T - 1 - t, NST - 2);  // tiles that may stay in flight
    static_assert(PPW == 4, "counted waits: 4 pieces");
    if (after == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (PPW == 4) {
      if (after >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else if (PPW == 8) {
      if (after >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (PPW == 12) {
      if (after >= 2) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else {
      if (after >= 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // 3-stage ring: the next K-tile's pieces are spread over the k-slices below, between MFMAs
    // (issued back to back they park the wave for their issue cost; 8192^3 NT 63.3 -> 65.7 TF/s).
    // 2-stage ring: spread over the first SPREAD2 k-slices, each after that slice's fragment reads
    // (the reads no longer wait behind the piece issue after the barrier; 65k step 16.10 ->
    // 16.23 placements/s over three interleaved repeats); SPREAD2 = 0 issues them all here.
    const bool more = t + NST - 1 < T;
    if (!SPREAD && more) issue(t + NST - 1);

    const double* As = smem + (t % NST) * SE + ((wm * WROWS) / GBM) * OPND_ELEMS;
    const double* Bs = smem + (t % NST) * SE + NSUB * OPND_ELEMS;
    const int64_t k0 = kbeg + (int64_t)t * GBKF;
    // masks only where needed: the last partial K-tile, and K-tiles that straddle the diagonal
    // of a triangular operand (k0 within 128 of the tile's first row / column)
    const bool mask = (partial_last && t == T - 1) || (TRIA && k0 < m0 + TBM && k0 + GBKF > m0) ||
                      (TRIB && k0 < n0 + GBN && k0 + GBKF > n0);
#pragma unroll
    for (int ks = 0; ks < GBKF / 4; ++ks) {
      const int k = ks * 4 + fk;
      double a[FI], b[4];
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int r = (wm * WROWS) % GBM + i * 16 + fr;  // row within the sub-tile
        a[i] = As[frag_off<A_KC>(r, k)];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = wn * 64 + j * 16 + fr;
        b[j] = Bs[frag_off<B_KC>(c, k)];
      }
      if (mask) {
        const int64_t gk = k0 + k;
#pragma unroll
        for (int i = 0; i < FI; ++i) {
          const int64_t gm = m0 + wm * WROWS + i * 16 + fr;
          if (gk >= kend || (TRIA && (TA ? gm > gk : gk > gm))) a[i] = 0.0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t gn = n0 + wn * 64 + j * 16 + fr;
          if (gk >= kend || (TRIB && (TB ? gk > gn : gn > gk))) b[j] = 0.0;
        }
      }
      if (SPREAD && more) {
        constexpr int NS = NST >= 3 ? GBKF / 4 : (SPREAD2 > 0 ? SPREAD2 : 4);
        if (ks < NS) {
#pragma unroll
          for (int q = (ks * PPW) / NS; q < ((ks + 1) * PPW) / NS; ++q) issue_piece(t + NST - 1, q);
        }
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  const bool lower = p.uplo_c == VGPOSP_LOWER;
#pragma unroll
  for (int i = 0; i < FI; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t col = n0 + wn * 64 + (B_IL ? 32 * (j >> 1) + 2 * fr + (j & 1) : j * 16 + fr);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int x = fk + 4 * r;
        const int64_t row = m0 + wm * WROWS + (A_IL ? 32 * (i >> 1) + 2 * x + (i & 1) : i * 16 + x);
        if (row < p.m && col < p.n && (!lower || col <= row)) {
          if (p.nsplit > 1) {
            p.part[bz * p.sP + (int64_t)zsplit * p.m * p.n + row * p.n + col] = p.alpha * acc[i][j][r];
            continue;
          }
          double* c = p.C + bz * p.sC + row * p.ldc + col;
          double v = p.alpha * acc[i][j][r];
          if (p.beta != 0.0) v += p.beta * *c;
          *c = v;
        }
      }
    }
  }
}

template <bool TA, bool TB, bool TRIA, bool TRIB, int CFG>
__global__ __launch_bounds__(64 * GemmCfg<CFG>::NW, GemmCfg<CFG>::OCC) void gemm_glds_kernel(
    GemmParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) double smem[glds_smem_elems<CFG>()];
  gemm_glds_body<TA, TB, TRIA, TRIB, CFG>(p, tiles_m, tiles_n, blockIdx.x, gridDim.x, blockIdx.y,
                                          smem);
}

// Grouped launch: up to GROUP_MAX independent problems (each its own shape, operands, flags and
// split-K) in ONE launch, problem g on blockIdx.y.  For the latency-bound M x M products of the
// VGP step, which each fill a few dozen CUs: one launch instead of one per product.
constexpr int GROUP_MAX = 8;
struct GemmGroup {
  GemmParams p[GROUP_MAX];
  int tiles_m[GROUP_MAX], tiles_n[GROUP_MAX], nwg[GROUP_MAX];
  int flags[GROUP_MAX];  // bit 0 transa, 1 transb, 2 tri_a, 3 tri_b
};

__global__ __launch_bounds__(256, 2) void gemm_group_kernel(GemmGroup gg) {
  __shared__ __attribute__((aligned(16))) double smem[glds_smem_elems<1>()];
  const int g = blockIdx.y;
  const int bid = blockIdx.x, nwg = gg.nwg[g];
  if (bid >= nwg) return;
  const GemmParams& p = gg.p[g];
  const int tm = gg.tiles_m[g], tn = gg.tiles_n[g];
#define VG_GROUP_CASE(F)                                                                         \
  case F:                                                                                      \
    gemm_glds_body<(F & 1) != 0, (F & 2) != 0, (F & 4) != 0, (F & 8) != 0, 1>(p, tm, tn, bid,   \
                                                                             nwg, 0, smem);    \
    break;
  switch (gg.flags[g]) {
    VG_GROUP_CASE(0) VG_GROUP_CASE(1) VG_GROUP_CASE(2) VG_GROUP_CASE(3)
    VG_GROUP_CASE(4) VG_GROUP_CASE(5) VG_GROUP_CASE(6) VG_GROUP_CASE(7)
    VG_GROUP_CASE(8) VG_GROUP_CASE(9) VG_GROUP_CASE(10) VG_GROUP_CASE(11)
    VG_GROUP_CASE(12) VG_GROUP_CASE(13) VG_GROUP_CASE(14) VG_GROUP_CASE(15)
  }
#undef VG_GROUP_CASE
}

template <int CFG, bool TA, bool TB, bool TRIA, bool TRIB>
static void launch_one(dim3 g1, hipStream_t stream, const GemmParams& p, int tm, int tn) {
  hipLaunchKernelGGL((gemm_glds_kernel<TA, TB, TRIA, TRIB, CFG>), g1, dim3(64 * GemmCfg<CFG>::NW),
                     0, stream, p, tm, tn);
}

// every (transa, transb, tri_a, tri_b) combination: the kernel's K-range and mask logic is
// generic in the four flags.
template <int CFG, bool TA, bool TB>
static void launch_tri(dim3 g1, hipStream_t stream, const GemmParams& p, int tm, int tn, int tri_a,
                       int tri_b) {
  if (CFG != 1 || (!tri_a && !tri_b)) return launch_one<CFG, TA, TB, false, false>(g1, stream, p, tm, tn);
  if (tri_a && tri_b) return launch_one<1, TA, TB, true, true>(g1, stream, p, tm, tn);
  if (tri_a) return launch_one<1, TA, TB, true, false>(g1, stream, p, tm, tn);
  launch_one<1, TA, TB, false, true>(g1, stream, p, tm, tn);
}

template <int CFG>
static void launch_glds(dim3 g1, hipStream_t stream, const GemmParams& p, int tm, int tn,
                        int transa, int transb, int tri_a, int tri_b) {
  if (!transa && !transb) launch_tri<CFG, false, false>(g1, stream, p, tm, tn, tri_a, tri_b);
  else if (!transa) launch_tri<CFG, false, true>(g1, stream, p, tm, tn, tri_a, tri_b);
  else if (!transb) launch_tri<CFG, true, false>(g1, stream, p, tm, tn, tri_a, tri_b);
  else launch_tri<CFG, true, true>(g1, stream, p, tm, tn, tri_a, tri_b);
}

// C = sum_z part[z] + beta * C over the (lower) output, fixed summation order.
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(int64_t m, int64_t n, int nsplit,
                                                                 const double* part, double beta,
                                                                 double* C, int64_t ldc,
                                                                 int lower, int64_t sP = 0,
                                                                 int64_t sC = 0) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= m * n) return;
  part += blockIdx.y * sP;
  C += blockIdx.y * sC;
  const int64_t row = e / n, col = e - row * n;
  if (lower && col > row) return;
  double v = 0.0;
  for (int z = 0; z < nsplit; ++z) v += part[(int64_t)z * m * n + e];
  double* c = C + row * ldc + col;
  if (beta != 0.0) v += beta * *c;
  *c = v;
}

// The split-K reduction of a grouped launch: problem g on blockIdx.y (no-op where unsplit).
struct ReduceGroup {
  int64_t m[GROUP_MAX], n[GROUP_MAX], ldc[GROUP_MAX];
  const double* part[GROUP_MAX];
  double* C[GROUP_MAX];
  double beta[GROUP_MAX];
  int nsplit[GROUP_MAX], lower[GROUP_MAX];
};

__global__ __launch_bounds__(256) void gemm_splitk_reduce_group_kernel(ReduceGroup r) {
  const int g = blockIdx.y;
  if (r.nsplit[g] <= 1) return;
  const int64_t m = r.m[g], n = r.n[g];
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= m * n) return;
  const int64_t row = e / n, col = e - row * n;
  if (r.lower[g] && col > row) return;
  double v = 0.0;
  for (int z = 0; z < r.nsplit[g]; ++z) v += r.part[g][(int64_t)z * m * n + e];
  double* c = r.C[g] + row * r.ldc[g] + col;
  if (r.beta[g] != 0.0) v += r.beta[g] * *c;
  *c = v;
}

// y = alpha * A x + beta * y for a single output column (C = A B with n == 1): one wave per row,
// HBM-bound (reads A once).  x is B's only column (stride ldb_x elements).
__global__ __launch_bounds__(256) void gemv_rows_kernel(int64_t m, int64_t k, double alpha,
                                                        const double* A, int64_t lda,
                                                        const double* x, int64_t incx, double beta,
                                                        double* y, int64_t incy, int tri) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= m) return;
  if (tri) k = min(k, r + 1);  // stored lower triangular: A[r][c] = 0 for c > r
  const double* row = A + r * lda;
  double s0 = 0.0, s1 = 0.0;
  int64_t c = lane;
  for (; c + 64 < k; c += 128) {
    s0 += row[c] * x[c * incx];
    s1 += row[c + 64] * x[(c + 64) * incx];
  }
  if (c < k) s0 += row[c] * x[c * incx];
  const double s = wave_sum(s0 + s1);
  if (lane == 0) {
    double v = alpha * s;
    if (beta != 0.0) v += beta * y[r * incy];
    y[r * incy] = v;
  }
}

// Split-K GEMV: wave (row r, split z) writes part[z][r]; then gemv_reduce.  For a few rows and a
// long K (c = Kzx y of the VGP: 512 rows x 262,144) one wave per row leaves most CUs idle.
__global__ __launch_bounds__(256) void gemv_rows_split_kernel(int64_t m, int64_t k, int64_t kchunk,
                                                              const double* A, int64_t lda,
                                                              const double* x, int64_t incx,
                                                              double* part, int tri) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= m) return;
  const int64_t k0 = (int64_t)blockIdx.y * kchunk, k1 = min(tri ? min(k, r + 1) : k, k0 + kchunk);
  const double* row = A + r * lda;
  double s0 = 0.0, s1 = 0.0;
  int64_t c = k0 + lane;
  for (; c + 64 < k1; c += 128) {
    s0 += row[c] * x[c * incx];
    s1 += row[c + 64] * x[(c + 64) * incx];
  }
  if (c < k1) s0 += row[c] * x[c * incx];
  const double s = wave_sum(s0 + s1);
  if (lane == 0) part[(int64_t)blockIdx.y * m + r] = s;
}

// y = alpha A^T x (+ beta y) with A stored k x m (row-major): thread j owns output j, the k rows
// it walks are read coalesced across the workgroup.  Split over k when part != null.
__global__ __launch_bounds__(256) void gemv_t_kernel(int64_t m, int64_t k, int64_t kchunk,
                                                     double alpha, const double* A, int64_t lda,
                                                     const double* x, int64_t incx, double beta,
                                                     double* y, int64_t incy, double* part,
                                                     int tri) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= m) return;
  // tri: A stored k x m lower triangular, A[c][j] = 0 for j > c, so only c >= j contribute
  const int64_t k0 = max((int64_t)blockIdx.y * kchunk, tri ? j : (int64_t)0);
  const int64_t k1 = min(k, (int64_t)blockIdx.y * kchunk + kchunk);
  double s0 = 0.0, s1 = 0.0;
  int64_t c = k0;
  for (; c + 1 < k1; c += 2) {
    s0 += A[c * lda + j] * x[c * incx];
    s1 += A[(c + 1) * lda + j] * x[(c + 1) * incx];
  }
  if (c < k1) s0 += A[c * lda + j] * x[c * incx];
  if (part) {
    part[(int64_t)blockIdx.y * m + j] = s0 + s1;
  } else {
    double v = alpha * (s0 + s1);
    if (beta != 0.0) v += beta * y[j * incy];
    y[j * incy] = v;
  }
}

__global__ __launch_bounds__(256) void gemv_reduce_kernel(int64_t m, int nsplit, const double* part,
                                                          double alpha, double beta, double* y,
                                                          int64_t incy) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= m) return;
  double s = 0.0;
  for (int z = 0; z < nsplit; ++z) s += part[(int64_t)z * m + r];
  double v = alpha * s;
  if (beta != 0.0) v += beta * y[r * incy];
  y[r * incy] = v;
}

// splits for the n == 1 paths: about 8192 (rows) / 4096 (transposed) waves in flight, >= 1024
// (rows) / 32 (transposed) K elements per split.  Short per-thread chains matter more than the
// partials: the VGP step's M x M triangular L^-T x (m = 512, k <= 512) ran 41 us on 2 workgroups
// of 256-long serial sums, its Kzb^T v (32,768 x 512) at 2.1 TB/s.
static int gemv_splits(int64_t m, int64_t k, int transa) {
  int64_t s = transa ? ceil_div(4096 * 64, std::max<int64_t>(m, 1)) : ceil_div(8192, m);
  s = std::min<int64_t>(s, transa ? k / 32 : k / 1024);
  return (int)std::max<int64_t>(std::min<int64_t>(s, 4096), 1);
}

static bool aligned16(const void* ptr, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(ptr) % 16 == 0) && (ld % 2 == 0);
}

// "gemm_f64[nt|nn|tn|tt][,triA][,triB][,narrow]": narrow = fewer than 512 workgroups (less than
// two per CU: the recursion's small levels, latency-bound)
static const char* gemm_class_name(int ta, int tb, int tra, int trb, bool wide) {
  static const char* names[32] = {
#define VG_CLS(L, T) "gemm_f64[" L T "]", "gemm_f64[" L T ",narrow]"
      VG_CLS("nn", ""), VG_CLS("nn", ",triA"), VG_CLS("nn", ",triB"), VG_CLS("nn", ",triA,triB"),
      VG_CLS("nt", ""), VG_CLS("nt", ",triA"), VG_CLS("nt", ",triB"), VG_CLS("nt", ",triA,triB"),
      VG_CLS("tn", ""), VG_CLS("tn", ",triA"), VG_CLS("tn", ",triB"), VG_CLS("tn", ",triA,triB"),
      VG_CLS("tt", ""), VG_CLS("tt", ",triA"), VG_CLS("tt", ",triB"), VG_CLS("tt", ",triA,triB"),
#undef VG_CLS
  };
  const int lay = (ta ? 2 : 0) + (tb ? 1 : 0);
  const int tri = (tra ? 1 : 0) + (trb ? 2 : 0);
  return names[(lay * 4 + tri) * 2 + (wide ? 0 : 1)];
}

int gemm_launch_batched(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                        const double* A, int64_t lda, int64_t sA, const double* B, int64_t ldb,
                        int64_t sB, double beta, double* C, int64_t ldc, int64_t sC, int uplo_c,
                        int tri_a, int tri_b, int nsplit, double* part, int64_t sP, int batch,
                        hipStream_t stream) {
  if (m <= 0 || n <= 0 || batch <= 0) return 0;
  if (n == 1 && !tri_b && uplo_c == VGPOSP_FULL && k > 0 && batch > 1) {
    for (int b = 0; b < batch; ++b) {
      int rc = gemm_launch_batched(transa, transb, m, n, k, alpha, A + b * sA, lda, 0, B + b * sB,
                                   ldb, 0, beta, C + b * sC, ldc, 0, uplo_c, tri_a, tri_b, nsplit,
                                   part ? part + b * sP : nullptr, 0, 1, stream);
      if (rc) return rc;
    }
    return 0;
  }
  if (n == 1 && !tri_b && uplo_c == VGPOSP_FULL && k > 0) {
    ProfScope ps("gemv_f64", stream, 2.0 * (double)m * k, 8.0 * ((double)m * k + k + 2.0 * m));
    const int64_t incx = transb ? 1 : ldb;
    const int S = (nsplit > 1 && part != nullptr) ? nsplit : 1;
    const int64_t kchunk = ceil_div(k, S);
    if (!transa) {
      if (S == 1) {
        hipLaunchKernelGGL(gemv_rows_kernel, dim3((unsigned)ceil_div(m, 4)), dim3(256), 0, stream, m,
                           k, alpha, A, lda, B, incx, beta, C, ldc, tri_a);
      } else {
        hipLaunchKernelGGL(gemv_rows_split_kernel, dim3((unsigned)ceil_div(m, 4), (unsigned)S),
                           dim3(256), 0, stream, m, k, kchunk, A, lda, B, incx, part, tri_a);
      }
    } else {
      hipLaunchKernelGGL(gemv_t_kernel, dim3((unsigned)ceil_div(m, 256), (unsigned)S), dim3(256), 0,
                         stream, m, k, kchunk, alpha, A, lda, B, incx, beta, C, ldc,
                         S > 1 ? part : nullptr, tri_a);
    }
    VG_LAUNCH_CHECK();
    if (S > 1) {
      hipLaunchKernelGGL(gemv_reduce_kernel, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, stream,
                         m, S, part, alpha, beta, C, ldc);
      VG_LAUNCH_CHECK();
    }
    return 0;
  }
  GemmParams p{m, n, k, alpha, beta, A, lda, B, ldb, C, ldc, uplo_c, tri_a, tri_b, 1, 0, 0, nullptr,
               sA, sB, sC, sP, tl_gemm_abort};
  const int va = aligned16(A, lda) && (batch == 1 || sA % 2 == 0);
  const int vb = aligned16(B, ldb) && (batch == 1 || sB % 2 == 0);
  const bool even = (m % 2 == 0) && (n % 2 == 0) && (k % 2 == 0) && k > 0;
  if (va && vb && even) {
    const int tm = (int)ceil_div(m, GBM), tn = (int)ceil_div(n, GBN);
    const int64_t nblk = (uplo_c == VGPOSP_LOWER) ? (int64_t)tm * (tm + 1) / 2 : (int64_t)tm * tn;
    const double outs = (uplo_c == VGPOSP_LOWER) ? 0.5 * (double)m * (double)(m + 1) : (double)m * n;
    // algorithmic flops: a triangular operand halves the useful products
    const double fl = 2.0 * batch * (double)k * outs * ((tri_a && tri_b) ? (1.0 / 3.0) : (tri_a || tri_b) ? 0.5 : 1.0);
    if (nsplit > 1 && part != nullptr) {
      p.nblk = (int)nblk;
      p.kchunk = ceil_div(ceil_div(k, nsplit), GBK) * GBK;
      p.nsplit = (int)ceil_div(k, p.kchunk);
      p.part = part;
    }
    const double by =
        8.0 * batch * ((double)m * k + (double)k * n + (beta != 0.0 ? 2.0 : 1.0) * outs);
    // recorded under its layout class; vgposp_prof_query("gemm_f64") sums the classes
    ProfScope ps(gemm_class_name(transa, transb, tri_a, tri_b, nblk * p.nsplit * batch >= 512),
                 stream, fl, by);
    dim3 g1((unsigned)(nblk * p.nsplit), (unsigned)batch);
    launch_glds<1>(g1, stream, p, tm, tn, transa, transb, tri_a, tri_b);
    VG_LAUNCH_CHECK();
    if (p.nsplit > 1) {
      hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)ceil_div(m * n, 256), (unsigned)batch),
                         dim3(256), 0, stream, m, n, p.nsplit, part, beta, C, ldc,
                         uplo_c == VGPOSP_LOWER, sP, sC);
      VG_LAUNCH_CHECK();
    }
    return 0;
  }
  dim3 grid((unsigned)ceil_div(n, GBN), (unsigned)ceil_div(m, GBM), (unsigned)batch);
  const double outs = (uplo_c == VGPOSP_LOWER) ? 0.5 * (double)m * (double)(m + 1) : (double)m * n;
  ProfScope ps("gemm_f64", stream, 2.0 * batch * (double)k * outs,
               8.0 * batch * ((double)m * k + (double)k * n + (beta != 0.0 ? 2.0 : 1.0) * outs));
  if (!transa && !transb) hipLaunchKernelGGL((gemm_ref_kernel<false, false>), grid, dim3(256), 0, stream, p, va, vb);
  else if (!transa && transb) hipLaunchKernelGGL((gemm_ref_kernel<false, true>), grid, dim3(256), 0, stream, p, va, vb);
  else if (transa && !transb) hipLaunchKernelGGL((gemm_ref_kernel<true, false>), grid, dim3(256), 0, stream, p, va, vb);
  else hipLaunchKernelGGL((gemm_ref_kernel<true, true>), grid, dim3(256), 0, stream, p, va, vb);
  VG_LAUNCH_CHECK();
  return 0;
}

int gemm_launch_split(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                      const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                      double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, int nsplit,
                      double* part, hipStream_t stream) {
  return gemm_launch_batched(transa, transb, m, n, k, alpha, A, lda, 0, B, ldb, 0, beta, C, ldc, 0,
                             uplo_c, tri_a, tri_b, nsplit, part, 0, 1, stream);
}

int gemm_launch(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, hipStream_t stream) {
  return gemm_launch_split(transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, uplo_c,
                           tri_a, tri_b, 1, nullptr, stream);
}

// Minimum depth of a short-K split (vgposp_gemm_set_split_depth).  Set explicitly by the caller,
// never from the environment: every workspace query and the launch that uses the workspace read
// the same value as long as the caller does not change it in between (round 3 read it from
// the environment on every launch, while tools/vgp_ab.py rewrote it between variants).
static std::atomic<int> g_split_min_k{16};

// Split count for a launch with few output tiles and a long K: enough workgroups for 256 CUs
// (about two per CU), each split at least 512 deep.
static int auto_splits(int64_t m, int64_t n, int64_t k, int uplo_c, int transa = 0) {
  if (n == 1 && uplo_c == VGPOSP_FULL) return gemv_splits(m, k, transa);
  const int64_t tm = ceil_div(m, GBM), tn = ceil_div(n, GBN);
  const int64_t nblk = uplo_c == VGPOSP_LOWER ? tm * (tm + 1) / 2 : tm * tn;
  // one full round of workgroup slots (256 CUs x 2 workgroups): the splits all run the same K
  // length, so a round that overflows by a few workgroups costs a whole second round (measured:
  // 10 lower tiles x 52 splits = 520 > 512 ran as slowly as the 16-tile full product)
  int64_t s = 512 / nblk;
  // long K: splits at least 512 deep.  Short K (few output tiles, e.g. the M x M products of the
  // VGP step, 16 tiles of a 512^3 product on 16 CUs, and the Cholesky recursion's 128..1024
  // levels): up to 8 splits, at least 16 deep (one K-tile).  Measured against 64 deep (the
  // VGPOSP_SPLIT_MIN_K override, profiles/r3_vgp_ab_streams_splitk_*.jsonl): C3 6.30 -> 6.19 ms,
  // C5 7.32 -> 7.26 ms, the 65k step unchanged (16.27 vs 16.30 placements/s): a split's partial
  // costs less than the serial K-steps it removes from a latency-bound chain.
  const int64_t deep = k / 512;
  const int64_t min_k = g_split_min_k.load(std::memory_order_relaxed);
  s = std::min<int64_t>(s, deep >= 8 ? deep : std::min<int64_t>(8, k / min_k));
  return (int)std::max<int64_t>(s, 1);
}

// Partial elements problem g of a group needs (0 when it runs unsplit or off the fast kernel).
static int64_t group_part_elems(int transa, int64_t m, int64_t n, int64_t k, int uplo_c) {
  if (m <= 0 || n <= 0 || k <= 0 || n == 1) return 0;
  const int sp = auto_splits(m, n, k, uplo_c, transa);
  return sp > 1 ? (int64_t)sp * m * n : 0;
}

// `count` independent GEMMs (flags[5 g ..]: transa, transb, uplo_c, tri_a, tri_b; dims[3 g ..]:
// m, n, k): every problem the fast kernel takes runs in ONE grouped launch (+ one grouped split-K
// reduction), the others (GEMV shapes, unaligned or odd operands) one by one.
int gemm_launch_group(int count, const int* flags, const int64_t* dims, const double* alpha,
                      const double* beta, const double* const* A, const int64_t* lda,
                      const double* const* B, const int64_t* ldb, double* const* C,
                      const int64_t* ldc, double* part, hipStream_t s) {
  GemmGroup gg{};
  ReduceGroup rg{};
  int ng = 0, maxwg = 0;
  int64_t poff = 0, maxel = 0;
  double fl = 0.0, by = 0.0;
  for (int g = 0; g < count; ++g) {
    const int ta = flags[5 * g], tb = flags[5 * g + 1], up = flags[5 * g + 2];
    const int tra = flags[5 * g + 3], trb = flags[5 * g + 4];
    const int64_t m = dims[3 * g], n = dims[3 * g + 1], k = dims[3 * g + 2];
    if (m <= 0 || n <= 0) continue;
    const bool fast = n > 1 && k > 0 && aligned16(A[g], lda[g]) && aligned16(B[g], ldb[g]) &&
                      m % 2 == 0 && n % 2 == 0 && k % 2 == 0 && ng < GROUP_MAX;
    const int64_t pe = group_part_elems(ta, m, n, k, up);
    if (!fast) {
      if (int rc = gemm_launch_split(ta, tb, m, n, k, alpha[g], A[g], lda[g], B[g], ldb[g], beta[g],
                                     C[g], ldc[g], up, tra, trb, pe > 0 ? (int)(pe / (m * n)) : 1,
                                     pe > 0 ? part + poff : nullptr, s))
        return rc;
      poff += pe;
      continue;
    }
    GemmParams p{m, n, k, alpha[g], beta[g], A[g], lda[g], B[g], ldb[g], C[g], ldc[g], up, tra, trb,
                 1, 0, 0, nullptr, 0, 0, 0, 0, tl_gemm_abort};
    const int tm = (int)ceil_div(m, GBM), tn = (int)ceil_div(n, GBN);
    const int64_t nblk = up == VGPOSP_LOWER ? (int64_t)tm * (tm + 1) / 2 : (int64_t)tm * tn;
    if (pe > 0) {
      const int sp = (int)(pe / (m * n));
      p.nblk = (int)nblk;
      p.kchunk = ceil_div(ceil_div(k, sp), GBK) * GBK;
      p.nsplit = (int)ceil_div(k, p.kchunk);
      p.part = part + poff;
      poff += pe;
    }
    const double outs = up == VGPOSP_LOWER ? 0.5 * (double)m * (double)(m + 1) : (double)m * n;
    fl += 2.0 * (double)k * outs * ((tra && trb) ? (1.0 / 3.0) : (tra || trb) ? 0.5 : 1.0);
    by += 8.0 * ((double)m * k + (double)k * n + (beta[g] != 0.0 ? 2.0 : 1.0) * outs);
    gg.p[ng] = p;
    gg.tiles_m[ng] = tm;
    gg.tiles_n[ng] = tn;
    gg.nwg[ng] = (int)(nblk * p.nsplit);
    gg.flags[ng] = (ta ? 1 : 0) | (tb ? 2 : 0) | (tra ? 4 : 0) | (trb ? 8 : 0);
    maxwg = std::max(maxwg, gg.nwg[ng]);
    rg.m[ng] = m;
    rg.n[ng] = n;
    rg.ldc[ng] = ldc[g];
    rg.part[ng] = p.part;
    rg.C[ng] = C[g];
    rg.beta[ng] = beta[g];
    rg.nsplit[ng] = p.nsplit;
    rg.lower[ng] = up == VGPOSP_LOWER;
    if (p.nsplit > 1) maxel = std::max(maxel, m * n);
    ++ng;
  }
  if (ng == 0) return 0;
  {
    ProfScope ps("gemm_f64", s, fl, by);
    hipLaunchKernelGGL(gemm_group_kernel, dim3((unsigned)maxwg, (unsigned)ng), dim3(256), 0, s, gg);
    VG_LAUNCH_CHECK();
  }
  if (maxel > 0) {
    hipLaunchKernelGGL(gemm_splitk_reduce_group_kernel, dim3((unsigned)ceil_div(maxel, 256), (unsigned)ng),
                       dim3(256), 0, s, rg);
    VG_LAUNCH_CHECK();
  }
  return 0;
}

void gemm_set_abort(const int* flag) { tl_gemm_abort = flag; }

int gemm_auto_splits(int64_t m, int64_t n, int64_t k, int uplo_c, int transa) {
  return auto_splits(m, n, k, uplo_c, transa);
}

}  // namespace vgposp

extern "C" int vgposp_gemm_set_split_depth(int min_k) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(min_k >= 16 && min_k <= 4096 && min_k % 16 == 0, 1);
  g_split_min_k.store(min_k, std::memory_order_relaxed);
  return 0;
}

extern "C" int vgposp_gemm_split_depth(void) { return vgposp::g_split_min_k.load(); }

extern "C" size_t vgposp_gemm_splitk_workspace_bytes(int64_t m, int64_t n, int64_t k, int uplo_c,
                                                     int splits) {
  using namespace vgposp;
  if (m <= 0 || n <= 0 || k <= 0) return 0;
  // the GEMV paths pick their split count by transa, which this query does not take: size for
  // the larger of the two
  if (splits <= 0)
    splits = std::max(auto_splits(m, n, k, uplo_c, 0), auto_splits(m, n, k, uplo_c, 1));
  return splits > 1 ? 8 * (size_t)splits * m * n : 0;
}

extern "C" int vgposp_gemm_splitk(int transa, int transb, int64_t m, int64_t n, int64_t k,
                                  double alpha, const double* A, int64_t lda, const double* B,
                                  int64_t ldb, double beta, double* C, int64_t ldc, int uplo_c,
                                  int tri_a, int tri_b, int splits, void* ws, size_t ws_bytes,
                                  void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(m >= 0, 3);
  VG_CHECK_ARG(n >= 0, 4);
  VG_CHECK_ARG(k >= 0, 5);
  VG_CHECK_ARG(A != nullptr || m == 0 || k == 0, 7);
  VG_CHECK_ARG(lda >= (transa ? (m > 0 ? m : 1) : (k > 0 ? k : 1)), 8);
  VG_CHECK_ARG(B != nullptr || n == 0 || k == 0, 9);
  VG_CHECK_ARG(ldb >= (transb ? (k > 0 ? k : 1) : (n > 0 ? n : 1)), 10);
  VG_CHECK_ARG(C != nullptr || m == 0 || n == 0, 12);
  VG_CHECK_ARG(ldc >= (n > 0 ? n : 1), 13);
  VG_CHECK_ARG(uplo_c == VGPOSP_FULL || (uplo_c == VGPOSP_LOWER && m == n), 14);
  if (m == 0 || n == 0) return 0;
  if (splits <= 0) splits = k > 0 ? auto_splits(m, n, k, uplo_c, transa) : 1;
  if (splits > 1) {
    const size_t need = 8 * (size_t)splits * m * n;
    if (ws == nullptr || ws_bytes < need) {
      set_error("vgposp_gemm_splitk: workspace %zu < %zu bytes", ws_bytes, need);
      return VGPOSP_E_WS;
    }
  }
  return gemm_launch_split(transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, uplo_c,
                           tri_a, tri_b, splits, static_cast<double*>(ws), as_stream(stream));
}

extern "C" int vgposp_gemm(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                           const double* A, int64_t lda, const double* B, int64_t ldb,
                           double beta, double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b,
                           void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(m >= 0, 3);
  VG_CHECK_ARG(n >= 0, 4);
  VG_CHECK_ARG(k >= 0, 5);
  VG_CHECK_ARG(A != nullptr || m == 0 || k == 0, 7);
  VG_CHECK_ARG(lda >= (transa ? (m > 0 ? m : 1) : (k > 0 ? k : 1)), 8);
  VG_CHECK_ARG(B != nullptr || n == 0 || k == 0, 9);
  VG_CHECK_ARG(ldb >= (transb ? (k > 0 ? k : 1) : (n > 0 ? n : 1)), 10);
  VG_CHECK_ARG(C != nullptr || m == 0 || n == 0, 12);
  VG_CHECK_ARG(ldc >= (n > 0 ? n : 1), 13);
  VG_CHECK_ARG(uplo_c == VGPOSP_FULL || (uplo_c == VGPOSP_LOWER && m == n), 14);
  return gemm_launch(transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, uplo_c, tri_a,
                     tri_b, as_stream(stream));
}

extern "C" size_t vgposp_gemm_batched_workspace_bytes(int64_t m, int64_t n, int64_t k, int uplo_c,
                                                      int batch) {
  using namespace vgposp;
  if (m <= 0 || n <= 0 || k <= 0 || batch <= 0 || n == 1) return 0;
  const int sp = auto_splits(m, n, k, uplo_c, 0);
  return sp > 1 ? 8 * (size_t)sp * m * n * batch : 0;
}

extern "C" int vgposp_gemm_batched(int transa, int transb, int64_t m, int64_t n, int64_t k,
                                   double alpha, const double* A, int64_t lda, int64_t sA,
                                   const double* B, int64_t ldb, int64_t sB, double beta, double* C,
                                   int64_t ldc, int64_t sC, int uplo_c, int tri_a, int tri_b,
                                   int batch, void* ws, size_t ws_bytes, void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(m >= 0, 3);
  VG_CHECK_ARG(n >= 0, 4);
  VG_CHECK_ARG(k >= 0, 5);
  VG_CHECK_ARG(A != nullptr || m == 0 || k == 0, 7);
  VG_CHECK_ARG(lda >= (transa ? (m > 0 ? m : 1) : (k > 0 ? k : 1)), 8);
  VG_CHECK_ARG(B != nullptr || n == 0 || k == 0, 10);
  VG_CHECK_ARG(ldb >= (transb ? (k > 0 ? k : 1) : (n > 0 ? n : 1)), 11);
  VG_CHECK_ARG(C != nullptr || m == 0 || n == 0, 14);
  VG_CHECK_ARG(ldc >= (n > 0 ? n : 1), 15);
  VG_CHECK_ARG(uplo_c == VGPOSP_FULL || (uplo_c == VGPOSP_LOWER && m == n), 17);
  VG_CHECK_ARG(batch >= 1 && batch <= 65535, 20);
  if (m == 0 || n == 0) return 0;
  int sp = (k > 0 && n > 1) ? auto_splits(m, n, k, uplo_c, transa) : 1;
  if (sp > 1 && (ws == nullptr || ws_bytes < 8 * (size_t)sp * m * n * batch)) sp = 1;
  return gemm_launch_batched(transa, transb, m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc,
                             sC, uplo_c, tri_a, tri_b, sp, sp > 1 ? static_cast<double*>(ws) : nullptr,
                             (int64_t)sp * m * n, batch, as_stream(stream));
}

extern "C" size_t vgposp_gemm_group_workspace_bytes(int count, const int* flags,
                                                    const int64_t* dims) {
  using namespace vgposp;
  if (count <= 0 || flags == nullptr || dims == nullptr) return 0;
  int64_t el = 0;
  for (int g = 0; g < count; ++g)
    el += group_part_elems(flags[5 * g], dims[3 * g], dims[3 * g + 1], dims[3 * g + 2],
                           flags[5 * g + 2]);
  return 8 * (size_t)el;
}

extern "C" int vgposp_gemm_group(int count, const int* flags, const int64_t* dims,
                                 const double* alpha, const double* beta, const double* const* A,
                                 const int64_t* lda, const double* const* B, const int64_t* ldb,
                                 double* const* C, const int64_t* ldc, void* ws, size_t ws_bytes,
                                 void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(count >= 0, 1);
  if (count == 0) return 0;
  VG_CHECK_ARG(flags != nullptr, 2);
  VG_CHECK_ARG(dims != nullptr, 3);
  VG_CHECK_ARG(alpha != nullptr && beta != nullptr, 4);
  VG_CHECK_ARG(A != nullptr && lda != nullptr && B != nullptr && ldb != nullptr, 6);
  VG_CHECK_ARG(C != nullptr && ldc != nullptr, 10);
  for (int g = 0; g < count; ++g) {
    const int ta = flags[5 * g], tb = flags[5 * g + 1], up = flags[5 * g + 2];
    const int64_t m = dims[3 * g], n = dims[3 * g + 1], k = dims[3 * g + 2];
    VG_CHECK_ARG(m >= 0 && n >= 0 && k >= 0, 3);
    VG_CHECK_ARG(up == VGPOSP_FULL || (up == VGPOSP_LOWER && m == n), 2);
    VG_CHECK_ARG(A[g] != nullptr || m == 0 || k == 0, 6);
    VG_CHECK_ARG(lda[g] >= (ta ? (m > 0 ? m : 1) : (k > 0 ? k : 1)), 7);
    VG_CHECK_ARG(B[g] != nullptr || n == 0 || k == 0, 8);
    VG_CHECK_ARG(ldb[g] >= (tb ? (k > 0 ? k : 1) : (n > 0 ? n : 1)), 9);
    VG_CHECK_ARG(C[g] != nullptr || m == 0 || n == 0, 10);
    VG_CHECK_ARG(ldc[g] >= (n > 0 ? n : 1), 11);
  }
  const size_t need = vgposp_gemm_group_workspace_bytes(count, flags, dims);
  if (need > 0 && (ws == nullptr || ws_bytes < need)) {
    set_error("vgposp_gemm_group: workspace %zu < %zu bytes", ws_bytes, need);
    return VGPOSP_E_WS;
  }
  return gemm_launch_group(count, flags, dims, alpha, beta, A, lda, B, ldb, C, ldc,
                           static_cast<double*>(ws), as_stream(stream));
}
