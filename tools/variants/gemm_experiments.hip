// EXPERIMENT SOURCE — not part of libvgposp.so.  The product GEMM is vgposp_amd/csrc/gemm.hip.
// This is the round-1 gemm.hip with every measured-and-rejected variant still in it:
// the one-wave-per-SIMD register-staged kernel gemm_rs_kernel (VGPOSP_GEMM_RS=1/2), the 256x128
// configurations (VGPOSP_GEMM_CFG=2/3), b128 fragment reads (-DVGPOSP_GEMM_B128=1), per-cluster
// s_setprio (-DVGPOSP_GEMM_EXP_PRIO, VGPOSP_GEMM_PRIO), the timing-only builds that give wrong
// results (-DVGPOSP_GEMM_EXP_NOVMWAIT / _NOBARRIER / _NOLOADS) and the reference-kernel switch
// (VGPOSP_GEMM_REF=1).  tools/build_variant.sh compiles it in place of gemm.hip into
// tools/variants/lib_NAME.so (loaded with VGPOSP_LIB=...) so the A/B scripts keep reproducing the
// numbers DESIGN.md quotes.  It includes the library's headers from vgposp_amd/csrc.
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
#include <cstdlib>
#include <type_traits>

#include "../../vgposp_amd/csrc/common.h"

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
  int prio;  // experiment (VGPOSP_GEMM_PRIO): 1 = s_setprio 1 for the second wave of each SIMD pair
};

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
  constexpr bool A_KC = !TA;  // A[m][k] is k-contiguous
  constexpr bool B_KC = TB;   // B[n][k] is k-contiguous
  __shared__ double smem[2 * 2 * TILE_ELEMS];  // [buf][A|B][tile]

  const int64_t m0 = (int64_t)blockIdx.y * GBM;
  const int64_t n0 = (int64_t)blockIdx.x * GBN;
  if (p.uplo_c == VGPOSP_LOWER && n0 > m0 + GBM - 1) return;  // tile entirely above diagonal

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
#ifndef VGPOSP_GEMM_STAGES
#define VGPOSP_GEMM_STAGES 2
#endif
#ifndef VGPOSP_GEMM_GROUP
#define VGPOSP_GEMM_GROUP 4
#endif
#ifndef VGPOSP_GEMM_OCC
#define VGPOSP_GEMM_OCC 2
#endif
constexpr int STAGES = VGPOSP_GEMM_STAGES;
constexpr int OPND_ELEMS = GBM * GBK;        // 2048 doubles = 16 KiB per operand per stage

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One 1-KiB wave-instruction ("piece" i = 0..15) of a 128-row x 16-k operand tile.
template <bool KC>
__device__ __forceinline__ void glds_piece(const double* base, int64_t ld, int64_t r0, int64_t k0,
                                           int64_t R, int64_t K, double* dst, int i, int lane) {
  {
    const double* src;
    if (KC) {
      const int row = 8 * i + (lane >> 3);
      const int kp = (lane & 7) ^ ((row & 15) >> 1);
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
  if (KC) return row * 16 + 2 * ((k >> 1) ^ ((row & 15) >> 1)) + (k & 1);
  return k * 128 + 2 * ((row >> 1) ^ ((k & 1) << 3)) + (row & 1);
}

__device__ __forceinline__ int tri_root(int64_t id) {
  int64_t t = (int64_t)((sqrt(8.0 * (double)id + 1.0) - 1.0) * 0.5);
  while ((t + 1) * (t + 2) / 2 <= id) ++t;
  while (t * (t + 1) / 2 > id) --t;
  return (int)t;
}

// CFG selects the tile shape (waves always in a (rows / 64 or 128) x 2 grid over the tile):
//   1 -> 128x128 tiles, 4 waves of 64x64 (4x4 fragments), STAGES-deep ring, 2 workgroups per CU;
//   2 -> 256x128 tiles, 4 waves of 128x64 (8x4 fragments, 128 accumulators in AGPRs), 3-stage
//        ring (144 KiB), 1 workgroup per CU;
//   3 -> 256x128 tiles, 8 waves of 64x64, 3-stage ring, 1 workgroup per CU: two waves per SIMD
//        as in 1, but 6 instead of 8 LDS-DMA pieces per wave per 64 MFMAs and a deeper ring.
template <int CFG> struct GemmCfg {
  static constexpr int NSUB = CFG == 1 ? 1 : 2;              // 128-row A sub-tiles
  static constexpr int NW = CFG == 3 ? 8 : 4;                // waves
  static constexpr int FI = CFG == 2 ? 8 : 4;                // 16-row fragments per wave
  static constexpr int NST = CFG == 1 ? STAGES : 3;          // ring depth
  static constexpr int OCC = CFG == 1 ? VGPOSP_GEMM_OCC : 1;  // workgroups per CU (launch bound)
};

template <bool TA, bool TB, bool TRIA, bool TRIB, int CFG>
__global__ __launch_bounds__(64 * GemmCfg<CFG>::NW, GemmCfg<CFG>::OCC) void gemm_glds_kernel(
    GemmParams p, int tiles_m, int tiles_n) {
  constexpr bool A_KC = !TA;
  constexpr bool B_KC = TB;
  constexpr int NSUB = GemmCfg<CFG>::NSUB, NW = GemmCfg<CFG>::NW, FI = GemmCfg<CFG>::FI;
  constexpr int NST = GemmCfg<CFG>::NST;
  constexpr int TBM = GBM * NSUB;                      // rows per tile
  constexpr int WROWS = 16 * FI;                       // rows per wave
  constexpr int SE = (NSUB + 1) * OPND_ELEMS;          // doubles per stage: A subs | B
  constexpr int PO = 16 / NW;                          // pieces per operand per wave
  constexpr int PPW = PO * (NSUB + 1);                 // pieces per wave per stage (8, 12 or 6)
  constexpr bool SPREAD = NST >= 3;                    // next-tile loads between the MFMAs
#if VGPOSP_GEMM_B128
  // b128 fragment reads (experiment): lane group fk covers k = 4 fk + s (s = 0..3), so a KC
  // operand's substeps 2h and 2h + 1 are one 16-byte pair; an MC operand's 16-byte pair is two
  // adjacent rows of one k, i.e. fragments 2g and 2g + 1 (rows 32 g + 2 x + {0, 1}).
  constexpr bool B128 = NST == 2;
#else
  constexpr bool B128 = false;
#endif
  constexpr bool A_IL = B128 && !A_KC, B_IL = B128 && !B_KC;  // row-interleaved fragments
  __shared__ __attribute__((aligned(16))) double smem[NST * SE];

  // Tile order.  Uniform-K launches: XCD-aware bijective remap (each XCD walks a contiguous range
  // of tiles, so neighbours share A rows / B columns in its L2).  A lower-triangular A (K range
  // grows with the row tile) must NOT hand contiguous ranges to XCDs — one XCD would get every
  // long tile — so it keeps the round-robin dispatch and walks row groups longest first.
  const int nwg = gridDim.x, bid = blockIdx.x;
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
    constexpr int GROUP = VGPOSP_GEMM_GROUP;  // row tiles per group: neighbours share A rows and B columns
    const int per_group = GROUP * tiles_n;
    const int g = wg / per_group, first = g * GROUP;
    const int gsize = min(GROUP, tiles_m - first);
    const int local = wg - g * per_group;
    ti = first + local % gsize;
    tj = local / gsize;
    if (TRIA && !TA) ti = tiles_m - 1 - ti;  // longest K ranges first
  }
  const int64_t m0 = (int64_t)ti * TBM, n0 = (int64_t)tj * GBN;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;
  if (p.prio == 1 && (NW == 8 ? wave >= 4 : (bid >> 3) & 1)) __builtin_amdgcn_s_setprio(1);

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
  kbeg = (kbeg / GBK) * GBK;
  if (kend < kbeg) kend = kbeg;
  const int T = (int)((kend - kbeg + GBK - 1) / GBK);
  const bool partial_last = ((kend - kbeg) % GBK) != 0;

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
    const int64_t k0 = kbeg + (int64_t)t * GBK;
    const int op = q / PO, j = wave * PO + q % PO;
    if (op < NSUB)
      glds_piece<A_KC>(p.A, p.lda, m0 + GBM * op, k0, p.m, p.k, st + op * OPND_ELEMS, j, lane);
    else
      glds_piece<B_KC>(p.B, p.ldb, n0, k0, p.n, p.k, st + NSUB * OPND_ELEMS, j, lane);
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
    static_assert(PPW == 8 || PPW == 12 || PPW == 6, "counted waits: 6, 8 or 12 pieces");
#ifdef VGPOSP_GEMM_EXP_NOVMWAIT  // timing experiment only: results are wrong
    if (false) {
#else
    if (after == 0) {
#endif
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
#ifndef VGPOSP_GEMM_EXP_NOBARRIER  // timing experiment only: results are wrong
    __builtin_amdgcn_s_barrier();
#endif
    // 3-stage ring: the next K-tile's pieces are spread over the k-slices below, between MFMAs
    // (issued back to back they park the wave for their issue cost; 8192^3 NT 63.3 -> 65.7 TF/s).
    // 2-stage ring: issued here, as early as possible — the tile is needed one K-step later.
#ifdef VGPOSP_GEMM_EXP_NOLOADS  // timing experiment only: no loads after the prologue
    const bool more = false;
#else
    const bool more = t + NST - 1 < T;
#endif
    if (!SPREAD && more) issue(t + NST - 1);

    const double* As = smem + (t % NST) * SE + ((wm * WROWS) / GBM) * OPND_ELEMS;
    const double* Bs = smem + (t % NST) * SE + NSUB * OPND_ELEMS;
    const int64_t k0 = kbeg + (int64_t)t * GBK;
    // masks only where needed: the last partial K-tile, and K-tiles that straddle the diagonal
    // of a triangular operand (k0 within 128 of the tile's first row / column)
    const bool mask = (partial_last && t == T - 1) || (TRIA && k0 < m0 + TBM && k0 + GBK > m0) ||
                      (TRIB && k0 < n0 + GBN && k0 + GBK > n0);
    if constexpr (B128) {
      // x[e][f]: substep 2h + e of fragment f; rb = the wave's first row of the operand image
      auto frags = [&](auto kc, const double* X, int rb, auto nf, int h, double (&x)[2][decltype(nf)::value]) {
        constexpr int F = decltype(nf)::value;
        if constexpr (decltype(kc)::value) {
#pragma unroll
          for (int f = 0; f < F; ++f) {
            const int r = rb + f * 16 + fr;
            const double2 v = *reinterpret_cast<const double2*>(X + r * 16 + 2 * ((2 * fk + h) ^ ((r & 15) >> 1)));
            x[0][f] = v.x;
            x[1][f] = v.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int k = 4 * fk + 2 * h + e;
#pragma unroll
            for (int g = 0; g < F / 2; ++g) {
              const int pr = (rb >> 1) + 16 * g + fr;
              const double2 v = *reinterpret_cast<const double2*>(X + k * 128 + 2 * (pr ^ ((k & 1) << 3)));
              x[e][2 * g] = v.x;
              x[e][2 * g + 1] = v.y;
            }
          }
        }
      };
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double a[2][FI], b[2][4];
        frags(std::integral_constant<bool, A_KC>{}, As, (wm * WROWS) % GBM, std::integral_constant<int, FI>{}, h, a);
        frags(std::integral_constant<bool, B_KC>{}, Bs, wn * 64, std::integral_constant<int, 4>{}, h, b);
        if (mask) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int64_t gk = k0 + 4 * fk + 2 * h + e;
#pragma unroll
            for (int i = 0; i < FI; ++i) {
              const int64_t gm = m0 + wm * WROWS + (A_IL ? 32 * (i >> 1) + 2 * fr + (i & 1) : i * 16 + fr);
              if (gk >= kend || (TRIA && (TA ? gm > gk : gk > gm))) a[e][i] = 0.0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int64_t gn = n0 + wn * 64 + (B_IL ? 32 * (j >> 1) + 2 * fr + (j & 1) : j * 16 + fr);
              if (gk >= kend || (TRIB && (TB ? gk > gn : gn > gk))) b[e][j] = 0.0;
            }
          }
        }
#ifdef VGPOSP_GEMM_EXP_PRIO
        __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[e][i], b[e][j], acc[i][j], 0, 0, 0);
#ifdef VGPOSP_GEMM_EXP_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
      }
    } else
#pragma unroll
    for (int ks = 0; ks < GBK / 4; ++ks) {
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
#pragma unroll
        for (int q = (ks * PPW) / 4; q < ((ks + 1) * PPW) / 4; ++q) issue_piece(t + NST - 1, q);
      }
#ifdef VGPOSP_GEMM_EXP_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
#ifdef VGPOSP_GEMM_EXP_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
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
            p.part[(int64_t)zsplit * p.m * p.n + row * p.n + col] = p.alpha * acc[i][j][r];
            continue;
          }
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
// "rs" path: one wave per SIMD, register-staged operands, 128x256 (FM = 4, FN = 8) or 256x128
// (FM = 8, FN = 4) tiles.  Each wave owns a (16 FM) x (16 FN) block of C: FM * FN = 32 f64 MFMA
// accumulators (256 registers, AGPRs), so one K-substep is 32 MFMAs (~2k cycles) against 6 LDS
// reads.  Per K-tile (16 deep) every thread issues FM + FN 16-byte global loads for the tile
// after next into registers, and writes the tile after this one from those registers to the other
// LDS buffer (one barrier per K-tile).  Zero-masking of triangular operands and of the K tail is
// applied in registers between the load and the LDS write, so the MFMA loop has no branches.
//
// LDS images (both read with ds_read_b128, both conflict-free for the b128 lane groups):
//   KC operand (stored [row][k]):  row-major [rows][16 k]; 16-byte pair P of row r at slot
//       P ^ ((r >> 1) & 5).  Lane (fr, fk) reads pair 2 fk + h: k = 4 fk + 2h, 4 fk + 2h + 1,
//       i.e. substeps 2h and 2h + 1 of k-map  k(s, fk) = 4 fk + s.
//   MC operand (stored [k][row]):  [16 k][rows]; lane (fr, fk) of substep s reads rows
//       32 g + 2 fr, 32 g + 2 fr + 1 of k-row 4 fk + s: fragment 2g holds the even rows and
//       fragment 2g + 1 the odd ones (the epilogue undoes the interleave).
// ---------------------------------------------------------------------------------------------
// sched_group_barrier patterns of gemm_rs_kernel (masks: 0x2 VALU, 0x8 MFMA, 0x20 VMEM read,
// 0x100 DS read, 0x200 DS write)
template <int R>
__device__ __forceinline__ void sgb_reads() {
  if constexpr (R > 0) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    sgb_reads<R - 1>();
  }
}
// MG MFMAs carrying one staged piece (mask VALU, LDS write, buffer load) and RD fragment reads
template <int MG, int RD>
__device__ __forceinline__ void sgb_group() {
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
  sgb_reads<RD>();
  if constexpr (MG - 4 - RD > 0) __builtin_amdgcn_sched_group_barrier(0x008, MG - 4 - RD, 0);
}
// after the barrier: RD reads under NM MFMAs
template <int RD, int NM>
__device__ __forceinline__ void sgb_tail() {
  if constexpr (RD > 0 && NM > 0) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    sgb_tail<RD - 1, NM - 1>();
  } else if constexpr (RD > 0) {
    __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
  } else if constexpr (NM > 0) {
    __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
  }
}

__device__ double g_rs_sink[64];  // dropped epilogue stores of gemm_rs_kernel

template <bool KC>
__device__ __forceinline__ int rs_row(int f, int x) {  // operand row of fragment f, lane index x
  return KC ? 16 * f + x : 32 * (f >> 1) + 2 * x + (f & 1);
}

template <int FM, int FN, bool TA, bool TB, bool TRIA, bool TRIB>
__global__ __launch_bounds__(256, 1) void gemm_rs_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int BM = 32 * FM, BN = 32 * FN;
  constexpr bool A_KC = !TA, B_KC = TB;
  constexpr int AE = BM * 16, BE = BN * 16;  // doubles per operand per stage
  constexpr int SE = AE + BE;
  __shared__ __attribute__((aligned(16))) double smem[2 * SE];

  const int nwg = gridDim.x, bid = blockIdx.x;
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
    // tiles on or below the diagonal, row by row: row ti holds c(ti) = (BM ti + BM - 1) / BN + 1
    // column tiles; with BM = 2 BN that is 2 ti + 2 (cumulative ti (ti + 1)), with BN = 2 BM it
    // is ti / 2 + 1 (cumulative over row pairs u: u (u + 1))
    if (BM >= BN) {
      ti = tri_root(wg / 2);
      while ((int64_t)(ti + 1) * (ti + 2) <= wg) ++ti;
      while ((int64_t)ti * (ti + 1) > wg) --ti;
      tj = wg - ti * (ti + 1);
    } else {
      int u = tri_root(wg / 2);
      while ((int64_t)(u + 1) * (u + 2) <= wg) ++u;
      while ((int64_t)u * (u + 1) > wg) --u;
      const int rem = wg - u * (u + 1);
      ti = 2 * u + rem / (u + 1);
      tj = rem % (u + 1);
    }
  } else {
    constexpr int GROUP = 8;
    const int per_group = GROUP * tiles_n;
    const int g = wg / per_group, first = g * GROUP;
    const int gsize = min(GROUP, tiles_m - first);
    const int local = wg - g * per_group;
    ti = first + local % gsize;
    tj = local / gsize;
    if (TRIA && !TA) ti = tiles_m - 1 - ti;  // longest K ranges first
  }
  const int m0 = ti * BM, n0 = tj * BN;

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;

  int64_t kbeg = 0, kend = p.k;
  if (TRIA) {
    if (TA) kbeg = max(kbeg, (int64_t)m0);
    else kend = min(kend, (int64_t)m0 + BM);
  }
  if (TRIB) {
    if (TB) kend = min(kend, (int64_t)n0 + BN);
    else kbeg = max(kbeg, (int64_t)n0);
  }
  if (p.nsplit > 1) {
    kbeg = max(kbeg, (int64_t)zsplit * p.kchunk);
    kend = min(kend, (int64_t)(zsplit + 1) * p.kchunk);
  }
  kbeg = (kbeg / GBK) * GBK;
  if (kend < kbeg) kend = kbeg;
  const int T = (int)((kend - kbeg + GBK - 1) / GBK);

  // ---- staging: FM pieces of A, FN of B per thread (buffer loads, out-of-range reads are 0) ----
  // piece e = t + 256 q.  KC: row e >> 3, pair e & 7.  MC: k-row e / (rows / 2), pair e % (rows / 2).
  // Every piece of an operand is the thread's first piece plus q times a fixed stride.  The resource is
  // rebuilt per K-tile: based at (tile row, k0) and sized to the tile's valid rows (KC) or k-rows
  // (MC), so rows past the matrix (KC) and the K tail (MC) read as zero.
  constexpr int AH = BM / 2, BH = BN / 2;  // MC pairs per k-row
  const int voffA = A_KC ? (int)(((t >> 3) * p.lda + 2 * (t & 7)) * 8)
                         : (int)(((t / AH) * p.lda + 2 * (t % AH)) * 8);
  const int voffB = B_KC ? (int)(((t >> 3) * p.ldb + 2 * (t & 7)) * 8)
                         : (int)(((t / BH) * p.ldb + 2 * (t % BH)) * 8);
  const int strA = A_KC ? (int)(32 * p.lda * 8) : (int)((256 / AH) * p.lda * 8);
  const int strB = B_KC ? (int)(32 * p.ldb * 8) : (int)((256 / BH) * p.ldb * 8);
  // LDS write offsets (doubles) of piece 0; piece q is + 512 q
  const int lA = A_KC ? (t >> 3) * 16 + 2 * ((t & 7) ^ (((t >> 3) >> 1) & 5)) : (t / AH) * BM + 2 * (t % AH);
  const int lB = AE + (B_KC ? (t >> 3) * 16 + 2 * ((t & 7) ^ (((t >> 3) >> 1) & 5))
                            : (t / BH) * BN + 2 * (t % BH));
  const int K = (int)p.k;
  const int nrowsA = min(BM, (int)p.m - m0), nrowsB = min(BN, (int)p.n - n0);
  auto rsrc = [&](bool isA, int tile) {
    const bool kc = isA ? A_KC : B_KC;
    const double* X = isA ? p.A : p.B;
    const int64_t ld = isA ? p.lda : p.ldb;
    const int r0 = isA ? m0 : n0, nrows = isA ? nrowsA : nrowsB;
    const int k0 = (int)kbeg + GBK * tile;
    const double* base;
    int64_t rec;
    // the range ends at the last valid element (not at the end of its row: the operand may be
    // the bottom-right block of a larger matrix, with nothing allocated after it)
    const int R = (int)(isA ? p.m : p.n);
    if (kc) {
      base = X + (int64_t)r0 * ld + min(k0, K);
      rec = nrows > 0 ? (int64_t)(nrows - 1) * ld + (K - min(k0, K)) : 0;
    } else {
      const int kr = min(GBK, K - min(k0, K));
      base = X + (int64_t)min(k0, K) * ld + r0;
      rec = kr > 0 ? (int64_t)(kr - 1) * ld + (R - r0) : 0;
    }
    // uniform by construction; readfirstlane keeps the resource in SGPRs (a VGPR resource
    // would turn every load into a waterfall loop)
    const uint64_t ba = reinterpret_cast<uint64_t>(base);
    const uint64_t bu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(ba >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ba);
    const int nrec = __builtin_amdgcn_readfirstlane((int)max(rec * 8, (int64_t)0));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(bu), (short)0, nrec, 0x00020000);
  };
  double2 stg[FM + FN];
  auto gload = [&](int q, int tile) {
    const bool isA = q < FM;
    const int qq = isA ? q : q - FM;
    // the whole offset in the VGPR: the buffer range check does not include soffset
    stg[q] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                                             rsrc(isA, tile), (isA ? voffA : voffB) + qq * (isA ? strA : strB),
                                             0, 0));
  };
  auto gload_all = [&](int tile) {
#pragma unroll
    for (int q = 0; q < FM + FN; ++q) gload(q, tile);
  };
  // pieces [q0, q1) of tile `tile`: mask in registers, write to LDS buffer buf
  auto gstore = [&](int q, int tile, int buf) {
    const bool isA = q < FM;
    const int qq = isA ? q : q - FM;
    const bool kc = isA ? A_KC : B_KC;
    const bool tri = isA ? TRIA : TRIB;
    const int rows = isA ? BM : BN;
    const int r0 = isA ? m0 : n0;
    const int k0 = (int)kbeg + GBK * tile;
    double2 v = stg[q];
    if (isA) {  // alpha is folded into A
      v.x *= p.alpha;
      v.y *= p.alpha;
    }
    if (kc) {  // elements (row, gk), (row, gk + 1); K tail; triangle: zero for k > row
      const int gk = k0 + 2 * (t & 7);
      const int row = r0 + (t >> 3) + 32 * qq;
      const bool ok0 = gk < K && (!tri || gk <= row);
      const bool ok1 = gk + 1 < K && (!tri || gk + 1 <= row);
      v.x = ok0 ? v.x : 0.0;
      v.y = ok1 ? v.y : 0.0;
    } else if (tri) {  // elements (gk, col), (gk, col + 1); triangle: zero for col > k
      const int half = rows / 2;
      const int gk = k0 + t / half + (256 / half) * qq;
      const int col = r0 + 2 * (t % half);
      v.x = col <= gk ? v.x : 0.0;
      v.y = col + 1 <= gk ? v.y : 0.0;
    }
    *reinterpret_cast<double2*>(smem + buf * SE + (isA ? lA : lB) + 512 * qq) = v;
  };

  // ---- fragments ----
  // KC: fa[h][i] = pair 2 fk + h of row (wave rows + 16 i + fr)  -> substeps 2h (.x), 2h + 1 (.y)
  // MC: fa[s & 1][g] = rows 32 g + 2 fr (+1) of k-row 4 fk + s  -> fragments 2g (.x), 2g + 1 (.y)
  constexpr int NA = A_KC ? FM : FM / 2, NB_ = B_KC ? FN : FN / 2;
  double2 fa[2][NA], fb[2][NB_];
  auto read_kc = [&](double2* dst, int n, const double* base, int row0, int h) {
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const int row = row0 + 16 * i + fr;
      const int P = 2 * fk + h;
      dst[i] = *reinterpret_cast<const double2*>(base + row * 16 + 2 * (P ^ ((row >> 1) & 5)));
    }
  };
  auto read_mc = [&](double2* dst, int n, const double* base, int rows, int row0, int s) {
#pragma unroll
    for (int g = 0; g < n; ++g)
      dst[g] = *reinterpret_cast<const double2*>(base + (4 * fk + s) * rows + row0 + 32 * g + 2 * fr);
  };
  // reads for substep s of the tile in buffer buf (KC operands only on even substeps)
  auto read_frags = [&](int s, int buf) {
    const double* As = smem + buf * SE;
    const double* Bs = As + AE;
    if (A_KC) {
      if ((s & 1) == 0) read_kc(fa[s >> 1], FM, As, wm * 16 * FM, s >> 1);
    } else {
      read_mc(fa[s & 1], FM / 2, As, BM, wm * 16 * FM, s);
    }
    if (B_KC) {
      if ((s & 1) == 0) read_kc(fb[s >> 1], FN, Bs, wn * 16 * FN, s >> 1);
    } else {
      read_mc(fb[s & 1], FN / 2, Bs, BN, wn * 16 * FN, s);
    }
  };
  auto aval = [&](int s, int i) -> double {
    if (A_KC) return (s & 1) ? fa[s >> 1][i].y : fa[s >> 1][i].x;
    return (i & 1) ? fa[s & 1][i >> 1].y : fa[s & 1][i >> 1].x;
  };
  auto bval = [&](int s, int j) -> double {
    if (B_KC) return (s & 1) ? fb[s >> 1][j].y : fb[s >> 1][j].x;
    return (j & 1) ? fb[s & 1][j >> 1].y : fb[s & 1][j >> 1].x;
  };

  // ---- C: beta (0 or 1, the host guarantees it) is applied by starting the accumulators at
  // beta * C; the epilogue stores them straight from the accumulator registers.  Elements outside
  // C (or above the diagonal of a lower C) get an out-of-range buffer offset: their loads read 0
  // and their stores are dropped. ----
  const bool lower = p.uplo_c == VGPOSP_LOWER;
  double* dst;
  int ldd;
  if (p.nsplit > 1) {
    dst = p.part + (int64_t)zsplit * p.m * p.n;
    ldd = (int)p.n;
  } else {
    dst = p.C;
    ldd = (int)p.ldc;
  }
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dst + (int64_t)m0 * ldd + n0), (short)0, 0x7ffffff8, 0x00020000);
  const bool with_beta = p.nsplit == 1 && p.beta != 0.0;
  auto coff = [&](int i, int j, int r) {
    const int cl = wn * 16 * FN + rs_row<B_KC>(j, fr);
    const int rl = wm * 16 * FM + rs_row<A_KC>(i, fk + 4 * r);
    const bool ok = m0 + rl < p.m && n0 + cl < p.n && (!lower || n0 + cl <= m0 + rl);
    return ok ? (rl * ldd + cl) * 8 : (int)0x7ffffff8;
  };
  dbl4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[i][j][r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                      rc, with_beta ? coff(i, j, r) : 0x7ffffff8, 0, 0));

  auto mfmas = [&](int s, int j0, int j1) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = j0; j < j1; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(aval(s, i), bval(s, j), acc[i][j], 0, 0, 0);
  };

  // prologue: tile 0 -> LDS buffer 0, tile 1 in flight, substep-0 fragments of tile 0
  gload_all(0);
#pragma unroll
  for (int q = 0; q < FM + FN; ++q) gstore(q, 0, 0);
  gload_all(1);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  read_frags(0, 0);

  // Schedule (enforced with sched_group_barrier, fenced per phase with sched_barrier): substeps
  // 0..2 interleave their 32 MFMAs with the next substep's fragment reads and a third of the
  // staged pieces (mask, LDS write of tile it+1, buffer load of tile it+2); substep 3 runs 3/4 of
  // its MFMAs, then the LDS barrier, then the first fragment reads of the next tile under the
  // last quarter of its MFMAs.
  constexpr int NQ = FM + FN;  // staged pieces, spread over substeps 0..2
  constexpr int MF = FM * FN;  // MFMAs per substep
  // LDS reads issued for substep s (s = 0 is issued at the end of the previous tile)
  constexpr int RD_KC_A = A_KC ? FM : 0, RD_KC_B = B_KC ? FN : 0;
  constexpr int RD_MC = (A_KC ? 0 : FM / 2) + (B_KC ? 0 : FN / 2);
  for (int it = 0; it < T; ++it) {
    const int buf = it & 1;
    auto phase = [&](auto S_) {
      constexpr int s = decltype(S_)::value;
      read_frags(s + 1, buf);
      constexpr int q0 = (s * NQ) / 3, q1 = ((s + 1) * NQ) / 3;
#pragma unroll
      for (int q = q0; q < q1; ++q) {
        gstore(q, it + 1, buf ^ 1);
        gload(q, it + 2);
      }
      mfmas(s, 0, FN);
      // MF MFMAs in np groups; each group carries one piece (VALU, LDS write, VMEM) and a share
      // of the reads (the remainder goes with the last group)
      constexpr int nrd = RD_MC + (((s + 1) & 1) == 0 ? RD_KC_A + RD_KC_B : 0);
      constexpr int np = q1 - q0, mg = MF / np, rg = nrd / np, rlast = nrd - rg * (np - 1);
      static_assert(mg >= 4 + rlast, "MFMA groups too small for the interleave");
      sgb_group<mg, rg>();
      if constexpr (np > 2) sgb_group<mg, rg>();
      if constexpr (np > 3) sgb_group<mg, rg>();
      if constexpr (np > 4) sgb_group<mg, rg>();
      static_assert(np <= 5, "at most 5 pieces per phase");
      sgb_group<mg, rlast>();
      __builtin_amdgcn_sched_barrier(0);
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    mfmas(3, 0, FN - FN / 4);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    read_frags(0, buf ^ 1);
    mfmas(3, FN - FN / 4, FN);
    sgb_tail<RD_MC + RD_KC_A + RD_KC_B, FM * (FN / 4)>();
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: plain stores; an element outside C (or above the diagonal of a lower C) is
  // sent to a per-lane sink slot instead (no branches around the accumulator reads).  (A buffer
  // store of an accumulator element miscompiles: every element of the dbl4 was stored from its
  // first register pair.) ----
  double* const cbase = dst + (int64_t)m0 * ldd + n0;
  double* const sink = g_rs_sink + lane;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int off = coff(i, j, r);
        double* const ptr = off != (int)0x7ffffff8 ? cbase + off / 8 : sink;
        *ptr = acc[i][j][r];
      }
}

template <int CFG, bool TA, bool TB, bool TRIA, bool TRIB>
static void launch_one(dim3 g1, hipStream_t stream, const GemmParams& p, int tm, int tn) {
  hipLaunchKernelGGL((gemm_glds_kernel<TA, TB, TRIA, TRIB, CFG>), g1, dim3(64 * GemmCfg<CFG>::NW),
                     0, stream, p, tm, tn);
}

// every (transa, transb, tri_a, tri_b) combination: the kernel's K-range and mask logic is
// generic in the four flags.  The 256x128 configurations are instantiated for plain operands only.
template <int CFG, bool TA, bool TB>
static void launch_tri(dim3 g1, hipStream_t stream, const GemmParams& p, int tm, int tn, int tri_a,
                       int tri_b) {
  if (CFG != 1 || (!tri_a && !tri_b)) return launch_one<CFG, TA, TB, false, false>(g1, stream, p, tm, tn);
  if (tri_a && tri_b) return launch_one<1, TA, TB, true, true>(g1, stream, p, tm, tn);
  if (tri_a) return launch_one<1, TA, TB, true, false>(g1, stream, p, tm, tn);
  launch_one<1, TA, TB, false, true>(g1, stream, p, tm, tn);
}

template <int FM, int FN, bool TA, bool TB>
static void launch_rs_tri(dim3 g1, hipStream_t stream, const GemmParams& p, int tm, int tn, int tri_a,
                          int tri_b) {
  if (tri_a && tri_b)
    hipLaunchKernelGGL((gemm_rs_kernel<FM, FN, TA, TB, true, true>), g1, dim3(256), 0, stream, p, tm, tn);
  else if (tri_a)
    hipLaunchKernelGGL((gemm_rs_kernel<FM, FN, TA, TB, true, false>), g1, dim3(256), 0, stream, p, tm, tn);
  else if (tri_b)
    hipLaunchKernelGGL((gemm_rs_kernel<FM, FN, TA, TB, false, true>), g1, dim3(256), 0, stream, p, tm, tn);
  else
    hipLaunchKernelGGL((gemm_rs_kernel<FM, FN, TA, TB, false, false>), g1, dim3(256), 0, stream, p, tm, tn);
}

template <int FM, int FN>
static void launch_rs(dim3 g1, hipStream_t stream, const GemmParams& p, int tm, int tn, int transa,
                      int transb, int tri_a, int tri_b) {
  if (!transa && !transb) launch_rs_tri<FM, FN, false, false>(g1, stream, p, tm, tn, tri_a, tri_b);
  else if (!transa) launch_rs_tri<FM, FN, false, true>(g1, stream, p, tm, tn, tri_a, tri_b);
  else if (!transb) launch_rs_tri<FM, FN, true, false>(g1, stream, p, tm, tn, tri_a, tri_b);
  else launch_rs_tri<FM, FN, true, true>(g1, stream, p, tm, tn, tri_a, tri_b);
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
                                                                 int lower) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= m * n) return;
  const int64_t row = e / n, col = e - row * n;
  if (lower && col > row) return;
  double v = 0.0;
  for (int z = 0; z < nsplit; ++z) v += part[(int64_t)z * m * n + e];
  double* c = C + row * ldc + col;
  if (beta != 0.0) v += beta * *c;
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

// splits for the n == 1 paths: about 2048 waves in flight, >= 2048 (rows) / 256 (transposed)
// K elements per split
static int gemv_splits(int64_t m, int64_t k, int transa) {
  int64_t s = transa ? ceil_div(2048 * 64, std::max<int64_t>(m, 1)) : ceil_div(2048, m);
  s = std::min<int64_t>(s, transa ? k / 256 : k / 2048);
  return (int)std::max<int64_t>(std::min<int64_t>(s, 4096), 1);
}

int g_fast_gemm = [] {  // 0 forces the register-staged reference kernel (VGPOSP_GEMM_REF=1)
  const char* e = getenv("VGPOSP_GEMM_REF");
  return e && e[0] == '1' ? 0 : 1;
}();
// 256x128 configurations (gemm_glds_kernel CFG 2 / 3) only on request, VGPOSP_GEMM_CFG=2 or 3,
// for full-C launches with at least two rounds of workgroups (measurements in DESIGN.md §4).
static const int g_prio = [] {
  const char* e = getenv("VGPOSP_GEMM_PRIO");
  return e ? atoi(e) : 0;
}();
static const int g_cfg = [] {
  const char* e = getenv("VGPOSP_GEMM_CFG");
  return (e && (e[0] == '2' || e[0] == '3')) ? e[0] - '0' : 1;
}();

// one-wave-per-SIMD register-staged kernel (gemm_rs_kernel): VGPOSP_GEMM_RS=1 -> 128x256 tiles,
// 2 -> 256x128 tiles, 0 -> off
static const int g_rs = [] {
  const char* e = getenv("VGPOSP_GEMM_RS");
  return e ? atoi(e) : 0;
}();

static bool aligned16(const void* ptr, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(ptr) % 16 == 0) && (ld % 2 == 0);
}

int gemm_launch_split(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                      const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                      double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, int nsplit,
                      double* part, hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
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
               g_prio};
  const int va = aligned16(A, lda), vb = aligned16(B, ldb);
  const bool even = (m % 2 == 0) && (n % 2 == 0) && (k % 2 == 0) && k > 0;
  // rs kernel: 32-bit buffer offsets (256 rows x ld x 8 bytes < 2^31), beta folded into the
  // accumulator start (0 or 1 only)
  const int64_t ldmax = (nsplit > 1 && part != nullptr) ? std::max(std::max(lda, ldb), n) : std::max(std::max(lda, ldb), ldc);
  const bool rs_ok = m < (1 << 30) && n < (1 << 30) && k < (1 << 30) && ldmax < (1 << 20) &&
                     (beta == 0.0 || beta == 1.0);
  if (va && vb && even && g_fast_gemm && g_rs && rs_ok) {
    const int FM = g_rs == 2 ? 8 : 4, FN = 12 - FM, BM = 32 * FM, BN = 32 * FN;
    const int tm = (int)ceil_div(m, BM), tn = (int)ceil_div(n, BN);
    int64_t nblk = (int64_t)tm * tn;
    if (uplo_c == VGPOSP_LOWER) {
      if (BM >= BN) nblk = (int64_t)tm * (tm + 1);
      else {
        nblk = 0;
        for (int i = 0; i < tm; ++i) nblk += i / 2 + 1;
      }
    }
    const double outs = (uplo_c == VGPOSP_LOWER) ? 0.5 * (double)m * (double)(m + 1) : (double)m * n;
    const double fl = 2.0 * (double)k * outs * ((tri_a && tri_b) ? (1.0 / 3.0) : (tri_a || tri_b) ? 0.5 : 1.0);
    if (nsplit > 1 && part != nullptr) {
      p.nblk = (int)nblk;
      p.kchunk = ceil_div(ceil_div(k, nsplit), GBK) * GBK;
      p.nsplit = (int)ceil_div(k, p.kchunk);
      p.part = part;
    }
    ProfScope ps("gemm_f64", stream, fl,
                 8.0 * ((double)m * k + (double)k * n + (beta != 0.0 ? 2.0 : 1.0) * outs));
    static const bool shapes = getenv("VGPOSP_PROF_SHAPES") != nullptr;
    char shape_name[96];
    if (shapes && prof_on())
      snprintf(shape_name, sizeof(shape_name), "gemm:%lldx%lldx%lld:%c%c%c%c%c:s%d", (long long)m,
               (long long)n, (long long)k, transa ? 'T' : 'N', transb ? 'T' : 'N',
               uplo_c == VGPOSP_LOWER ? 'L' : 'F', tri_a ? 'a' : '-', tri_b ? 'b' : '-', p.nsplit);
    ProfScope pshape(shape_name, stream, fl, 0.0, shapes && prof_on());
    dim3 g1((unsigned)(nblk * p.nsplit));
    if (FM == 4) launch_rs<4, 8>(g1, stream, p, tm, tn, transa, transb, tri_a, tri_b);
    else launch_rs<8, 4>(g1, stream, p, tm, tn, transa, transb, tri_a, tri_b);
    VG_LAUNCH_CHECK();
    static const bool dbg_sync = getenv("VGPOSP_GEMM_SYNC") != nullptr;  // debugging aid
    if (dbg_sync) {
      const hipError_t e = hipStreamSynchronize(stream);
      if (e != hipSuccess) {
        fprintf(stderr, "gemm_rs fault: m=%lld n=%lld k=%lld ta=%d tb=%d uplo=%d tri=%d%d lda=%lld ldb=%lld ldc=%lld "
                "beta=%g splits=%d A=%p B=%p C=%p\n", (long long)m, (long long)n, (long long)k, transa, transb,
                uplo_c, tri_a, tri_b, (long long)lda, (long long)ldb, (long long)ldc, beta, p.nsplit, (const void*)A,
                (const void*)B, (void*)C);
        set_error("gemm_rs fault: %s", hipGetErrorString(e));
        return VGPOSP_E_HIP;
      }
    }
    if (p.nsplit > 1) {
      hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)ceil_div(m * n, 256)), dim3(256),
                         0, stream, m, n, p.nsplit, part, beta, C, ldc, uplo_c == VGPOSP_LOWER);
      VG_LAUNCH_CHECK();
    }
    return 0;
  }
  if (va && vb && even && g_fast_gemm) {
    // 256x128 tiles for full-C launches with at least two rounds of workgroups, on request
    const int cfg = (uplo_c == VGPOSP_FULL && g_cfg > 1 && !tri_a && !tri_b &&
                     ceil_div(m, 2 * GBM) * ceil_div(n, GBN) >= 512) ? g_cfg : 1;
    const int tm = (int)ceil_div(m, GBM * (cfg == 1 ? 1 : 2)), tn = (int)ceil_div(n, GBN);
    const int64_t nblk = (uplo_c == VGPOSP_LOWER) ? (int64_t)tm * (tm + 1) / 2 : (int64_t)tm * tn;
    const double outs = (uplo_c == VGPOSP_LOWER) ? 0.5 * (double)m * (double)(m + 1) : (double)m * n;
    // algorithmic flops: a triangular operand halves the useful products
    const double fl = 2.0 * (double)k * outs * ((tri_a && tri_b) ? (1.0 / 3.0) : (tri_a || tri_b) ? 0.5 : 1.0);
    if (nsplit > 1 && part != nullptr) {
      p.nblk = (int)nblk;
      p.kchunk = ceil_div(ceil_div(k, nsplit), GBK) * GBK;
      p.nsplit = (int)ceil_div(k, p.kchunk);
      p.part = part;
    }
    ProfScope ps("gemm_f64", stream, fl,
                 8.0 * ((double)m * k + (double)k * n + (beta != 0.0 ? 2.0 : 1.0) * outs));
    // optional per-shape breakdown (VGPOSP_PROF_SHAPES=1): "gemm:MxNxK:flags:splits"
    static const bool shapes = getenv("VGPOSP_PROF_SHAPES") != nullptr;
    char shape_name[96];
    if (shapes && prof_on())
      snprintf(shape_name, sizeof(shape_name), "gemm:%lldx%lldx%lld:%c%c%c%c%c:s%d", (long long)m,
               (long long)n, (long long)k, transa ? 'T' : 'N', transb ? 'T' : 'N',
               uplo_c == VGPOSP_LOWER ? 'L' : 'F', tri_a ? 'a' : '-', tri_b ? 'b' : '-', p.nsplit);
    ProfScope pshape(shape_name, stream, fl, 0.0, shapes && prof_on());
    dim3 g1((unsigned)(nblk * p.nsplit));
    if (cfg == 2) launch_glds<2>(g1, stream, p, tm, tn, transa, transb, tri_a, tri_b);
    else if (cfg == 3) launch_glds<3>(g1, stream, p, tm, tn, transa, transb, tri_a, tri_b);
    else launch_glds<1>(g1, stream, p, tm, tn, transa, transb, tri_a, tri_b);
    VG_LAUNCH_CHECK();
    if (p.nsplit > 1) {
      hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)ceil_div(m * n, 256)), dim3(256),
                         0, stream, m, n, p.nsplit, part, beta, C, ldc, uplo_c == VGPOSP_LOWER);
      VG_LAUNCH_CHECK();
    }
    return 0;
  }
  dim3 grid((unsigned)ceil_div(n, GBN), (unsigned)ceil_div(m, GBM));
  const double outs = (uplo_c == VGPOSP_LOWER) ? 0.5 * (double)m * (double)(m + 1) : (double)m * n;
  ProfScope ps("gemm_f64", stream, 2.0 * (double)k * outs,
               8.0 * ((double)m * k + (double)k * n + (beta != 0.0 ? 2.0 : 1.0) * outs));
  if (!transa && !transb) hipLaunchKernelGGL((gemm_ref_kernel<false, false>), grid, dim3(256), 0, stream, p, va, vb);
  else if (!transa && transb) hipLaunchKernelGGL((gemm_ref_kernel<false, true>), grid, dim3(256), 0, stream, p, va, vb);
  else if (transa && !transb) hipLaunchKernelGGL((gemm_ref_kernel<true, false>), grid, dim3(256), 0, stream, p, va, vb);
  else hipLaunchKernelGGL((gemm_ref_kernel<true, true>), grid, dim3(256), 0, stream, p, va, vb);
  VG_LAUNCH_CHECK();
  return 0;
}

int gemm_launch(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, hipStream_t stream) {
  return gemm_launch_split(transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, uplo_c,
                           tri_a, tri_b, 1, nullptr, stream);
}

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
  // VGP step, 16 tiles of a 512^3 product on 16 CUs): up to 8 splits, at least 64 deep — each
  // split's 128x128 partial costs 256 KB of HBM traffic, about the time of 64 K-steps on one CU.
  const int64_t deep = k / 512;
  s = std::min<int64_t>(s, deep >= 8 ? deep : std::min<int64_t>(8, k / 64));
  return (int)std::max<int64_t>(s, 1);
}

int gemm_auto_splits(int64_t m, int64_t n, int64_t k, int uplo_c, int transa) {
  return auto_splits(m, n, k, uplo_c, transa);
}

}  // namespace vgposp

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


// ---------------------------------------------------------------------------------------------
// Round 5 hygiene: the explicitly sequenced K-loop (formerly -DVGPOSP_GEMM_ASM=1/2 and
// -DVGPOSP_GEMM_ACC_AGPR=1 inside vgposp_amd/csrc/gemm.hip's gemm_glds_body).  Measured slower
// than the compiler-scheduled loop (profiles/r3_gemm_asm_ab.txt); NOT BUILT.  The helpers, then
// the loop as it sat in the kernel body in front of the default loop:
// ---- explicitly sequenced K-loop (VGPOSP_GEMM_ASM) -------------------------------------------
// Every LDS fragment read, LDS-DMA piece, MFMA, counter wait and barrier of the main loop is its
// own `asm volatile` statement, so the issue order is the one written below (volatile asm is never
// reordered against volatile asm); the compiler only places the address arithmetic between them.
// The fragments of k-slice s + 1 are read while slice s is multiplied (two fragment sets), so a
// wave never waits on LDS latency inside a K-tile.  The compiler's waitcnt pass does not see into
// inline asm: every wait is explicit, and a wait takes the fragments it guards as in/out operands
// so that no use (mask, MFMA) can be scheduled above it.
#ifndef VGPOSP_GEMM_ASM
#define VGPOSP_GEMM_ASM 0
#endif

template <int OFF>
__device__ __forceinline__ double ds_rd(uint32_t addr) {
  double v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

__device__ __forceinline__ void lgkm_wait0(double (&a)[4], double (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]),
                 "+v"(b[3]));
}

#ifndef VGPOSP_GEMM_ACC_AGPR
#define VGPOSP_GEMM_ACC_AGPR 0
#endif
// VGPOSP_GEMM_ACC_AGPR: accumulators (srcC / vdst) in AGPRs, so the MFMA's 8-register srcC read
// and result write do not share the architectural VGPR file with the fragment loads
__device__ __forceinline__ void mfma_asm(dbl4& c, double a, double b) {
#if VGPOSP_GEMM_ACC_AGPR
  asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
#else
  asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
#endif
}

// One LDS-DMA piece: 64 lanes x 16 bytes from src (per lane) to LDS [lds, lds + 1 KiB).
__device__ __forceinline__ void dma_asm(const double* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(lds)
               : "memory", "m0");
}

template <bool KC>
__device__ __forceinline__ const double* glds_src(const double* base, int64_t ld, int64_t r0,
                                                  int64_t k0, int64_t R, int64_t K, int i, int lane) {
  if (KC) {
    const int row = 8 * i + (lane >> 3);
    const int kp = (lane & 7) ^ ((row & 15) >> 1);
    const int64_t gr = min(r0 + row, R - 1);
    const int64_t gk = min(k0 + 2 * kp, K - 2);
    return base + gr * ld + gk;
  }
  const int p = lane ^ ((i & 1) << 3);
  const int64_t gk = min(k0 + i, K - 1);
  const int64_t gc = min(r0 + 2 * p, R - 2);
  return base + gk * ld + gc;
}

// Fragments 0..3 of one operand for one k-slice: fragment 2q + p at base[p] + q * D bytes
// (D = 4096 for a k-contiguous image, 256 for a row-contiguous one).
template <bool KC>
__device__ __forceinline__ void rd_frags(uint32_t b0, uint32_t b1, double (&f)[4]) {
  constexpr int D = KC ? 4096 : 256;
  f[0] = ds_rd<0>(b0);
  f[1] = ds_rd<0>(b1);
  f[2] = ds_rd<D>(b0);
  f[3] = ds_rd<D>(b1);
}


#if VGPOSP_GEMM_ASM
  static_assert(NST == 2 && NSUB == 1 && FI == 4 && PPW == 8, "sequenced loop: 2-stage 128x128");
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  // per-lane byte offsets (within a stage) of fragments 0 and 1 of each k-slice
  uint32_t ab[4][2], bb[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      ab[ks][q] = 8 * frag_off<A_KC>((wm * WROWS) % GBM + q * 16 + fr, ks * 4 + fk);
      bb[ks][q] = 8 * (NSUB * OPND_ELEMS + frag_off<B_KC>(wn * 64 + q * 16 + fr, ks * 4 + fk));
    }
  // ASM = 1: each K-tile starts with the counted wait + barrier.  ASM = 2: the barrier sits
  // before the tile's LAST k-slice, whose fragments are already in registers, and the next tile's
  // slice-0 reads and the tile-after-next's DMA pieces are issued behind it, so the barrier skew
  // and the LDS latency of the tile change hide under that slice's 16 MFMAs.
  constexpr bool XT = VGPOSP_GEMM_ASM >= 2;
  auto dma_piece = [&](int tt, int q) {  // piece q (0..7) of this wave for K-tile tt
    const int op = q / PO, jj = wave * PO + q % PO;
    const int64_t kk = kbeg + (int64_t)tt * GBK;
    const double* src = op == 0 ? glds_src<A_KC>(gA, p.lda, m0, kk, p.m, p.k, jj, lane)
                                : glds_src<B_KC>(gB, p.ldb, n0, kk, p.n, p.k, jj, lane);
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        (int)(lds0 + (uint32_t)(((tt & 1) * SE + op * OPND_ELEMS + jj * 128) * 8)));
    dma_asm(src, dst);
  };
  double fa[2][4], fb[2][4];
  if (XT && T > 0) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    rd_frags<A_KC>(lds0 + ab[0][0], lds0 + ab[0][1], fa[0]);
    rd_frags<B_KC>(lds0 + bb[0][0], lds0 + bb[0][1], fb[0]);
    if (T > 1) {
#pragma unroll
      for (int q = 0; q < PPW; ++q) dma_piece(1, q);
    }
  }
  for (int t = 0; t < T; ++t) {
    const uint32_t sb = lds0 + (uint32_t)((t & 1) * SE * 8);
    const uint32_t nb = lds0 + (uint32_t)(((t + 1) & 1) * SE * 8);
    const bool more = t + 1 < T;
    const int64_t k0 = kbeg + (int64_t)t * GBK;
    const bool mask = (partial_last && t == T - 1) || (TRIA && k0 < m0 + TBM && k0 + GBK > m0) ||
                      (TRIB && k0 < n0 + GBN && k0 + GBK > n0);
    if (!XT) {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      rd_frags<A_KC>(sb + ab[0][0], sb + ab[0][1], fa[0]);
      rd_frags<B_KC>(sb + bb[0][0], sb + bb[0][1], fb[0]);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = ks & 1;
      lgkm_wait0(fa[c], fb[c]);
      if (mask) {
        const int64_t gk = k0 + ks * 4 + fk;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t gm = m0 + wm * WROWS + i * 16 + fr;
          if (gk >= kend || (TRIA && (TA ? gm > gk : gk > gm))) fa[c][i] = 0.0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t gn = n0 + wn * 64 + j * 16 + fr;
          if (gk >= kend || (TRIB && (TB ? gk > gn : gn > gk))) fb[c][j] = 0.0;
        }
      }
      if (ks < 3) {
        rd_frags<A_KC>(sb + ab[ks + 1][0], sb + ab[ks + 1][1], fa[c ^ 1]);
        rd_frags<B_KC>(sb + bb[ks + 1][0], sb + bb[ks + 1][1], fb[c ^ 1]);
      } else if (XT && more) {
        // every wave has its tile-t fragments in registers and its tile-(t+1) pieces landed
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        rd_frags<A_KC>(nb + ab[0][0], nb + ab[0][1], fa[0]);
        rd_frags<B_KC>(nb + bb[0][0], nb + bb[0][1], fb[0]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          mfma_asm(acc[i][j], fa[c][i], fb[c][j]);
          if (!XT) {
            // the next K-tile's 8 pieces of this wave: one per 4 MFMAs of slices 0 and 1
            if (ks < 2 && j == 0 && more) dma_piece(t + 1, ks * 4 + i);
          } else {
            // the tile-after-next's pieces into the buffer tile t just released: one per 2 MFMAs
            // of the last slice
            if (ks == 3 && (j & 1) == 0 && t + 2 < T) dma_piece(t + 2, i * 2 + (j >> 1));
          }
        }
    }
  }
  // f64 MFMA results are read by VALU below: cover the XDL write -> VALU read hazard, which the
  // compiler's hazard recognizer cannot see through inline asm
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  if (false)
#endif
