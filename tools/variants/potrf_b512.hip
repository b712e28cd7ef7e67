// VARIANT (round 6, measured and not kept): potrf.hip with the fused 512-block
// factor-and-invert kernel (potrf_block512_kernel).  Build: SRC=../../tools/variants/potrf_b512.hip
// tools/build_potrf_variant.sh b512
// Recursive Cholesky (lower, in place) and recursive triangular inverse, built so that nearly all
// flops land in large-K fp64 MFMA GEMMs (gemm.hip):
//
//   potrf_rec(A):  L11 = potrf_rec(A11)
//                  A21 <- A21 L11^-T           trsm_rec: leaves multiply by the saved 128x128
//                                              diagonal-block inverses, inner steps are GEMMs
//                  A22 -= A21 A21^T (lower)    SYRK with K = n1 ~ n/2
//                  L22 = potrf_rec(A22)
//   trtri_rec(L):  X11 = trtri_rec(L11), X22 = trtri_rec(L22)
//                  W   = L21 X11               TRMM (X11 lower)        K = n1
//                  X21 = -X22 W                TRMM (X22 lower)        K = n2
// Leaves (<= 128) are factored and inverted in LDS by one workgroup (potrf_leaf_kernel); their
// inverses are kept in the workspace for the trsm leaves and the trtri leaves.
//
// Replaces the Eigen LLT that tf.linalg.cholesky runs inside tfd.GaussianProcess.log_prob
// (gp_functions.py:166-172, main.py:105) and, through L^-1, the per-candidate SVD pinv of
// placement_algorithm2.denominator (placement_algorithm2.py:399-413).
// The strictly upper triangle is never read or written.
#include "common.h"

namespace vgposp {

int gemm_launch_split(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                      const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                      double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, int nsplit,
                      double* part, hipStream_t stream);
int gemm_auto_splits(int64_t m, int64_t n, int64_t k, int uplo_c, int transa);
void gemm_set_abort(const int* flag);
int gemm_launch_batched(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                        const double* A, int64_t lda, int64_t sA, const double* B, int64_t ldb,
                        int64_t sB, double beta, double* C, int64_t ldc, int64_t sC, int uplo_c,
                        int tri_a, int tri_b, int nsplit, double* part, int64_t sP, int batch,
                        hipStream_t stream);

constexpr int NB = 128;        // leaf size (== GEMM tile, so trsm leaves are in place)


// ---------------------------------------------------------------------------------------------
// Blocked leaf: Cholesky + inverse of a jb x jb (jb <= 128) block in LDS, one workgroup of 4 waves.
// Left-looking over 16-column panels: all waves bring the panel up to date with MFMA
// (A[c0:, c0:c0+16] -= L[c0:, :c0] L[c0:c0+16, :c0]^T), then wave 0 factors the whole tall panel
// in registers (a lane per row, broadcasts through SGPRs), which also solves the rows below the
// diagonal block — two barriers per panel.  The inverse follows: the 16x16 diagonal blocks by
// forward substitution (all blocks at once), then X_ij = -X_ii * sum_{k=j}^{i-1} L_ik X_kj as
// independent block-column chains per wave (two MFMA chains per 16x16 tile, the first chain's
// accumulator feeding the second directly as its B operand).  X (strictly lower) lives transposed
// in the upper triangle of the LDS image, diag(X) = 1 / diag(L) in rdiag.  jb is padded to a
// multiple of 16 with an identity block.
// ---------------------------------------------------------------------------------------------
typedef double dbl4 __attribute__((ext_vector_type(4)));

// (The phase-stamped build of this file, -DVGPOSP_STAMPS with vgposp_potrf_stamps, is
// tools/variants/potrf_stamps.hip; tools/leaf_probe.py reads it.)

constexpr int LW = 16;                 // panel width
constexpr int LP2 = NB + 4;            // LDS pitch (doubles)
constexpr int LEAF_THREADS = 256;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Broadcast a double from a (wave-uniform) lane.
__device__ __forceinline__ double readlane_d(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ int leaf_tri_root(int t) {
  int r = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  return r;
}

// 1 / sqrt(d) from the hardware estimate plus two Newton steps (full fp64 precision, not
// correctly rounded): 7 dependent VALU ops instead of the ~25 of sqrt() followed by 1.0 / x.
__device__ __forceinline__ double rsqrt_nr(double d) {
  double r = __builtin_amdgcn_rsq(d);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double e = fma(-d * r, r, 1.0);
    r = fma(0.5 * r, e, r);
  }
  return r;
}

// Register panel factor, one wave: lane l owns panel rows r0 = c0 + l (D0) and, when the panel is
// taller than 64, r1 = c0 + 64 + l (D1); register k holds column c0 + k.  The pivot and
// L[c0 + k][c0 + c] (k > c) are broadcast through SGPRs (v_readlane), so a column costs one
// reciprocal square root and 2 (15 - c) readlanes + FMAs with no LDS traffic and no barrier.  Rows
// below the 16x16 diagonal block come out solved (the panel TRSM is part of the elimination).
// (Measured alternative: 64-bit DPP row_newbcast folded into v_fmac_f64 is ~12x slower on gfx950.)
template <bool TALL>
__device__ __forceinline__ void leaf_panel(double (&D0)[LW], double (&D1)[LW], int lane, int c0,
                                           int jb, int64_t col0, int* info, double* rdiag,
                                           double* pcol) {
  double my_d = 1.0, my_inv = 1.0;  // lane c < 16 keeps column c's pivot and its reciprocal
#pragma unroll
  for (int c = 0; c < LW; ++c) {
    const double d = readlane_d(D0[c], c);
    const double inv = rsqrt_nr(d), piv = d * inv;
    if (lane == c) {
      my_d = d;
      my_inv = inv;
    }
    D0[c] = lane == c ? piv : D0[c] * inv;
    if (TALL) D1[c] *= inv;
    // L[c0 + k][c0 + c] for k > c, the scaled column on lanes k: through the wave's LDS slot (one
    // store, then broadcast reads issued together) instead of a v_readlane pair per k
    if (c + 1 < LW) {
      if (lane < LW) pcol[lane] = D0[c];
      wave_sync();
#pragma unroll
      for (int k = c + 1; k < LW; ++k) {
        const double lkc = pcol[k];
        D0[k] -= D0[c] * lkc;
        if (TALL) D1[k] -= D1[c] * lkc;
      }
      wave_sync();  // (the next column's store waits for these reads)
    }
  }
  // statuses and reciprocals once per panel (no branches inside the column steps)
  const unsigned long long bad = __ballot(lane < LW && c0 + lane < jb && !(my_d > 0.0));
  if (lane < LW) rdiag[c0 + lane] = my_inv;
  if (lane == 0 && bad) atomicCAS(info, 0, (int)(col0 + c0 + __ffsll((long long)bad)));
}

// The leaf's body, for workgroup `bx` of a batched launch (potrf_leaf_kernel) or for the diagonal
// tiles of the fused 512-block kernel below.  Uses the kernel's dynamic LDS (leaf_shmem()).
__device__ __forceinline__ void leaf_body(double* A, int64_t lda, int jb, int64_t col0, int invert,
                                          double* linv, double* diag_out, int* info,
                                          int64_t stride_a, int64_t stride_linv,
                                          int64_t stride_diag, const int bx) {
  extern __shared__ double L[];  // [NB][LP2]
  __shared__ double rdiag[NB];
  __shared__ double XD[(NB / LW) * LW * LW];  // dense diagonal blocks of L^-1
  __shared__ double pcol[LW];                  // wave 0's panel column broadcast (leaf_panel)
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  // invert: 0 = factor (lower(A) <- L), 1 = factor and invert (lower(A) <- L^-1), 2 = A already
  // holds L: only form L^-1 into linv (A is read, never written; the TRSM leaves).
  const bool factor = invert != 2;
  A += bx * stride_a;
  info += bx;
  if (linv) linv += (int64_t)bx * stride_linv;
  if (diag_out) diag_out += (int64_t)bx * (stride_diag < 0 ? jb : stride_diag);
  const int JP = (jb + LW - 1) & ~(LW - 1), NP = JP / LW;
  // Block load: thread t reads column t & 127 of rows 2u + (t >> 7), 16 loads in flight per
  // batch from clamped (always valid) addresses; a loop with one load per iteration waited on each
  // load in turn (64 round trips, about half of the leaf's time).
  for (int u0 = 0; u0 < NB / 2; u0 += 16) {
    double v[16];
    const int c = t & (NB - 1), cc = min(c, jb - 1);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = 2 * (u0 + u) + (t >> 7);
      v[u] = A[(int64_t)min(r, jb - 1) * lda + cc];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = 2 * (u0 + u) + (t >> 7);
      if (r < JP && c <= r) L[r * LP2 + c] = (r < jb && c < jb) ? v[u] : (r == c ? 1.0 : 0.0);
    }
  }
  if (!factor)
    for (int c = t; c < JP; c += LEAF_THREADS) rdiag[c] = c < jb ? 1.0 / A[(int64_t)c * lda + c] : 1.0;
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;

  // Left-looking over 16-column panels:
  //   A[c0:, c0:c0+16] -= L[c0:, :c0] L[c0:c0+16, :c0]^T   (MFMA, 16-row tiles over the 4 waves)
  //   factor the tall panel A[c0:, c0:c0+16] in wave 0's registers (leaf_panel)
  for (int p = 0; factor && p < NP; ++p) {
    const int c0 = p * LW;
    if (p > 0) {
      const int nrt = NP - p;
      for (int tt = wave; tt < nrt; tt += 4) {
        const int r0 = c0 + LW * tt;
        dbl4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < c0; k0 += LW) {  // c0 is a multiple of 16: loads issued together
          double a[4], b[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            a[s4] = L[(r0 + fr) * LP2 + k0 + 4 * s4 + fk];
            b[s4] = L[(c0 + fr) * LP2 + k0 + 4 * s4 + fk];
          }
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s4], b[s4], acc, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) L[(r0 + fk + 4 * reg) * LP2 + c0 + fr] -= acc[reg];
      }
      __syncthreads();
    }
    if (wave == 0) {
      const int r0 = c0 + lane, r1 = c0 + 64 + lane;
      const bool tall = JP - c0 > 64;
      double D0[LW], D1[LW];
#pragma unroll
      for (int k = 0; k < LW; ++k) {
        D0[k] = r0 < JP ? L[r0 * LP2 + c0 + k] : 0.0;
        D1[k] = (tall && r1 < JP) ? L[r1 * LP2 + c0 + k] : 0.0;
      }
      if (tall) leaf_panel<true>(D0, D1, lane, c0, jb, col0, info, rdiag, pcol);
      else leaf_panel<false>(D0, D1, lane, c0, jb, col0, info, rdiag, pcol);
#pragma unroll
      for (int k = 0; k < LW; ++k) {
        if (r0 < JP && (lane >= LW || k <= lane)) L[r0 * LP2 + c0 + k] = D0[k];
        if (tall && r1 < JP) L[r1 * LP2 + c0 + k] = D1[k];
      }
    }
    __syncthreads();
  }

  if (invert || linv) {
    // Diagonal-block inverses, all blocks at once: lane group fk of wave w inverts block
    // b = 4 fk + w, lane fr its column by forward substitution (x[k] = 0 for k < column).  Kept
    // dense in XD (zeros above the diagonal) for branch-free MFMA operands, and strictly lower
    // transposed into the block's upper triangle of L for the output pass.
    {
      const int b = 4 * fk + wave, j = fr, b0 = b * LW;
      if (b < NP) {
        double x[LW];
#pragma unroll
        for (int i = 0; i < LW; ++i) {
          double s = 0.0;
#pragma unroll
          for (int k = 0; k < i; ++k) s += L[(b0 + i) * LP2 + b0 + k] * x[k];
          x[i] = i < j ? 0.0 : (i == j ? rdiag[b0 + i] : -rdiag[b0 + i] * s);
          XD[b * LW * LW + i * LW + j] = x[i];
        }
#pragma unroll
        for (int i = 0; i < LW; ++i)
          if (i > j) L[(b0 + j) * LP2 + b0 + i] = x[i];
      }
    }
    __syncthreads();
    // Off-diagonal blocks, one block column per chain: X_ij = -X_ii sum_{k=j}^{i-1} L_ik X_kj for
    // i = j+1 .. NP-1 depends only on block column j, so a wave owns whole columns (j and
    // NP-1-j: balanced work for NP <= 8) and needs wave-level ordering only.
    for (int h = 0; h < 2; ++h) {
      const int j = h == 0 ? wave : NP - 1 - wave;
      if (wave > NP - 1 - wave || (h == 1 && j == wave)) break;
      const int j0 = j * LW;
      const double* xjj = XD + j * LW * LW;
      for (int i = j + 1; i < NP; ++i) {
        const int i0 = i * LW;
        const double* li = L + (i0 + fr) * LP2 + fk;
        dbl4 S = {0.0, 0.0, 0.0, 0.0};
        {
          double a[4], b[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            a[s4] = li[j0 + 4 * s4];
            b[s4] = xjj[(4 * s4 + fk) * LW + fr];
          }
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            S = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s4], b[s4], S, 0, 0, 0);
        }
        const double* xcol = L + (j0 + fr) * LP2 + fk;  // X_kj, k > j, stored transposed
        for (int k0 = j0 + LW; k0 < i0; k0 += LW) {
          double a[4], b[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            a[s4] = li[k0 + 4 * s4];
            b[s4] = xcol[k0 + 4 * s4];
          }
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            S = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s4], b[s4], S, 0, 0, 0);
        }
        const double* xii = XD + i * LW * LW + fr * LW + fk;
        dbl4 X = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          X = __builtin_amdgcn_mfma_f64_16x16x4f64(xii[4 * s4], S[s4], X, 0, 0, 0);
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) L[(j0 + fr) * LP2 + i0 + fk + 4 * reg] = -X[reg];
        wave_sync();
      }
    }
    __syncthreads();
  }

  for (int e = t; e < NB * NB; e += LEAF_THREADS) {
    const int r = e / NB, c = e % NB;
    double x = 0.0;
    if (r < jb && c <= r) x = (r == c) ? rdiag[c] : L[c * LP2 + r];
    if (linv) linv[e] = x;
    if (factor && r < jb && c <= r) A[(int64_t)r * lda + c] = invert ? x : L[r * LP2 + c];
  }
  if (diag_out != nullptr) {
    for (int c = t; c < jb; c += LEAF_THREADS) diag_out[c] = L[c * LP2 + c];
  }
}

__global__ __launch_bounds__(LEAF_THREADS) void potrf_leaf_kernel(double* A, int64_t lda, int jb,
                                                                  int64_t col0, int invert,
                                                                  double* linv, double* diag_out,
                                                                  int* info, int64_t stride_a,
                                                                  int64_t stride_linv = NB * NB,
                                                                  int64_t stride_diag = -1,
                                                                  const int* abort = nullptr) {
  if (abort != nullptr && *abort != 0) return;  // an earlier pivot failed (early mode)
  leaf_body(A, lda, jb, col0, invert, linv, diag_out, info, stride_a, stride_linv, stride_diag,
            (int)blockIdx.x);
}

static size_t leaf_shmem() { return (size_t)NB * LP2 * sizeof(double); }

// A (jb x jb lower) <- linv (the saved leaf inverse); batch element blockIdx.y at the strides
__global__ __launch_bounds__(256) void copy_leaf_kernel(double* A, int64_t lda, int jb, const double* linv,
                                 int64_t sA = 0, int64_t sL = 0) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  A += blockIdx.y * sA;
  linv += blockIdx.y * sL;
  const int r = e / NB, c = e % NB;
  if (r < jb && c <= r) A[(int64_t)r * lda + c] = linv[e];
}

static int64_t split_point(int64_t n) {
  const int64_t nb = (n + NB - 1) / NB;
  return NB * (nb / 2);  // >= NB for n > NB
}

// Diagonal blocks of up to NBI columns (the recursion's blocks with NB < n <= NBI) are inverted
// as a whole right after they are factored.  The TRSMs below them are then one K <= 512
// triangular GEMM per block instead of K = 128 GEMMs against the 128x128 leaf inverses plus the
// updates between them, and the final inverse stops at 512 (a copy) instead of recursing to 128.
constexpr int NBI = 4 * NB;

// ---------------------------------------------------------------------------------------------
// Fused 512-block: factor AND invert one NBI x NBI diagonal block in ONE launch (the recursion's
// `whole` blocks).  The launch-per-step chain it replaces (4 leaves, ~10 split-K GEMMs and their
// reductions, the block's trtri recursion and copies: ~35 dependent launches, ~0.87 ms per block,
// 128 blocks in the 65k step and on every rank at R > 1) becomes a right-looking tile DAG on a
// 4 x 4 grid of 128-tiles: one workgroup per lower tile (10), each owning its tile.
//   tile (i, j), i >= j:  A_ij -= sum_{k<j} L_ik L_jk^T   (NT, K = 128 j, waits for L_ik, L_jk)
//     i == j: the leaf (L_jj and Linv_jj, leaf_body)               -> posts L(j,j), LINV(j)
//     i >  j: L_ij = A_ij Linv_jj^T                       (waits LINV(j)) -> posts L(i,j)
//   then, i > j:  S = L_ij Linv_jj + sum_{j<k<i} L_ik X_kj            (waits L(i,k), X(k,j))
//                 X_ij = -Linv_ii S                         (waits LINV(i)) -> posts X(i,j)
// Outputs as the chain: L in A's lower block (the strict upper of A never written), the 4 leaf
// inverses in linv, X = the block's inverse in xblk (pitch NBI, zeros above the diagonal).
// Cross-workgroup hand-over: each tile's data is stored, every thread fences at agent scope, and
// thread 0 stores the flag with release semantics; a waiter's thread 0 polls with acquire loads
// (bounded: on timeout the launch records info = VG_B512_TIMEOUT and stops, it never hangs).  All
// 10 workgroups are resident at once (one per CU by LDS).  The flags are zeroed before every
// launch (vg_memset on the stream).
// ---------------------------------------------------------------------------------------------
constexpr int B512_T = NBI / NB;                 // 4 tiles per side
constexpr int B512_WG = B512_T * (B512_T + 1) / 2;  // 10 lower tiles
constexpr int B512_FLAGS = 32;                   // L: 0..9, LINV: 10..13, X: 14..19
constexpr int VG_B512_TIMEOUT = -1000;           // info on a hand-over timeout
constexpr int GK = 16;                           // K-tile of the tile GEMM
constexpr int TKC = GK + 2;                      // KC image pitch (doubles)
constexpr int TMC = NB + 16;                     // MC image pitch (doubles)
constexpr int TIMG = NB * TKC;                   // == GK * TMC == 2304 doubles
static_assert(NB * TKC == GK * TMC, "tile images must be the same size");

__device__ __forceinline__ int b512_lidx(int i, int j) { return i * (i + 1) / 2 + j; }
__device__ __forceinline__ int b512_flag_l(int i, int j) { return b512_lidx(i, j); }
__device__ __forceinline__ int b512_flag_linv(int j) { return B512_WG + j; }
__device__ __forceinline__ int b512_flag_x(int i, int j) { return B512_WG + B512_T + i * (i - 1) / 2 + j; }

__device__ __forceinline__ void b512_post(int* flags, int f) {
  __threadfence();  // this thread's tile stores, visible at agent scope
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flags + f, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// false on timeout (then info records it and the caller returns)
__device__ __forceinline__ bool b512_wait(int* flags, int f, int* info) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    int good = 1;
    for (long it = 0; __hip_atomic_load(flags + f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0;
         ++it) {
      if (it > (1L << 24)) {  // far beyond any legitimate wait (the whole launch is < 1 ms)
        good = 0;
        atomicCAS(info, 0, VG_B512_TIMEOUT);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    ok = good;
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return ok != 0;
}

// acc (this wave's 64 x 64 quarter of a 128 x 128 tile) += A (128 x 128, stored [r][k], lda) times
// B: B_KC -> B stored [c][k] (A B^T), else B stored [k][c] (A B).  Register-staged, the next
// K-tile's loads issued before the current one's MFMAs; sm = 2 x 2 tile images.
template <bool B_KC>
__device__ __forceinline__ void b512_gemm(dbl4 (&acc)[4][4], const double* A, int64_t lda,
                                          const double* B, int64_t ldb, double* sm) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fk = lane >> 4;
  typedef double d2 __attribute__((ext_vector_type(2)));
  d2 ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = t + 256 * it;
      ra[it] = *reinterpret_cast<const d2*>(A + (int64_t)(e >> 3) * lda + k0 + (e & 7) * 2);
      if (B_KC) rb[it] = *reinterpret_cast<const d2*>(B + (int64_t)(e >> 3) * ldb + k0 + (e & 7) * 2);
      else rb[it] = *reinterpret_cast<const d2*>(B + (int64_t)(k0 + (e >> 6)) * ldb + (e & 63) * 2);
    }
  };
  auto store = [&](double* img) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = t + 256 * it;
      *reinterpret_cast<d2*>(img + (e >> 3) * TKC + (e & 7) * 2) = ra[it];
      if (B_KC) *reinterpret_cast<d2*>(img + TIMG + (e >> 3) * TKC + (e & 7) * 2) = rb[it];
      else *reinterpret_cast<d2*>(img + TIMG + (e >> 6) * TMC + (e & 63) * 2) = rb[it];
    }
  };
  load(0);
  store(sm);
  __syncthreads();
  for (int k0 = 0, buf = 0; k0 < NB; k0 += GK, buf ^= 1) {
    const bool more = k0 + GK < NB;
    if (more) load(k0 + GK);
    const double* As = sm + buf * 2 * TIMG;
    const double* Bs = As + TIMG;
#pragma unroll
    for (int ks = 0; ks < GK / 4; ++ks) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[(wm * 64 + i * 16 + fr) * TKC + ks * 4 + fk];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = wn * 64 + j * 16 + fr, k = ks * 4 + fk;
        b[j] = B_KC ? Bs[c * TKC + k] : Bs[k * TMC + c];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(sm + (buf ^ 1) * 2 * TIMG);
    __syncthreads();
  }
}

__device__ __forceinline__ void b512_zero(dbl4 (&acc)[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};
}

// out (128 x 128, ld) = alpha acc + (accumulate ? out : 0); lower: only c <= r written
__device__ __forceinline__ void b512_store(const dbl4 (&acc)[4][4], double* out, int64_t ld,
                                           double alpha, bool accumulate, bool lower) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + fk + 4 * r, col = wn * 64 + j * 16 + fr;
        if (lower && col > row) continue;
        double* o = out + (int64_t)row * ld + col;
        const double v = alpha * acc[i][j][r];
        *o = accumulate ? *o + v : v;
      }
}

__global__ __launch_bounds__(LEAF_THREADS) void potrf_block512_kernel(
    double* A, int64_t lda, int64_t col0, double* linv, double* X, double* scratch, int* flags,
    int* info, double* diag_out, const int* abort) {
  if (abort != nullptr && *abort != 0) return;
  extern __shared__ double sm[];
  // tile of this workgroup: the diagonal ones first in the grid (they lead the DAG)
  int i, j;
  {
    const int b = blockIdx.x;
    if (b < B512_T) {
      i = j = b;
    } else {
      int q = b - B512_T;  // the 6 strictly lower tiles, row by row
      i = 1;
      while (q >= i) {
        q -= i;
        ++i;
      }
      j = q;
    }
  }
  double* Aij = A + (int64_t)i * NB * lda + j * NB;
  auto Lt = [&](int r, int c) { return A + (int64_t)r * NB * lda + c * NB; };
  auto Linv = [&](int c) { return linv + (int64_t)c * NB * NB; };
  dbl4 acc[4][4];
  // A_ij -= sum_{k<j} L_ik L_jk^T
  if (j > 0) {
    b512_zero(acc);
    for (int k = 0; k < j; ++k) {
      if (!b512_wait(flags, b512_flag_l(i, k), info)) return;
      if (i != j && !b512_wait(flags, b512_flag_l(j, k), info)) return;
      b512_gemm<true>(acc, Lt(i, k), lda, Lt(j, k), lda, sm);
    }
    b512_store(acc, Aij, lda, -1.0, true, i == j);
    __threadfence_block();
    __syncthreads();
  }
  if (i == j) {
    leaf_body(Aij, lda, NB, col0 + (int64_t)j * NB, 0, Linv(j),
              diag_out ? diag_out + (int64_t)j * NB : nullptr, info, 0, NB * NB, -1, 0);
    // X_jj = Linv_jj (zeros above), read back from this workgroup's own stores
    __threadfence_block();
    __syncthreads();
    for (int e = threadIdx.x; e < NB * NB; e += LEAF_THREADS)
      X[(int64_t)(j * NB + e / NB) * NBI + j * NB + e % NB] = Linv(j)[e];
    b512_post(flags, b512_flag_l(j, j));
    if (threadIdx.x == 0) __hip_atomic_store(flags + b512_flag_linv(j), 1, __ATOMIC_RELEASE,
                                             __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // L_ij = A_ij Linv_jj^T
  if (!b512_wait(flags, b512_flag_linv(j), info)) return;
  b512_zero(acc);
  b512_gemm<true>(acc, Aij, lda, Linv(j), NB, sm);
  b512_store(acc, Aij, lda, 1.0, false, false);
  b512_post(flags, b512_flag_l(i, j));
  // S = L_ij Linv_jj + sum_{j<k<i} L_ik X_kj  -> scratch
  b512_zero(acc);
  b512_gemm<false>(acc, Aij, lda, Linv(j), NB, sm);
  for (int k = j + 1; k < i; ++k) {
    if (!b512_wait(flags, b512_flag_l(i, k), info)) return;
    if (!b512_wait(flags, b512_flag_x(k, j), info)) return;
    b512_gemm<false>(acc, Lt(i, k), lda, X + (int64_t)k * NB * NBI + j * NB, NBI, sm);
  }
  double* S = scratch + (int64_t)b512_lidx(i, j) * NB * NB;
  b512_store(acc, S, NB, 1.0, false, false);
  __threadfence_block();
  __syncthreads();
  // X_ij = -Linv_ii S; the mirrored upper tile of X is zero
  if (!b512_wait(flags, b512_flag_linv(i), info)) return;
  b512_zero(acc);
  b512_gemm<false>(acc, Linv(i), NB, S, NB, sm);
  b512_store(acc, X + (int64_t)i * NB * NBI + j * NB, NBI, -1.0, false, false);
  for (int e = threadIdx.x; e < NB * NB; e += LEAF_THREADS)
    X[(int64_t)(j * NB + e / NB) * NBI + i * NB + e % NB] = 0.0;
  b512_post(flags, b512_flag_x(i, j));
}


struct Fact {
  int64_t lda;
  double* linv_all;  // ceil(n/NB) leaf inverses, NB*NB each, indexed by global column / NB
  double* work;      // trtri scratch, >= n1 * n2 doubles of the top split
  double* xinv;      // n x NBI: block inverses, rows [col0, col0 + nb) hold block col0's (or null)
  double* tmp;       // n x NBI: out-of-place TRSM leaf output (or null)
  double* diag_out;  // [n] or null
  int* info;
  double* part;      // split-K partials, part_elems doubles (or null)
  hipStream_t s;
  int64_t part_elems = 0;
  int* flags = nullptr;  // the fused 512-block's hand-over flags (B512_FLAGS ints) or null
  int64_t diag_n = 0;  // batched: diag_out stride (the matrix order)
  // batched recursion: `batch` matrices at stride sA, each with its own copy of the workspace
  // (stride sW doubles from ws0); a pointer into [ws0, ws0 + sW) is a workspace operand
  int batch = 1;
  int64_t sA = 0, sW = 0;
  const double* ws0 = nullptr;
  // stop early on a failed pivot: every later leaf / GEMM launch reads `info` on the device and
  // exits once it is set (no host synchronisation)
  bool early = false;
  double* leaf(int64_t col0) const { return linv_all + (col0 / NB) * NB * NB; }
  double* xblk(int64_t col0) const { return xinv + col0 * NBI; }
  int64_t stride(const void* p) const {
    const double* d = static_cast<const double*>(p);
    return (ws0 && d >= ws0 && d < ws0 + sW) ? sW : sA;
  }
};

// Split-K partials for the recursion's few-tile GEMMs (the 128..2048 levels: a 128^3 TRSM or SYRK
// is one 128x128 tile, i.e. one CU): up to 8 splits, bounded by the partials area.  One matrix:
// 64 MB.  At 16 MB the 2048-level SYRKs and TRSMs (136..256 tiles, K = 512..2048) ran unsplit on
// half the CUs or less; 64 MB splits them: the 65k step 0.3 % faster on one GPU, and each rank's
// factor share at R = 8 6 % faster (those levels are replicated on every rank;
// profiles/r6_splitk_part_ab.json, profiles/r6_sharded_step_part_ab.json).  Batched
// factorizations (the VGP step's M x M matrices, the multifrontal fronts) keep 16 MB per matrix:
// their products are at most 1024 wide, and the larger per-matrix workspace stride cost the C3
// step 0.05 ms (profiles/r6_vgp_part_ab.txt).
constexpr int64_t PART_ELEMS = 8 << 20;
constexpr int64_t PART_ELEMS_BATCHED = 2 << 20;

// C = alpha op(A) op(B) + beta C with the split count of vgposp_gemm_splitk, reduced to what the
// partials area holds.  In-place operands (C also read as A) are safe: the split kernels only
// write the partials, the reduction writes C after all of them.
static int pgemm(const Fact& f, int transa, int transb, int64_t m, int64_t n, int64_t k,
                 double alpha, const double* A, int64_t lda, const double* B, int64_t ldb,
                 double beta, double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b) {
  int sp = f.part ? gemm_auto_splits(m, n, k, uplo_c, transa) : 1;
  while (sp > 1 && (int64_t)sp * m * n > f.part_elems) --sp;
  if (f.batch > 1)
    return gemm_launch_batched(transa, transb, m, n, k, alpha, A, lda, f.stride(A), B, ldb,
                               f.stride(B), beta, C, ldc, f.stride(C), uplo_c, tri_a, tri_b, sp,
                               sp > 1 ? f.part : nullptr, f.sW, f.batch, f.s);
  return gemm_launch_split(transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, uplo_c,
                           tri_a, tri_b, sp, sp > 1 ? f.part : nullptr, f.s);
}

// dst (n x n lower, ldd) <- src (lower, lds); zero_upper: also zero dst's strict upper triangle
// (dst is then a full-matrix GEMM operand); otherwise dst's upper triangle is left untouched.
__global__ __launch_bounds__(256) void copy_lower_kernel(double* dst, int64_t ldd, const double* src, int64_t lds,
                                  int64_t n, int zero_upper, int64_t sd = 0, int64_t ss = 0) {
  const int64_t r = blockIdx.y;
  dst += blockIdx.z * sd;
  src += blockIdx.z * ss;
  for (int64_t c = threadIdx.x; c < n; c += blockDim.x) {
    if (c <= r) dst[r * ldd + c] = src[r * lds + c];
    else if (zero_upper) dst[r * ldd + c] = 0.0;
  }
}

static int copy_lower(const Fact& f, double* dst, int64_t ldd, const double* src, int64_t lds,
                      int64_t n, int zero_upper) {
  hipLaunchKernelGGL(copy_lower_kernel, dim3(1, (unsigned)n, (unsigned)f.batch), dim3(256), 0, f.s,
                     dst, ldd, src, lds, n, zero_upper, f.stride(dst), f.stride(src));
  VG_LAUNCH_CHECK();
  return 0;
}

static int leaf_factor(const Fact& f, double* A, int jb, int64_t col0, int invert) {
  ProfScope ps("potrf_diag", f.s, f.batch * 2.0 * jb * (double)jb * jb / 3.0,
               f.batch * 8.0 * jb * (double)jb * 2);
  // batched: one workgroup per matrix; element b's status is info[b], its diagonal diag_out + b n
  hipLaunchKernelGGL(potrf_leaf_kernel, dim3((unsigned)f.batch), dim3(LEAF_THREADS), leaf_shmem(),
                     f.s, A, f.lda, jb, col0, invert, f.leaf(col0),
                     f.diag_out ? f.diag_out + col0 : nullptr, f.info, f.sA, f.sW,
                     f.batch > 1 ? f.diag_n : (int64_t)-1, f.early ? f.info : nullptr);
  VG_LAUNCH_CHECK();
  return 0;
}

// B (m x nL, ldb) <- B L^-T, L = the nL x nL lower factor at Lp (already factored), col0 = global
// column of L's first column (locates the leaf / block inverses).  Mirrors potrf_rec's splits, so
// its leaves are exactly the factored leaves / blocks.
static int trsm_rec(const Fact& f, double* B, int64_t m, int64_t ldb, const double* Lp, int64_t nL,
                    int64_t col0, bool blocks) {
  int rc;
  if (nL <= NB) {
    // in place: the output is a single 128-wide column tile
    return pgemm(f, 0, 1, m, nL, nL, 1.0, B, ldb, f.leaf(col0), NB, 0.0, B, ldb, VGPOSP_FULL, 0, 0);
  }
  if (blocks && nL <= NBI) {
    // out of place (several output column tiles read the same rows): tmp = B X^T, X lower
    if ((rc = pgemm(f, 0, 1, m, nL, nL, 1.0, B, ldb, f.xblk(col0), NBI, 0.0, f.tmp, NBI,
                    VGPOSP_FULL, 0, 1)))
      return rc;
    for (int b = 0; b < f.batch; ++b)
      VG_HIP(vg_memcpy2d(B + b * f.stride(B), ldb * sizeof(double), f.tmp + b * f.sW,
                              NBI * sizeof(double), nL * sizeof(double), m,
                              hipMemcpyDeviceToDevice, f.s));
    return 0;
  }
  const int64_t a = split_point(nL), b = nL - a;
  if ((rc = trsm_rec(f, B, m, ldb, Lp, a, col0, blocks))) return rc;
  // B2 -= B1 Lb^T,  Lb = L[a:, :a]
  if ((rc = pgemm(f, 0, 1, m, b, a, -1.0, B, ldb, Lp + a * f.lda, f.lda, 1.0, B + a, ldb,
                  VGPOSP_FULL, 0, 0)))
    return rc;
  return trsm_rec(f, B + a, m, ldb, Lp + a * f.lda + a, b, col0 + a, blocks);
}

// Lower triangle of A (lda) holds L (leaf inverses saved) -> L^-1.  blocks: stop at the saved
// block inverses (n <= NBI) instead of recursing to the leaves.  done: subtrees of at most this
// order are already inverted (trtri_levels).
static int trtri_rec(const Fact& f, double* A, int64_t lda, int64_t n, int64_t col0, bool blocks,
                     int64_t done = 0) {
  if (n <= done) return 0;
  if (n <= NB) {
    ProfScope ps("trtri_leaf", f.s, 0.0, 8.0 * NB * NB * 2);
    hipLaunchKernelGGL(copy_leaf_kernel, dim3(NB * NB / 256, (unsigned)f.batch), dim3(256), 0, f.s,
                       A, lda, (int)n, f.leaf(col0), f.stride(A), f.sW);
    VG_LAUNCH_CHECK();
    return 0;
  }
  if (blocks && n <= NBI) return copy_lower(f, A, lda, f.xblk(col0), NBI, n, 0);
  const int64_t n1 = split_point(n), n2 = n - n1;
  int rc;
  double* A21 = A + n1 * lda;
  double* A22 = A21 + n1;
  if ((rc = trtri_rec(f, A, lda, n1, col0, blocks, done))) return rc;
  if ((rc = trtri_rec(f, A22, lda, n2, col0 + n1, blocks, done))) return rc;
  // W = L21 X11   (X11 lower, stored [k][j])
  if ((rc = pgemm(f, 0, 0, n2, n1, n1, 1.0, A21, lda, A, lda, 0.0, f.work, n1, VGPOSP_FULL, 0, 1)))
    return rc;
  // X21 = -X22 W  (X22 lower, stored [i][k])
  return pgemm(f, 0, 0, n2, n1, n2, -1.0, A22, lda, f.work, n1, 0.0, A21, lda, VGPOSP_FULL, 1, 0);
}

// Level-batched inverse of the small subtrees (single matrix, n = NBI 2^j): every node of order s
// (s = 1024 .. smax) is independent of the others of its level, so the level is TWO batched
// launches (W_i = L21_i X11_i, X21_i = -X22_i W_i over all n / s nodes at the stride
// s (lda + 1)) instead of two narrow launches per node (a 512^3 TRMM is 16 tiles on 16 CUs;
// measured in the 65k step: 992 launches at 10.6 TF/s).  The 512-block inverses are copied in
// one launch first.  Afterwards trtri_rec(done = smax) does the levels above.
static bool pow2_blocks(int64_t n) {
  const int64_t q = n / NBI;
  return n % NBI == 0 && q >= 2 && (q & (q - 1)) == 0;
}

static int trtri_levels(const Fact& f, double* A, int64_t lda, int64_t n, int64_t smax) {
  hipLaunchKernelGGL(copy_lower_kernel, dim3(1, NBI, (unsigned)(n / NBI)), dim3(256), 0, f.s, A,
                     lda, f.xinv, (int64_t)NBI, (int64_t)NBI, 0, (int64_t)NBI * (lda + 1),
                     (int64_t)NBI * NBI);
  VG_LAUNCH_CHECK();
  for (int64_t s = 2 * NBI; s <= smax && s <= n; s *= 2) {
    const int64_t h = s / 2, cnt = n / s, st = s * (lda + 1);
    int rc;
    // W_i = L21_i X11_i  (X11_i lower)
    if ((rc = gemm_launch_batched(0, 0, h, h, h, 1.0, A + h * lda, lda, st, A, lda, st, 0.0, f.work,
                                  h, h * h, VGPOSP_FULL, 0, 1, 1, nullptr, 0, (int)cnt, f.s)))
      return rc;
    // X21_i = -X22_i W_i  (X22_i lower)
    if ((rc = gemm_launch_batched(0, 0, h, h, h, -1.0, A + h * lda + h, lda, st, f.work, h, h * h,
                                  0.0, A + h * lda, lda, st, VGPOSP_FULL, 1, 0, 1, nullptr, 0,
                                  (int)cnt, f.s)))
      return rc;
  }
  return 0;
}

// The whole inverse after the factorization (blocks = the 512-block inverses are saved).
static int trtri_all(const Fact& f, double* A, int64_t lda, int64_t n, bool blocks) {
  if (f.batch == 1 && blocks && f.xinv != nullptr && pow2_blocks(n)) {
    constexpr int64_t SMAX = 4096;  // above it a node's launches fill the GPU on their own
    const int64_t smax = std::min<int64_t>(SMAX, n);
    if (int rc = trtri_levels(f, A, lda, n, smax)) return rc;
    return trtri_rec(f, A, lda, n, 0, blocks, smax);
  }
  return trtri_rec(f, A, lda, n, 0, blocks);
}

// Early stop (Fact::early): every leaf and GEMM launch of the recursion (and of the inverse after
// it) first reads `info` on the device and does nothing once a pivot has failed, so a failed
// factorization costs the work up to the failed pivot plus empty launches — with no host
// synchronisation (the call only enqueues work and can be captured into a graph).
struct AbortScope {
  explicit AbortScope(const int* flag) { gemm_set_abort(flag); }
  ~AbortScope() { gemm_set_abort(nullptr); }
};

// One NBI x NBI diagonal block factored and inverted by potrf_block512_kernel: the same outputs as
// the recursion below (L in place, the leaf inverses, the block inverse in xblk with zeros above).
static bool block512_ok(const Fact& f, const double* A) {
  return f.batch == 1 && f.flags != nullptr && f.tmp != nullptr && f.xinv != nullptr &&
         f.lda % 2 == 0 && reinterpret_cast<uintptr_t>(A) % 16 == 0;
}

static int block512(const Fact& f, double* A, int64_t col0) {
  ProfScope ps("potrf_block512", f.s, 2.0 * 2.0 * NBI * (double)NBI * NBI / 3.0,
               8.0 * NBI * (double)NBI * 3);
  VG_HIP(vg_memset(f.flags, 0, B512_FLAGS * sizeof(int), f.s));
  hipLaunchKernelGGL(potrf_block512_kernel, dim3(B512_WG), dim3(LEAF_THREADS), leaf_shmem(), f.s,
                     A, f.lda, col0, f.leaf(col0), f.xblk(col0), f.tmp, f.flags, f.info,
                     f.diag_out ? f.diag_out + col0 : nullptr, f.early ? f.info : nullptr);
  VG_LAUNCH_CHECK();
  return 0;
}

// blocks: form the inverse of every NB < n <= NBI diagonal block (for trsm / trtri above it).
static int potrf_rec(const Fact& f, double* A, int64_t n, int64_t col0, bool blocks) {
  if (n <= NB) return leaf_factor(f, A, (int)n, col0, 0);
  if (blocks && n == NBI && block512_ok(f, A)) return block512(f, A, col0);
  const bool whole = blocks && n <= NBI;
  const int64_t n1 = split_point(n), n2 = n - n1;
  int rc;
  double* A21 = A + n1 * f.lda;
  double* A22 = A21 + n1;
  const bool sub = blocks && !whole;  // inside a block the leaf-level path is used
  if ((rc = potrf_rec(f, A, n1, col0, sub))) return rc;
  if ((rc = trsm_rec(f, A21, n2, f.lda, A, n1, col0, sub))) return rc;
  if ((rc = pgemm(f, 0, 1, n2, n2, n1, -1.0, A21, f.lda, A21, f.lda, 1.0, A22, f.lda,
                  VGPOSP_LOWER, 0, 0)))
    return rc;
  if ((rc = potrf_rec(f, A22, n2, col0 + n1, sub))) return rc;
  if (!whole) return 0;
  // this block's inverse: X <- L (zero above the diagonal), then the leaf-level trtri in place
  double* X = f.xblk(col0);
  if ((rc = copy_lower(f, X, NBI, A, f.lda, n, 1))) return rc;
  return trtri_rec(f, X, NBI, n, col0, false);
}

size_t potrf_ws_bytes(int64_t n) {
  const int64_t leaves = (n + NB - 1) / NB;
  const int64_t n1 = n > NB ? split_point(n) : 0;
  const int64_t blk = n > NBI ? 2 * n * NBI : 0;  // xinv + tmp
  const int64_t part = n > NB ? PART_ELEMS : 0;
  return (size_t)(leaves * NB * NB + n1 * (n - n1) + blk + part + 64) * sizeof(double);
}

static int ensure_leaf_attr() {
  static bool attr_set = false;
  if (!attr_set) {
    VG_HIP(hipFuncSetAttribute((const void*)potrf_leaf_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)leaf_shmem()));
    VG_HIP(hipFuncSetAttribute((const void*)potrf_block512_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)leaf_shmem()));
    attr_set = true;
  }
  return 0;
}

static int trsm_left_rec(const Fact& f, const double* Lp, int64_t ldl, int64_t n, int64_t col0,
                         int trans, double* B, int64_t m, int64_t ldb);

static Fact make_fact(int64_t n, int64_t lda, void* ws, double* diag_out, int* info,
                      hipStream_t stream) {
  const int64_t leaves = (n + NB - 1) / NB;
  const int64_t n1 = n > NB ? split_point(n) : 0;
  double* base = static_cast<double*>(ws);
  double* work = base + leaves * NB * NB;
  const bool blocks = n > NBI;  // a whole problem <= NBI never needs block inverses
  double* xinv = blocks ? work + n1 * (n - n1) : nullptr;
  double* tmp = blocks ? xinv + n * NBI : nullptr;
  double* part = n > NB ? work + n1 * (n - n1) + (blocks ? 2 * n * NBI : 0) : nullptr;
  Fact f{lda, base, work, xinv, tmp, diag_out, info, part, stream};
  f.part_elems = PART_ELEMS;
  // in the workspace's 64-double tail after the partials (potrf_ws_bytes)
  if (part != nullptr) f.flags = reinterpret_cast<int*>(part + PART_ELEMS);
  return f;
}

// `batch` matrices at stride sA factored by ONE recursion: every launch covers all of them (the
// leaves as one workgroup per matrix, the GEMMs with a batch grid dimension), so B small
// factorizations cost the launches and the latency chain of one.  ws holds B copies of the
// single-matrix workspace.
// Per-matrix workspace of a batched factorization: the single-matrix layout with a 16 MB partials
// area (use_part) or none (large batches fill the GPU through the batch dimension; 16 MB of
// partials per matrix would not fit).
size_t potrf_ws_bytes_opt(int64_t n, bool use_part) {
  const int64_t part = n > NB ? (use_part ? PART_ELEMS_BATCHED : 0) : 0;
  return potrf_ws_bytes(n) - (size_t)((n > NB ? PART_ELEMS : 0) - part) * sizeof(double);
}

int potrf_batched(double* A, int64_t n, int64_t lda, int64_t sA, int batch, int invert,
                  double* diag_out, int* info, void* ws, hipStream_t stream, bool use_part) {
  if (int rc = ensure_leaf_attr()) return rc;
  if (n <= NB) {
    // one launch, one workgroup per matrix (no workspace needed)
    ProfScope ps("potrf_diag", stream, batch * 2.0 * n * (double)n * n / 3.0,
                 batch * 16.0 * n * (double)n);
    hipLaunchKernelGGL(potrf_leaf_kernel, dim3(batch), dim3(LEAF_THREADS), leaf_shmem(), stream, A,
                       lda, (int)n, (int64_t)0, invert, (double*)nullptr, diag_out, info, sA,
                       (int64_t)0, batch > 1 ? n : (int64_t)-1);
    VG_LAUNCH_CHECK();
    return 0;
  }
  const bool blocks = n > NBI;
  Fact f = make_fact(n, lda, ws, diag_out, info, stream);
  if (!use_part) f.part = nullptr;
  f.part_elems = PART_ELEMS_BATCHED;
  f.batch = batch;
  f.sA = sA;
  f.sW = (int64_t)(potrf_ws_bytes_opt(n, use_part) / sizeof(double));
  f.ws0 = static_cast<const double*>(ws);
  f.diag_n = n;
  int rc = potrf_rec(f, A, n, 0, blocks);
  if (rc || !invert) return rc;
  return trtri_rec(f, A, lda, n, 0, blocks);
}

int potrf_one(double* A, int64_t n, int64_t lda, int invert, double* diag_out, int* info,
              void* ws, hipStream_t stream, bool early) {
  if (int rc = ensure_leaf_attr()) return rc;
  const bool blocks = n > NBI;
  Fact f = make_fact(n, lda, ws, diag_out, info, stream);
  f.early = early;
  AbortScope scope(early ? info : nullptr);
  int rc = potrf_rec(f, A, n, 0, blocks);
  if (rc || !invert) return rc;
  return trtri_all(f, A, lda, n, blocks);
}

size_t partial_inverse_tmp_bytes(int64_t n, int64_t c0, int64_t c1) {
  return (size_t)((n - c1) * (c1 - c0) + NB * (c1 - c0)) * sizeof(double);
}

// After potrf_one(A, invert = 0) with the same ws (its leaf inverses): the lower part of columns
// [c0, c1) of A (rows >= c0) <- the same columns of L^-1, the rest of L untouched.  With
//   L = [L11 0; L21 L22] split at c1 (L11 = L[c0:c1, c0:c1], L21 = L[c1:, c0:c1]):
//   X11 = L11^-1 (in place, leaf-level trtri), X21 = -L22^-1 (L21 X11) (a GEMM and a TRSM through
//   tmp).  About the flops of this slab's share of a full trtri (a candidate-sharded rank forms
//   only the columns of L^-1 its candidates need).  c0 and c1 are multiples of 128, or c1 = n.
int partial_inverse(double* A, int64_t n, int64_t lda, int64_t c0, int64_t c1, double* tmp,
                    void* ws, hipStream_t s) {
  const int64_t w = c1 - c0, m2 = n - c1;
  if (w <= 0) return 0;
  Fact f = make_fact(n, lda, ws, nullptr, nullptr, s);
  f.tmp = tmp + m2 * w;  // the TRSM leaves' out-of-place scratch: NB x w
  int rc;
  double* A11 = A + c0 * lda + c0;
  if ((rc = trtri_rec(f, A11, lda, w, c0, false))) return rc;
  if (m2 == 0) return 0;
  double* L21 = A + c1 * lda + c0;
  // tmp = -L21 X11  (X11 lower, stored [k][j])
  if ((rc = pgemm(f, 0, 0, m2, w, w, -1.0, L21, lda, A11, lda, 0.0, tmp, w, VGPOSP_FULL, 0, 1)))
    return rc;
  // tmp <- L22^-1 tmp
  if ((rc = trsm_left_rec(f, A + c1 * lda + c1, lda, m2, c1, 0, tmp, w, w))) return rc;
  VG_HIP(vg_memcpy2d(L21, lda * sizeof(double), tmp, w * sizeof(double), w * sizeof(double),
                          m2, hipMemcpyDeviceToDevice, s));
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Pieces of a Cholesky distributed over R ranks that each hold the whole matrix (the host mirrors
// potrf_rec's splits, vgposp_amd/dist_cholesky.py).  ws is a potrf workspace for the WHOLE n, so the
// leaf / block inverses of every diagonal block sit at their global columns, exactly where the
// single-GPU recursion leaves them (partial_inverse and trsm_rec read them from there).
// ---------------------------------------------------------------------------------------------

// The diagonal block [col0, col0 + nb) factored in place by the single-GPU recursion.
int potrf_block(double* A, int64_t n, int64_t lda, int64_t col0, int64_t nb, int* info, void* ws,
                hipStream_t s) {
  if (int rc = ensure_leaf_attr()) return rc;
  Fact f = make_fact(n, lda, ws, nullptr, info, s);
  return potrf_rec(f, A + col0 * (lda + 1), nb, col0, n > NBI);
}

// Node (col0, nsub) split at n1: rows [r0, r1) of its panel (global rows col0 + n1 + r0 ...)
//   A21 <- A21 L11^-T
int potrf_panel(double* A, int64_t n, int64_t lda, int64_t col0, int64_t n1, int64_t r0,
                int64_t r1, void* ws, hipStream_t s) {
  Fact f = make_fact(n, lda, ws, nullptr, nullptr, s);
  double* A11 = A + col0 * (lda + 1);
  return trsm_rec(f, A11 + (n1 + r0) * lda, r1 - r0, lda, A11, n1, col0, n > NBI);
}

// Node (col0, nsub) split at n1, n2 = nsub - n1: rows [b0, b1) of the lower triangle of A22
//   A22 -= L21 L21^T   (the rectangle left of the band's diagonal square, then the square)
int potrf_trailing(double* A, int64_t n, int64_t lda, int64_t col0, int64_t n1, int64_t b0,
                   int64_t b1, void* ws, hipStream_t s) {
  Fact f = make_fact(n, lda, ws, nullptr, nullptr, s);
  double* L21 = A + (col0 + n1) * lda + col0;
  double* A22 = L21 + n1;
  const int64_t m = b1 - b0;
  int rc;
  if (m <= 0) return 0;
  if (b0 > 0 && (rc = pgemm(f, 0, 1, m, b0, n1, -1.0, L21 + b0 * lda, lda, L21, lda, 1.0,
                            A22 + b0 * lda, lda, VGPOSP_FULL, 0, 0)))
    return rc;
  return pgemm(f, 0, 1, m, m, n1, -1.0, L21 + b0 * lda, lda, L21 + b0 * lda, lda, 1.0,
               A22 + b0 * lda + b0, lda, VGPOSP_LOWER, 0, 0);
}

// Row block <-> contiguous buffer, for the all-gathers between the pieces above.  Rows [r0, r1),
// columns [c0, c1) (lower = 0), or the lower trapezoid: columns [c0, r] of row r (lower = 1,
// c0 <= r0 and c1 >= r1), packed row after row.
__global__ void pack_lower_kernel(double* A, int64_t lda, int64_t r0, int64_t c0, double* buf,
                                  int unpack) {
  const int64_t i = blockIdx.x, r = r0 + i;
  const int64_t len = r + 1 - c0;
  const int64_t off = i * (r0 + 1 - c0) + i * (i - 1) / 2;
  double* row = A + r * lda + c0;
  for (int64_t c = threadIdx.x; c < len; c += blockDim.x) {
    if (unpack) row[c] = buf[off + c];
    else buf[off + c] = row[c];
  }
}

int64_t pack_elems(int64_t r0, int64_t r1, int64_t c0, int64_t c1, int lower) {
  const int64_t m = r1 - r0;
  if (m <= 0) return 0;
  if (!lower) return m * (c1 - c0);
  return m * (r0 + 1 - c0) + m * (m - 1) / 2;
}

int pack_rows(double* A, int64_t lda, int64_t r0, int64_t r1, int64_t c0, int64_t c1, int lower,
              double* buf, int unpack, hipStream_t s) {
  const int64_t m = r1 - r0;
  if (m <= 0) return 0;
  if (!lower) {
    const size_t w = (size_t)(c1 - c0) * sizeof(double);
    if (unpack)
      VG_HIP(vg_memcpy2d(A + r0 * lda + c0, lda * sizeof(double), buf, w, w, m,
                              hipMemcpyDeviceToDevice, s));
    else
      VG_HIP(vg_memcpy2d(buf, w, A + r0 * lda + c0, lda * sizeof(double), w, m,
                              hipMemcpyDeviceToDevice, s));
    return 0;
  }
  hipLaunchKernelGGL(pack_lower_kernel, dim3((unsigned)m), dim3(256), 0, s, A, lda, r0, c0, buf,
                     unpack);
  VG_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Left-side triangular solve with a factor from vgposp_potrf_lower(invert = 0):
//   B (n x m) <- L^-1 B (trans = 0, forward)  or  L^-T B (trans = 1, backward)
// Recursion on the same splits as potrf_rec: the off-diagonal part is one GEMM per level
// (B2 -= L21 X1, or B1 -= L21^T X2), and the <= 128 diagonal blocks multiply by their inverses,
// formed up front by the leaf kernel's invert-only mode (all full blocks in one launch).
// ---------------------------------------------------------------------------------------------
static int trsm_left_rec(const Fact& f, const double* Lp, int64_t ldl, int64_t n, int64_t col0,
                         int trans, double* B, int64_t m, int64_t ldb) {
  int rc;
  if (n <= NB) {  // out of place (the n == 1 column path is a GEMV that may not alias), copy back
    if ((rc = pgemm(f, trans, 0, n, m, n, 1.0, f.leaf(col0), NB, B, ldb, 0.0, f.tmp, m,
                    VGPOSP_FULL, 0, 0)))
      return rc;
    VG_HIP(vg_memcpy2d(B, ldb * sizeof(double), f.tmp, m * sizeof(double), m * sizeof(double),
                            n, hipMemcpyDeviceToDevice, f.s));
    return 0;
  }
  const int64_t a = split_point(n), b = n - a;
  const double* L21 = Lp + a * ldl;
  if (!trans) {
    if ((rc = trsm_left_rec(f, Lp, ldl, a, col0, 0, B, m, ldb))) return rc;
    if ((rc = pgemm(f, 0, 0, b, m, a, -1.0, L21, ldl, B, ldb, 1.0, B + a * ldb, ldb, VGPOSP_FULL,
                    0, 0)))
      return rc;
    return trsm_left_rec(f, L21 + a, ldl, b, col0 + a, 0, B + a * ldb, m, ldb);
  }
  if ((rc = trsm_left_rec(f, L21 + a, ldl, b, col0 + a, 1, B + a * ldb, m, ldb))) return rc;
  if ((rc = pgemm(f, 1, 0, a, m, b, -1.0, L21, ldl, B + a * ldb, ldb, 1.0, B, ldb, VGPOSP_FULL, 0,
                  0)))
    return rc;
  return trsm_left_rec(f, Lp, ldl, a, col0, 1, B, m, ldb);
}

size_t trsm_ws_bytes(int64_t n, int64_t m) {
  const int64_t leaves = (n + NB - 1) / NB;
  return (size_t)(leaves * NB * NB + NB * m + PART_ELEMS_BATCHED + 64) * sizeof(double);
}

int trsm_left(const double* L, int64_t n, int64_t ldl, int trans, double* B, int64_t m,
              int64_t ldb, void* ws, hipStream_t s) {
  if (int rc = ensure_leaf_attr()) return rc;
  double* leaves = static_cast<double*>(ws);
  const int64_t nl = (n + NB - 1) / NB, nfull = n / NB;
  double* tmp = leaves + nl * NB * NB;
  double* part = tmp + NB * m;
  int* dummy = reinterpret_cast<int*>(part + PART_ELEMS_BATCHED);  // the invert-only leaves never write it
  {
    ProfScope ps("trtri_leaf", s, 0.0, 8.0 * NB * NB * 2 * nl);
    if (nfull > 0)
      hipLaunchKernelGGL(potrf_leaf_kernel, dim3((unsigned)nfull), dim3(LEAF_THREADS), leaf_shmem(),
                         s, const_cast<double*>(L), ldl, NB, (int64_t)0, 2, leaves,
                         (double*)nullptr, dummy, (int64_t)NB * (ldl + 1));
    if (nl > nfull)
      hipLaunchKernelGGL(potrf_leaf_kernel, dim3(1), dim3(LEAF_THREADS), leaf_shmem(), s,
                         const_cast<double*>(L) + nfull * NB * (ldl + 1), ldl, (int)(n - nfull * NB),
                         (int64_t)0, 2, leaves + nfull * NB * NB, (double*)nullptr, dummy,
                         (int64_t)0);
    VG_LAUNCH_CHECK();
  }
  Fact f{ldl, leaves, nullptr, nullptr, tmp, nullptr, dummy, part, s};
  f.part_elems = PART_ELEMS_BATCHED;  // the TRSM's products are at most n x m: 16 MB as before
  return trsm_left_rec(f, L, ldl, n, 0, trans, B, m, ldb);
}

}  // namespace vgposp

extern "C" size_t vgposp_trsm_workspace_bytes(int64_t n, int64_t nrhs) {
  return n > 0 && nrhs > 0 ? vgposp::trsm_ws_bytes(n, nrhs) : 0;
}

extern "C" int vgposp_trsm_lower(const double* L, int64_t n, int64_t ldl, int trans, double* B,
                                 int64_t nrhs, int64_t ldb, void* ws, size_t ws_bytes,
                                 void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(L != nullptr || n == 0, 1);
  VG_CHECK_ARG(n >= 0, 2);
  VG_CHECK_ARG(ldl >= (n > 0 ? n : 1), 3);
  VG_CHECK_ARG(trans == 0 || trans == 1, 4);
  VG_CHECK_ARG(B != nullptr || n == 0 || nrhs == 0, 5);
  VG_CHECK_ARG(nrhs >= 0, 6);
  VG_CHECK_ARG(ldb >= (nrhs > 0 ? nrhs : 1), 7);
  VG_CHECK_ARG(ws != nullptr || n == 0, 8);
  if (n == 0 || nrhs == 0) return 0;
  if (ws_bytes < trsm_ws_bytes(n, nrhs)) {
    set_error("vgposp_trsm_lower: workspace %zu < %zu bytes", ws_bytes, trsm_ws_bytes(n, nrhs));
    return VGPOSP_E_WS;
  }
  return trsm_left(L, n, ldl, trans, B, nrhs, ldb, ws, as_stream(stream));
}

extern "C" size_t vgposp_potrf_workspace_bytes(int64_t n) {
  return n > 0 ? vgposp::potrf_ws_bytes(n) : 0;
}

extern "C" size_t vgposp_potrf_batched_workspace_bytes(int64_t n, int batch) {
  return n > 0 && batch > 0 ? (size_t)batch * vgposp::potrf_ws_bytes(n) : 0;
}

extern "C" int vgposp_potrf_lower(double* A, int64_t n, int64_t lda, int64_t stride, int batch,
                                  int invert, double* diag_out, int* info, void* ws,
                                  size_t ws_bytes, void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(A != nullptr || n == 0, 1);
  VG_CHECK_ARG(n >= 0, 2);
  VG_CHECK_ARG(lda >= (n > 0 ? n : 1), 3);
  VG_CHECK_ARG(batch >= 1, 5);
  VG_CHECK_ARG(batch == 1 || stride >= lda * n, 4);
  VG_CHECK_ARG(info != nullptr, 8);
  VG_CHECK_ARG(ws != nullptr || n == 0, 9);
  hipStream_t s = as_stream(stream);
  VG_HIP(vg_memset(info, 0, sizeof(int) * batch, s));
  if (n == 0) return 0;
  if (ws_bytes < potrf_ws_bytes(n)) {
    set_error("vgposp_potrf_lower: workspace %zu < %zu bytes", ws_bytes, potrf_ws_bytes(n));
    return VGPOSP_E_WS;
  }
  if (n <= NB && batch > 1) {
    // one launch, one workgroup per matrix (e.g. the calc_H likelihood surface)
    static bool attr_set = false;
    if (!attr_set) {
      VG_HIP(hipFuncSetAttribute((const void*)potrf_leaf_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)leaf_shmem()));
      attr_set = true;
    }
    ProfScope ps("potrf_diag", s, batch * 2.0 * n * (double)n * n / 3.0, batch * 16.0 * n * (double)n);
    hipLaunchKernelGGL(potrf_leaf_kernel, dim3(batch), dim3(LEAF_THREADS), leaf_shmem(), s, A, lda,
                       (int)n, (int64_t)0, invert, (double*)nullptr, diag_out, info, stride);
    VG_LAUNCH_CHECK();
    return 0;
  }
  if (batch > 1 && ws_bytes >= (size_t)batch * potrf_ws_bytes(n))
    return potrf_batched(A, n, lda, stride, batch, invert, diag_out, info, ws, s, true);
  for (int b = 0; b < batch; ++b) {
    int rc = potrf_one(A + b * stride, n, lda, invert, diag_out ? diag_out + (int64_t)b * n : nullptr,
                       info + b, ws, s, false);
    if (rc) return rc;
  }
  return 0;
}

extern "C" int64_t vgposp_potrf_split(int64_t n) {
  return n > vgposp::NB ? vgposp::split_point(n) : 0;
}

extern "C" int vgposp_potrf_block(double* A, int64_t n, int64_t lda, int64_t col0, int64_t nb,
                                  int* info, void* ws, size_t ws_bytes, void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(A != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(lda >= n, 3);
  VG_CHECK_ARG(col0 >= 0 && col0 % NB == 0, 4);
  VG_CHECK_ARG(nb >= 1 && col0 + nb <= n, 5);
  VG_CHECK_ARG(info != nullptr, 6);
  VG_CHECK_ARG(ws != nullptr, 7);
  if (ws_bytes < potrf_ws_bytes(n)) {
    set_error("vgposp_potrf_block: workspace %zu < %zu bytes", ws_bytes, potrf_ws_bytes(n));
    return VGPOSP_E_WS;
  }
  return potrf_block(A, n, lda, col0, nb, info, ws, as_stream(stream));
}

extern "C" int vgposp_potrf_panel(double* A, int64_t n, int64_t lda, int64_t col0, int64_t nsub,
                                  int64_t r0, int64_t r1, void* ws, size_t ws_bytes,
                                  void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(A != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(lda >= n, 3);
  VG_CHECK_ARG(col0 >= 0 && col0 % NB == 0, 4);
  VG_CHECK_ARG(nsub > NBI && col0 + nsub <= n, 5);  // smaller nodes: vgposp_potrf_block
  const int64_t n1 = split_point(nsub);
  VG_CHECK_ARG(r0 >= 0 && r0 <= r1, 6);
  VG_CHECK_ARG(r1 <= nsub - n1, 7);
  VG_CHECK_ARG(ws != nullptr, 8);
  if (ws_bytes < potrf_ws_bytes(n)) {
    set_error("vgposp_potrf_panel: workspace %zu < %zu bytes", ws_bytes, potrf_ws_bytes(n));
    return VGPOSP_E_WS;
  }
  if (r1 == r0) return 0;
  return potrf_panel(A, n, lda, col0, n1, r0, r1, ws, as_stream(stream));
}

extern "C" int vgposp_potrf_trailing(double* A, int64_t n, int64_t lda, int64_t col0,
                                     int64_t nsub, int64_t b0, int64_t b1, void* ws,
                                     size_t ws_bytes, void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(A != nullptr, 1);
  VG_CHECK_ARG(n >= 1, 2);
  VG_CHECK_ARG(lda >= n, 3);
  VG_CHECK_ARG(col0 >= 0 && col0 % NB == 0, 4);
  VG_CHECK_ARG(nsub > NBI && col0 + nsub <= n, 5);
  const int64_t n1 = split_point(nsub);
  VG_CHECK_ARG(b0 >= 0 && b0 <= b1, 6);
  VG_CHECK_ARG(b1 <= nsub - n1, 7);
  VG_CHECK_ARG(ws != nullptr, 8);
  if (ws_bytes < potrf_ws_bytes(n)) {
    set_error("vgposp_potrf_trailing: workspace %zu < %zu bytes", ws_bytes, potrf_ws_bytes(n));
    return VGPOSP_E_WS;
  }
  return potrf_trailing(A, n, lda, col0, n1, b0, b1, ws, as_stream(stream));
}

extern "C" int64_t vgposp_pack_elems(int64_t r0, int64_t r1, int64_t c0, int64_t c1, int lower) {
  if (r0 < 0 || c0 < 0 || r1 < r0 || c1 < c0) return -1;
  if (lower && (c0 > r0 || c1 < r1)) return -1;
  return vgposp::pack_elems(r0, r1, c0, c1, lower);
}

extern "C" int vgposp_pack_rows(double* A, int64_t lda, int64_t r0, int64_t r1, int64_t c0,
                                int64_t c1, int lower, double* buf, int unpack, void* stream) {
  using namespace vgposp;
  clear_error();
  VG_CHECK_ARG(A != nullptr || r1 == r0, 1);
  VG_CHECK_ARG(lda >= c1, 2);
  VG_CHECK_ARG(r0 >= 0 && r0 <= r1, 3);
  VG_CHECK_ARG(c0 >= 0 && c0 <= c1, 5);
  VG_CHECK_ARG(lower == 0 || (lower == 1 && c0 <= r0 && c1 >= r1), 7);
  VG_CHECK_ARG(buf != nullptr || r1 == r0, 8);
  return pack_rows(A, lda, r0, r1, c0, c1, lower, buf, unpack, as_stream(stream));
}
