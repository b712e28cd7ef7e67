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

int gemm_launch(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, hipStream_t stream);

constexpr int NB = 128;        // leaf size (== GEMM tile, so trsm leaves are in place)


// ---------------------------------------------------------------------------------------------
// Blocked leaf: Cholesky + inverse of a jb x jb (jb <= 128) block in LDS, one workgroup of 4 waves.
// Panels of 16 columns: wave 0 factors the 16x16 diagonal block (and inverts it) with wave-level
// syncs only; all waves apply it to the rows below (TRSM by the block inverse) and update the
// trailing lower triangle with v_mfma_f64_16x16x4f64 (16x16 tiles, K = 16).  The inverse is then
// formed block row by block row:  X_ij = -X_ii * sum_{k=j}^{i-1} L_ik X_kj  (two MFMA chains per
// 16x16 tile, the first chain's accumulator feeding the second directly as its B operand).
// ~3 barriers per panel instead of 3 per column.  X (strictly lower) lives transposed in the
// upper triangle of the LDS image, diag(X) = 1 / diag(L) in rdiag.  jb is padded to a multiple of
// 16 with an identity block.
// ---------------------------------------------------------------------------------------------
typedef double dbl4 __attribute__((ext_vector_type(4)));

// Phase stamps for tools/diag_probe.hip (debug builds only; compiled out otherwise).
#ifdef VGPOSP_STAMPS
__device__ long long g_stamps[16];
#define STAMP_NOW() ((long long)__builtin_amdgcn_s_memtime())
#define STAMP_ADD(i, t0) \
  if (threadIdx.x == 0) g_stamps[i] += STAMP_NOW() - (t0)
#else
#define STAMP_NOW() 0LL
#define STAMP_ADD(i, t0)
#endif

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

// X[R][C] of the inverse (lower, R >= C) from the LDS image.
__device__ __forceinline__ double xval(const double* L, const double* rdiag, int R, int C) {
  return R > C ? L[C * LP2 + R] : (R == C ? rdiag[R] : 0.0);
}

__global__ __launch_bounds__(LEAF_THREADS) void potrf_leaf_kernel(double* A, int64_t lda, int jb,
                                                                  int64_t col0, int invert,
                                                                  double* linv, double* diag_out,
                                                                  int* info, int64_t stride_a) {
  extern __shared__ double L[];  // [NB][LP2]
  __shared__ double rdiag[NB];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  A += blockIdx.x * stride_a;
  info += blockIdx.x;
  if (diag_out) diag_out += (int64_t)blockIdx.x * jb;
  const int JP = (jb + LW - 1) & ~(LW - 1), NP = JP / LW;
  for (int e = t; e < JP * JP; e += LEAF_THREADS) {
    const int r = e / JP, c = e - r * JP;
    if (c <= r) L[r * LP2 + c] = r < jb ? A[(int64_t)r * lda + c] : (r == c ? 1.0 : 0.0);
  }
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  long long ts = STAMP_NOW();

  for (int p = 0; p < NP; ++p) {
    const int c0 = p * LW;
    if (wave == 0) {
      // 16x16 diagonal block in registers, symmetric (both triangles kept): lane (g, j) holds
      // D[4g + q][j], q = 0..3.  Column step c: pivot by readlane, scale column c and row c,
      // rank-1 update of the trailing block; the inverse X = L^-1 is eliminated alongside
      // ([L | I] -> [I | L^-1]: row c /= L[c][c], rows r > c -= L[r][c] row c) with the same
      // broadcasts.  No LDS traffic and no barriers inside the 16 steps.
      const int j = lane & 15, g = lane >> 4;
      double D[4], X[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 4 * g + q;
        D[q] = r >= j ? L[(c0 + r) * LP2 + c0 + j] : L[(c0 + j) * LP2 + c0 + r];
        X[q] = r == j ? 1.0 : 0.0;
      }
#pragma unroll
      for (int c = 0; c < LW; ++c) {
        const int gc = c >> 2, qc = c & 3;
        const double d = readlane_d(D[qc], gc * 16 + c);
        const double piv = sqrt(d), inv = 1.0 / piv;
        if (lane == 0) {
          if (!(d > 0.0) && c0 + c < jb) atomicCAS(info, 0, (int)(col0 + c0 + c + 1));
          rdiag[c0 + c] = inv;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 4 * g + q;
          if (j == c) D[q] = r == c ? piv : (r > c ? D[q] * inv : D[q]);
          else if (r == c && j > c) D[q] *= inv;
          if (r == c) X[q] *= inv;
        }
        const double xc = __shfl(X[qc], gc * 16 + j, 64);  // X[c][j]
        const double dc = __shfl(D[qc], gc * 16 + j, 64);  // D[c][j] = L[j][c] (j > c)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 4 * g + q;
          const double a = __shfl(D[q], (lane & 0x30) | c, 64);  // L[r][c]
          if (r > c) {
            if (j > c) D[q] -= a * dc;
            X[q] -= a * xc;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 4 * g + q;
        if (r >= j) L[(c0 + r) * LP2 + c0 + j] = D[q];
        if (r > j) L[(c0 + j) * LP2 + c0 + r] = X[q];  // X strictly lower, stored transposed
      }
    }
    __syncthreads();
    STAMP_ADD(1, ts);
    ts = STAMP_NOW();
    // rows below: P = A_panel X^T on MFMA, one 16-row tile (K = 16) per wave-iteration; each
    // tile is read and rewritten by one wave only
    const int nrt = (JP - c0 - LW) / 16;
    for (int tt = wave; tt < nrt; tt += 4) {
      const int r0 = c0 + LW + 16 * tt;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int k = 4 * s4 + fk;
        const double a = L[(r0 + fr) * LP2 + c0 + k];
        const double b = fr > k ? L[(c0 + k) * LP2 + c0 + fr] : (fr == k ? rdiag[c0 + k] : 0.0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) L[(r0 + fk + 4 * reg) * LP2 + c0 + fr] = acc[reg];
    }
    __syncthreads();
    STAMP_ADD(2, ts);
    ts = STAMP_NOW();
    // trailing lower triangle -= P P^T on MFMA, 16x16 tiles
    const int NT = NP - p - 1, ntile = NT * (NT + 1) / 2;
    for (int tt = wave; tt < ntile; tt += 4) {
      const int ti = leaf_tri_root(tt), tj = tt - ti * (ti + 1) / 2;
      const int r0 = c0 + LW + LW * ti, s0 = c0 + LW + LW * tj;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const double a = L[(r0 + fr) * LP2 + c0 + 4 * s4 + fk];
        const double b = L[(s0 + fr) * LP2 + c0 + 4 * s4 + fk];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = r0 + fk + 4 * reg, col = s0 + fr;
        if (ti != tj || col <= row) L[row * LP2 + col] -= acc[reg];
      }
    }
    __syncthreads();
    STAMP_ADD(3, ts);
    ts = STAMP_NOW();
  }

  if (invert || linv) {
    for (int i = 1; i < NP; ++i) {
      const int i0 = i * LW;
      for (int j = wave; j < i; j += 4) {
        const int j0 = j * LW;
        dbl4 S = {0.0, 0.0, 0.0, 0.0};
        for (int k = j; k < i; ++k) {
          const int k0 = k * LW;
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const double a = L[(i0 + fr) * LP2 + k0 + 4 * s4 + fk];
            const double b = xval(L, rdiag, k0 + 4 * s4 + fk, j0 + fr);
            S = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, S, 0, 0, 0);
          }
        }
        dbl4 X = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const double a = xval(L, rdiag, i0 + fr, i0 + 4 * s4 + fk);
          X = __builtin_amdgcn_mfma_f64_16x16x4f64(a, S[s4], X, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) L[(j0 + fr) * LP2 + i0 + fk + 4 * reg] = -X[reg];
      }
      __syncthreads();
    }
  }
  STAMP_ADD(4, ts);
  ts = STAMP_NOW();

  for (int e = t; e < NB * NB; e += LEAF_THREADS) {
    const int r = e / NB, c = e % NB;
    double x = 0.0;
    if (r < jb && c <= r) x = (r == c) ? rdiag[c] : L[c * LP2 + r];
    if (linv) linv[e] = x;
    if (r < jb && c <= r) A[(int64_t)r * lda + c] = invert ? x : L[r * LP2 + c];
  }
  if (diag_out != nullptr) {
    for (int c = t; c < jb; c += LEAF_THREADS) diag_out[c] = L[c * LP2 + c];
  }
  STAMP_ADD(5, ts);
  (void)ts;
}

static size_t leaf_shmem() { return (size_t)NB * LP2 * sizeof(double); }

// A (jb x jb lower) <- linv (the saved leaf inverse)
__global__ void copy_leaf_kernel(double* A, int64_t lda, int jb, const double* linv) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
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

struct Fact {
  int64_t lda;
  double* linv_all;  // ceil(n/NB) leaf inverses, NB*NB each, indexed by global column / NB
  double* work;      // trtri scratch, >= n1 * n2 doubles of the top split
  double* xinv;      // n x NBI: block inverses, rows [col0, col0 + nb) hold block col0's (or null)
  double* tmp;       // n x NBI: out-of-place TRSM leaf output (or null)
  double* diag_out;  // [n] or null
  int* info;
  hipStream_t s;
  double* leaf(int64_t col0) const { return linv_all + (col0 / NB) * NB * NB; }
  double* xblk(int64_t col0) const { return xinv + col0 * NBI; }
};

// dst (n x n lower, ldd) <- src (lower, lds); zero_upper: also zero dst's strict upper triangle
// (dst is then a full-matrix GEMM operand); otherwise dst's upper triangle is left untouched.
__global__ void copy_lower_kernel(double* dst, int64_t ldd, const double* src, int64_t lds,
                                  int64_t n, int zero_upper) {
  const int64_t r = blockIdx.y;
  for (int64_t c = threadIdx.x; c < n; c += blockDim.x) {
    if (c <= r) dst[r * ldd + c] = src[r * lds + c];
    else if (zero_upper) dst[r * ldd + c] = 0.0;
  }
}

static int copy_lower(const Fact& f, double* dst, int64_t ldd, const double* src, int64_t lds,
                      int64_t n, int zero_upper) {
  hipLaunchKernelGGL(copy_lower_kernel, dim3(1, (unsigned)n), dim3(256), 0, f.s, dst, ldd, src, lds,
                     n, zero_upper);
  VG_LAUNCH_CHECK();
  return 0;
}

static int leaf_factor(const Fact& f, double* A, int jb, int64_t col0, int invert) {
  ProfScope ps("potrf_diag", f.s, 2.0 * jb * (double)jb * jb / 3.0, 8.0 * jb * (double)jb * 2);
  hipLaunchKernelGGL(potrf_leaf_kernel, dim3(1), dim3(LEAF_THREADS), leaf_shmem(), f.s, A, f.lda,
                     jb, col0, invert, f.leaf(col0), f.diag_out ? f.diag_out + col0 : nullptr,
                     f.info, (int64_t)0);
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
    return gemm_launch(0, 1, m, nL, nL, 1.0, B, ldb, f.leaf(col0), NB, 0.0, B, ldb, VGPOSP_FULL, 0,
                       0, f.s);
  }
  if (blocks && nL <= NBI) {
    // out of place (several output column tiles read the same rows): tmp = B X^T, X lower
    if ((rc = gemm_launch(0, 1, m, nL, nL, 1.0, B, ldb, f.xblk(col0), NBI, 0.0, f.tmp, NBI,
                          VGPOSP_FULL, 0, 1, f.s)))
      return rc;
    VG_HIP(hipMemcpy2DAsync(B, ldb * sizeof(double), f.tmp, NBI * sizeof(double),
                            nL * sizeof(double), m, hipMemcpyDeviceToDevice, f.s));
    return 0;
  }
  const int64_t a = split_point(nL), b = nL - a;
  if ((rc = trsm_rec(f, B, m, ldb, Lp, a, col0, blocks))) return rc;
  // B2 -= B1 Lb^T,  Lb = L[a:, :a]
  if ((rc = gemm_launch(0, 1, m, b, a, -1.0, B, ldb, Lp + a * f.lda, f.lda, 1.0, B + a, ldb,
                        VGPOSP_FULL, 0, 0, f.s)))
    return rc;
  return trsm_rec(f, B + a, m, ldb, Lp + a * f.lda + a, b, col0 + a, blocks);
}

// Lower triangle of A (lda) holds L (leaf inverses saved) -> L^-1.  blocks: stop at the saved
// block inverses (n <= NBI) instead of recursing to the leaves.
static int trtri_rec(const Fact& f, double* A, int64_t lda, int64_t n, int64_t col0, bool blocks) {
  if (n <= NB) {
    ProfScope ps("trtri_leaf", f.s, 0.0, 8.0 * NB * NB * 2);
    hipLaunchKernelGGL(copy_leaf_kernel, dim3(NB * NB / 256), dim3(256), 0, f.s, A, lda, (int)n,
                       f.leaf(col0));
    VG_LAUNCH_CHECK();
    return 0;
  }
  if (blocks && n <= NBI) return copy_lower(f, A, lda, f.xblk(col0), NBI, n, 0);
  const int64_t n1 = split_point(n), n2 = n - n1;
  int rc;
  double* A21 = A + n1 * lda;
  double* A22 = A21 + n1;
  if ((rc = trtri_rec(f, A, lda, n1, col0, blocks))) return rc;
  if ((rc = trtri_rec(f, A22, lda, n2, col0 + n1, blocks))) return rc;
  // W = L21 X11   (X11 lower, stored [k][j])
  if ((rc = gemm_launch(0, 0, n2, n1, n1, 1.0, A21, lda, A, lda, 0.0, f.work, n1, VGPOSP_FULL, 0,
                        1, f.s)))
    return rc;
  // X21 = -X22 W  (X22 lower, stored [i][k])
  return gemm_launch(0, 0, n2, n1, n2, -1.0, A22, lda, f.work, n1, 0.0, A21, lda, VGPOSP_FULL, 1, 0,
                     f.s);
}

// blocks: form the inverse of every NB < n <= NBI diagonal block (for trsm / trtri above it).
static int potrf_rec(const Fact& f, double* A, int64_t n, int64_t col0, bool blocks) {
  if (n <= NB) return leaf_factor(f, A, (int)n, col0, 0);
  const bool whole = blocks && n <= NBI;
  const int64_t n1 = split_point(n), n2 = n - n1;
  int rc;
  double* A21 = A + n1 * f.lda;
  double* A22 = A21 + n1;
  const bool sub = blocks && !whole;  // inside a block the leaf-level path is used
  if ((rc = potrf_rec(f, A, n1, col0, sub))) return rc;
  if ((rc = trsm_rec(f, A21, n2, f.lda, A, n1, col0, sub))) return rc;
  if ((rc = gemm_launch(0, 1, n2, n2, n1, -1.0, A21, f.lda, A21, f.lda, 1.0, A22, f.lda,
                        VGPOSP_LOWER, 0, 0, f.s)))
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
  return (size_t)(leaves * NB * NB + n1 * (n - n1) + blk + 64) * sizeof(double);
}

int potrf_one(double* A, int64_t n, int64_t lda, int invert, double* diag_out, int* info,
              void* ws, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    VG_HIP(hipFuncSetAttribute((const void*)potrf_leaf_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)leaf_shmem()));
    attr_set = true;
  }
  const int64_t leaves = (n + NB - 1) / NB;
  const int64_t n1 = n > NB ? split_point(n) : 0;
  double* base = static_cast<double*>(ws);
  double* work = base + leaves * NB * NB;
  const bool blocks = n > NBI;  // a whole problem <= NBI never needs block inverses
  double* xinv = blocks ? work + n1 * (n - n1) : nullptr;
  double* tmp = blocks ? xinv + n * NBI : nullptr;
  Fact f{lda, base, work, xinv, tmp, diag_out, info, stream};
  int rc = potrf_rec(f, A, n, 0, blocks);
  if (rc || !invert) return rc;
  return trtri_rec(f, A, lda, n, 0, blocks);
}

}  // namespace vgposp

extern "C" size_t vgposp_potrf_workspace_bytes(int64_t n) {
  return n > 0 ? vgposp::potrf_ws_bytes(n) : 0;
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
  VG_HIP(hipMemsetAsync(info, 0, sizeof(int) * batch, s));
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
  for (int b = 0; b < batch; ++b) {
    int rc = potrf_one(A + b * stride, n, lda, invert, diag_out ? diag_out + (int64_t)b * n : nullptr,
                       info + b, ws, s);
    if (rc) return rc;
  }
  return 0;
}
