// fp64 GEMM on CDNA4 matrix cores (v_mfma_f64_16x16x4f64), the dense contraction behind the
// Cholesky trailing update, the fused block Gauss-Jordan inverse and C^-1 = M^T M formation.
//
//   C = alpha * op(A) * op(B) + beta * C        (row-major, fp64)
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves in a 2x2 grid, 64x64 = 4x4 MFMA
// fragments per wave), BK = 16, two LDS buffers with register staging (global loads of tile t+1
// are in flight while tile t is multiplied).  Operands are staged in one of two LDS images, both
// bank-conflict-free for the MFMA fragment reads (lane l reads row l&15, k = l>>4):
//   KC image [row][k] with a row pitch of 18 doubles   (operand stored k-contiguous)
//   MC image [k][row] with a row pitch of 144 doubles  (operand stored row-contiguous)
// so no operand ever needs an explicit transpose in HBM.
#include "common.h"

namespace vgposp {

typedef double dbl4 __attribute__((ext_vector_type(4)));

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
__global__ __launch_bounds__(256) void gemm_f64_kernel(GemmParams p, int vec_a, int vec_b) {
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

static bool aligned16(const void* ptr, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(ptr) % 16 == 0) && (ld % 2 == 0);
}

int gemm_launch(int transa, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                double* C, int64_t ldc, int uplo_c, int tri_a, int tri_b, hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  GemmParams p{m, n, k, alpha, beta, A, lda, B, ldb, C, ldc, uplo_c, tri_a, tri_b};
  dim3 grid((unsigned)ceil_div(n, GBN), (unsigned)ceil_div(m, GBM));
  const int va = aligned16(A, lda), vb = aligned16(B, ldb);
  const double outs = (uplo_c == VGPOSP_LOWER) ? 0.5 * (double)m * (double)(m + 1) : (double)m * n;
  ProfScope ps("gemm_f64", stream, 2.0 * (double)k * outs,
               8.0 * ((double)m * k + (double)k * n + (beta != 0.0 ? 2.0 : 1.0) * outs));
  if (!transa && !transb) hipLaunchKernelGGL((gemm_f64_kernel<false, false>), grid, dim3(256), 0, stream, p, va, vb);
  else if (!transa && transb) hipLaunchKernelGGL((gemm_f64_kernel<false, true>), grid, dim3(256), 0, stream, p, va, vb);
  else if (transa && !transb) hipLaunchKernelGGL((gemm_f64_kernel<true, false>), grid, dim3(256), 0, stream, p, va, vb);
  else hipLaunchKernelGGL((gemm_f64_kernel<true, true>), grid, dim3(256), 0, stream, p, va, vb);
  VG_LAUNCH_CHECK();
  return 0;
}

}  // namespace vgposp

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
