// HBM write-rate probe for the kernel-assembly layout question (kernel_matrix):
// write an n x n fp64 matrix (n = 65,536, 34.4 GB) with
//   0: 128 x 128 tiles, one 16-byte non-temporal store per lane, 4 rows in flight per workgroup
//      (kernel_matrix_kernel's store pattern, no arithmetic)
//   1: the same with plain (temporal) stores
//   2: 64-row x 256-column tiles, two 16-byte stores per lane (2 KiB contiguous per wave and row)
//   3: whole rows: one workgroup per row, 16-byte non-temporal stores, grid-stride
//   4: pattern 0 plus an fp64 exp per entry (the EQ kernel's arithmetic)
// and report TB/s per pattern (best of 3).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef double d2v __attribute__((ext_vector_type(2)));

template <int NT, int EXP>
__global__ __launch_bounds__(256) void tile128(double* K, long n) {
  const long r0 = (long)blockIdx.y * 128, c0 = (long)blockIdx.x * 128;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long ca = c0 + 2 * tx;
  for (long r = r0 + ty; r < r0 + 128; r += 4) {
    double va = (double)(r - ca), vb = va + 1.0;
    if (EXP) {
      va = exp(-1e-9 * va * va);
      vb = exp(-1e-9 * vb * vb);
    }
    d2v* p = reinterpret_cast<d2v*>(K + r * n + ca);
    if (NT) __builtin_nontemporal_store(d2v{va, vb}, p);
    else *p = d2v{va, vb};
  }
}

__global__ __launch_bounds__(256) void tile64x256(double* K, long n) {
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 256;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long ca = c0 + 2 * tx;
  for (long r = r0 + ty; r < r0 + 64; r += 4) {
    const double va = (double)(r - ca);
    __builtin_nontemporal_store(d2v{va, va + 1.0}, reinterpret_cast<d2v*>(K + r * n + ca));
    __builtin_nontemporal_store(d2v{va + 128.0, va + 129.0},
                                reinterpret_cast<d2v*>(K + r * n + ca + 128));
  }
}

__global__ __launch_bounds__(256) void rows(double* K, long n) {
  const long r = blockIdx.x;
  for (long c = 2 * threadIdx.x; c < n; c += 512) {
    const double v = (double)(r - c);
    __builtin_nontemporal_store(d2v{v, v + 1.0}, reinterpret_cast<d2v*>(K + r * n + c));
  }
}

int main() {
  const long n = 65536;
  double* K;
  if (hipMalloc(&K, n * n * sizeof(double)) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"tile128 nt", "tile128 plain", "tile64x256 nt", "rows nt", "tile128 nt + exp"};
  for (int p = 0; p < 5; ++p) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      switch (p) {
        case 0: hipLaunchKernelGGL((tile128<1, 0>), dim3(n / 128, n / 128), dim3(256), 0, 0, K, n); break;
        case 1: hipLaunchKernelGGL((tile128<0, 0>), dim3(n / 128, n / 128), dim3(256), 0, 0, K, n); break;
        case 2: hipLaunchKernelGGL(tile64x256, dim3(n / 256, n / 64), dim3(256), 0, 0, K, n); break;
        case 3: hipLaunchKernelGGL(rows, dim3(n), dim3(256), 0, 0, K, n); break;
        default: hipLaunchKernelGGL((tile128<1, 1>), dim3(n / 128, n / 128), dim3(256), 0, 0, K, n); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("%-18s %8.3f ms  %6.2f TB/s\n", names[p], best, n * n * 8.0 / (best * 1e-3) / 1e12);
  }
  hipFree(K);
  return 0;
}
