// Phase timing of potrf_leaf_kernel (s_memtime stamps, debug build only):
//   hipcc -O3 --offload-arch=gfx950 tools/diag_probe.hip vgposp_amd/csrc/abi.hip -o tools/diag_probe
#define VGPOSP_STAMPS 1
#include "../vgposp_amd/csrc/potrf.hip"
#include <cstdlib>
#include <vector>
int vgposp::gemm_launch(int, int, int64_t, int64_t, int64_t, double, const double*, int64_t,
                        const double*, int64_t, double, double*, int64_t, int, int, int,
                        hipStream_t) {
  return 0;  // not used by the leaf
}
int main() {
  using namespace vgposp;
  const int n = 128, lda = 128;
  std::vector<double> h(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i * n + j] = (i == j ? n : 0.0) + 1.0 / (1.0 + abs(i - j));
  double *A, *linv, *dg;
  int* info;
  hipMalloc(&A, n * n * 8); hipMalloc(&linv, n * n * 8); hipMalloc(&dg, n * 8); hipMalloc(&info, 4);
  hipFuncSetAttribute((const void*)potrf_leaf_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)leaf_shmem());
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(A, h.data(), n * n * 8, hipMemcpyHostToDevice);
    hipMemset(info, 0, 4);
    long long z[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(potrf_leaf_kernel, dim3(1), dim3(LEAF_THREADS), leaf_shmem(), 0, A, lda, n,
                       (int64_t)0, 1, linv, dg, info, (int64_t)0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long st[16]; hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
    printf("kernel %.1f us | panel %lld | trsm %lld | syrk %lld | inverse %lld | out %lld (memtime ticks)\n",
           ms * 1e3, st[1], st[2], st[3], st[4], st[5]);
  }
  return 0;
}
