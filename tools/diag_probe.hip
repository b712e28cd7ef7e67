// Phase timing of potrf_diag_kernel (s_memtime stamps, debug build only).
#define VGPOSP_STAMPS 1
#include "../vgposp_amd/csrc/potrf.hip"
#include <cstdlib>
#include <vector>
int main() {
  using namespace vgposp;
  const int n = 128, lda = 128;
  std::vector<double> h(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i * n + j] = (i == j ? n : 0.0) + 1.0 / (1.0 + abs(i - j));
  double *A, *linv, *dg;
  int* info;
  hipMalloc(&A, n * n * 8); hipMalloc(&linv, n * n * 8); hipMalloc(&dg, n * 8); hipMalloc(&info, 4);
  
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(A, h.data(), n * n * 8, hipMemcpyHostToDevice);
    hipMemset(info, 0, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipFuncSetAttribute((const void*)potrf_diag_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, NB * DP * 8);
    hipLaunchKernelGGL(potrf_diag_kernel, dim3(1), dim3(DIAG_THREADS), NB * DP * 8, 0, A, lda, n, 0, 1, linv, dg, info);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long st[8]; hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
    printf("kernel %.1f us | chol %lld | write L %lld | inverse+out %lld (memtime ticks)\n", ms * 1e3,
           st[1] - st[0], st[2] - st[1], st[3] - st[2]);
  }
  return 0;
}
