// TF1 AdamOptimizer update on device (tf.train.AdamOptimizer used by gp_functions.tf_train_gp_adam,
// gp_functions.py:179-182, and variational_Gaussian_process_example.py:101-102):
//   lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;  theta -= lr_t * m / (sqrt(v) + eps)
// `step` (int64 on device, incremented here) keeps the whole optimisation loop free of host syncs.
#include "common.h"

namespace vgposp {

__global__ void adam_kernel(double* theta, const double* grad, double* m, double* v, int64_t n,
                            double lr, double b1, double b2, double eps, long long* step,
                            double grad_scale) {
  const long long t = *step + 1;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const double g = grad_scale * grad[i];
    const double lr_t = lr * sqrt(1.0 - pow(b2, (double)t)) / (1.0 - pow(b1, (double)t));
    const double mi = b1 * m[i] + (1.0 - b1) * g;
    const double vi = b2 * v[i] + (1.0 - b2) * g * g;
    m[i] = mi;
    v[i] = vi;
    theta[i] -= lr_t * mi / (sqrt(vi) + eps);
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0 && gridDim.x == 1) *step = t;
}

__global__ void adam_step_kernel(long long* step) { *step += 1; }

}  // namespace vgposp

using namespace vgposp;

extern "C" int vgposp_adam_update(double* theta, const double* grad, double* m, double* v,
                                  int64_t n, double lr, double beta1, double beta2, double eps,
                                  int64_t* step, double grad_scale, void* stream) {
  clear_error();
  VG_CHECK_ARG(theta != nullptr, 1);
  VG_CHECK_ARG(grad != nullptr, 2);
  VG_CHECK_ARG(m != nullptr, 3);
  VG_CHECK_ARG(v != nullptr, 4);
  VG_CHECK_ARG(n >= 1, 5);
  VG_CHECK_ARG(lr > 0.0, 6);
  VG_CHECK_ARG(step != nullptr, 10);
  hipStream_t s = as_stream(stream);
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, s, theta, grad, m, v, n, lr, beta1,
                     beta2, eps, (long long*)step, grad_scale);
  VG_LAUNCH_CHECK();
  if (blocks > 1) {
    hipLaunchKernelGGL(adam_step_kernel, dim3(1), dim3(1), 0, s, (long long*)step);
    VG_LAUNCH_CHECK();
  }
  return 0;
}
