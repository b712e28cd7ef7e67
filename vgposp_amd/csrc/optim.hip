// TF1 AdamOptimizer update on device (tf.train.AdamOptimizer used by gp_functions.tf_train_gp_adam,
// gp_functions.py:179-182, and variational_Gaussian_process_example.py:101-102):
//   lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;  theta -= lr_t * m / (sqrt(v) + eps)
// `step` (int64 on device, incremented here) keeps the whole optimisation loop free of host syncs.
#include "common.h"

namespace vgposp {

// Softplus-constrained parameters (variables.Softplus: offset + softplus(var), torch's threshold 20)
// whose unconstrained vars sit at theta[slot[k]]: their values in one launch, and their gradients
// chained through d softplus / d var = sigmoid(var) inside the Adam update.
struct SoftplusSlots {
  int n;
  int slot[4];
  const double* g[4];  // chain: grad of theta[slot[k]] = *g[k] * sigmoid(theta[slot[k]])
  double off[4];
};

__global__ void softplus_values_kernel(const double* theta, SoftplusSlots a, double* out) {
  const int k = threadIdx.x;
  if (k < a.n) {
    const double x = theta[a.slot[k]];
    out[k] = a.off[k] + (x > 20.0 ? x : log1p(exp(x)));
  }
}

__global__ void adam_kernel(double* theta, const double* grad, double* m, double* v, int64_t n,
                            double lr, double b1, double b2, double eps, long long* step,
                            double grad_scale, SoftplusSlots chain) {
  const long long t = *step + 1;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    double gi = grad[i];
    for (int k = 0; k < chain.n; ++k)
      if (chain.slot[k] == i) gi = *chain.g[k] * (1.0 / (1.0 + exp(-theta[i])));
    const double g = grad_scale * gi;
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

static int adam_launch(double* theta, const double* grad, double* m, double* v, int64_t n,
                       double lr, double beta1, double beta2, double eps, int64_t* step,
                       double grad_scale, const SoftplusSlots& chain, hipStream_t s) {
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, s, theta, grad, m, v, n, lr, beta1,
                     beta2, eps, (long long*)step, grad_scale, chain);
  VG_LAUNCH_CHECK();
  if (blocks > 1) {
    hipLaunchKernelGGL(adam_step_kernel, dim3(1), dim3(1), 0, s, (long long*)step);
    VG_LAUNCH_CHECK();
  }
  return 0;
}

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
  return adam_launch(theta, grad, m, v, n, lr, beta1, beta2, eps, step, grad_scale, SoftplusSlots{},
                     as_stream(stream));
}

static bool softplus_slots(int nparam, const int* slots, const double* const* g,
                           const double* offsets, int64_t n, SoftplusSlots* a) {
  if (nparam < 0 || nparam > 4 || (nparam > 0 && slots == nullptr)) return false;
  *a = SoftplusSlots{};
  a->n = nparam;
  for (int k = 0; k < nparam; ++k) {
    if (slots[k] < 0 || slots[k] >= n) return false;
    a->slot[k] = slots[k];
    a->g[k] = g ? g[k] : nullptr;
    if (g && g[k] == nullptr) return false;
    a->off[k] = offsets ? offsets[k] : 0.0;
  }
  return true;
}

// out[k] = offsets[k] + softplus(theta[slots[k]]), k < nparam <= 4: one launch.
extern "C" int vgposp_softplus_values(const double* theta, int64_t n, int nparam, const int* slots,
                                      const double* offsets, double* out, void* stream) {
  clear_error();
  VG_CHECK_ARG(theta != nullptr, 1);
  VG_CHECK_ARG(out != nullptr, 6);
  SoftplusSlots a;
  VG_CHECK_ARG(softplus_slots(nparam, slots, nullptr, offsets, n, &a), 4);
  hipLaunchKernelGGL(softplus_values_kernel, dim3(1), dim3(64), 0, as_stream(stream), theta, a, out);
  VG_LAUNCH_CHECK();
  return 0;
}

// vgposp_adam_update with the softplus chain rule folded in: the gradient of theta[slots[k]] is
// *gsrc[k] * sigmoid(theta[slots[k]]) (grad[slots[k]] is not read), k < nparam <= 4.
extern "C" int vgposp_adam_update_softplus(double* theta, const double* grad, double* m, double* v,
                                           int64_t n, double lr, double beta1, double beta2,
                                           double eps, int64_t* step, double grad_scale,
                                           int nparam, const int* slots,
                                           const double* const* gsrc, void* stream) {
  clear_error();
  VG_CHECK_ARG(theta != nullptr, 1);
  VG_CHECK_ARG(grad != nullptr, 2);
  VG_CHECK_ARG(m != nullptr, 3);
  VG_CHECK_ARG(v != nullptr, 4);
  VG_CHECK_ARG(n >= 1, 5);
  VG_CHECK_ARG(lr > 0.0, 6);
  VG_CHECK_ARG(step != nullptr, 10);
  SoftplusSlots a;
  VG_CHECK_ARG(nparam == 0 || gsrc != nullptr, 14);
  VG_CHECK_ARG(softplus_slots(nparam, slots, gsrc, nullptr, n, &a), 12);
  return adam_launch(theta, grad, m, v, n, lr, beta1, beta2, eps, step, grad_scale, a,
                     as_stream(stream));
}
