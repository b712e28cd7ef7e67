// PSD kernel functions shared by kernel assembly, the kernel-matrix-vector product and friends.
// TFP evaluates k(r) = exp(2 log amp + log k_unit(r / ls)); the Matern 3/2 and 5/2 forms here take
// the polynomial factor out of the exponential (amp^2 p(s) exp(-s), no log1p: the same value to
// rounding, and the fp64 log1p was what made Matern assembly ALU-bound).
#pragma once

#include "common.h"

namespace vgposp {

template <int KIND>
__device__ __forceinline__ double kfun(double d2, double two_log_amp, double inv_ls, double inv_ls2) {
  if (KIND == VGPOSP_KERNEL_EQ) {
    return exp(two_log_amp - 0.5 * d2 * inv_ls2);
  }
  const double r = sqrt(d2) * inv_ls;
  if (KIND == VGPOSP_KERNEL_MATERN12) return exp(two_log_amp - r);
  if (KIND == VGPOSP_KERNEL_MATERN32) {
    const double s = 1.7320508075688772 * r;
    return (1.0 + s) * exp(two_log_amp - s);
  }
  const double s = 2.23606797749979 * r;  // MATERN52
  return (1.0 + s + s * s * (1.0 / 3.0)) * exp(two_log_amp - s);
}

// K, dK/dls and the coefficient c with dK/dx1 = c * (x1 - x2), for one entry.
template <int KIND>
__device__ __forceinline__ void kvjp_entry(double d2, double tla, double inv_l, double inv_l2,
                                           double& K, double& dkl, double& cx) {
  if (KIND == VGPOSP_KERNEL_EQ) {
    K = exp(tla - 0.5 * d2 * inv_l2);
    dkl = K * d2 * inv_l2 * inv_l;
    cx = -K * inv_l2;
  } else if (KIND == VGPOSP_KERNEL_MATERN12) {
    const double r = sqrt(d2) * inv_l;
    K = exp(tla - r);
    dkl = K * r * inv_l;
    cx = r > 0.0 ? -K * inv_l2 / r : 0.0;  // direction undefined at r = 0: sub-gradient 0
  } else if (KIND == VGPOSP_KERNEL_MATERN32) {
    const double s = 1.7320508075688772 * sqrt(d2) * inv_l;
    const double E = exp(tla - s);
    K = E * (1.0 + s);
    dkl = E * s * s * inv_l;
    cx = -3.0 * E * inv_l2;
  } else {
    const double s = 2.23606797749979 * sqrt(d2) * inv_l;
    const double E = exp(tla - s);
    K = E * (1.0 + s + s * s * (1.0 / 3.0));
    dkl = E * (s * s * (1.0 / 3.0)) * (1.0 + s) * inv_l;
    cx = -(5.0 / 3.0) * (1.0 + s) * E * inv_l2;
  }
}

}  // namespace vgposp
