// TEST INFRASTRUCTURE (tests/test_gpu_wave.py): the library's cross-lane wave reductions
// (vgposp_amd/csrc/common.h: DPP / v_permlane*_swap butterflies) against the __shfl_xor
// (ds_bpermute) butterflies they replaced, bit for bit.  Built by __graft_entry__.build() into
// tests/_build/libwavecheck.so.
#include "../../vgposp_amd/csrc/common.h"

using namespace vgposp;

__device__ double shfl_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ double shfl_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ void shfl_keymax(double& v, long long& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o, 64);
    const long long oi = __shfl_xor(i, o, 64);
    if (key_gt(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
}

// One wave per 64 inputs; out[w * 64 * 8 + lane * 8 + j]: j = 0 / 1 sum (new / old), 2 / 3 min,
// 4 / 5 key value, 6 / 7 key index (as double bits), 8th slot unused.
__global__ __launch_bounds__(256) void wave_check_kernel(const double* in, const long long* idx,
                                                         int nw, double* out) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= nw) return;
  const double x = in[w * 64 + lane];
  const long long ix = idx[w * 64 + lane];
  double* o = out + ((size_t)w * 64 + lane) * 8;
  o[0] = wave_sum(x);
  o[1] = shfl_sum(x);
  o[2] = wave_min(x);
  o[3] = shfl_min(x);
  double v1 = x, v2 = x;
  long long i1 = ix, i2 = ix;
  wave_keymax(v1, i1);
  shfl_keymax(v2, i2);
  o[4] = v1;
  o[5] = v2;
  o[6] = __builtin_bit_cast(double, i1);
  o[7] = __builtin_bit_cast(double, i2);
}

// Host entry: nw waves of inputs (host arrays), results into out (nw * 64 * 8 doubles).
extern "C" int wave_check(const double* in, const long long* idx, int nw, double* out) {
  double *din, *dout;
  long long* didx;
  const size_t n = (size_t)nw * 64;
  if (hipMalloc(&din, n * 8) != hipSuccess) return 1;
  if (hipMalloc(&didx, n * 8) != hipSuccess) return 1;
  if (hipMalloc(&dout, n * 64) != hipSuccess) return 1;
  hipMemcpy(din, in, n * 8, hipMemcpyHostToDevice);
  hipMemcpy(didx, idx, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(wave_check_kernel, dim3((nw + 3) / 4), dim3(256), 0, 0, din, didx, nw, dout);
  const hipError_t e = hipMemcpy(out, dout, n * 64, hipMemcpyDeviceToHost);
  hipFree(din);
  hipFree(didx);
  hipFree(dout);
  return e == hipSuccess ? 0 : 2;
}
