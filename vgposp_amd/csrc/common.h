// Shared helpers for the vgposp HIP library (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/vgposp.h"

namespace vgposp {

// Thread-local last error message (vgposp_last_error()).
void set_error(const char* fmt, ...);
void clear_error();

#define VG_CHECK_ARG(cond, idx)                                                       \
  do {                                                                                \
    if (!(cond)) {                                                                    \
      ::vgposp::set_error("%s: bad argument %d (%s)", __func__, (idx), #cond);        \
      return -(idx);                                                                  \
    }                                                                                 \
  } while (0)

#define VG_HIP(expr)                                                                  \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      ::vgposp::set_error("%s: HIP error %s at %s:%d", __func__, hipGetErrorString(_e), \
                          __FILE__, __LINE__);                                        \
      return VGPOSP_E_HIP;                                                            \
    }                                                                                 \
  } while (0)

#define VG_LAUNCH_CHECK() VG_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Device-to-device fills and 2-D copies as KERNELS (same signatures as hipMemsetAsync /
// hipMemcpy2DAsync).  Everything the library enqueues is then a kernel node when a caller
// captures it into a HIP graph (the VGP training step): replays of captured memset / memcpy
// nodes were the one ordering hazard seen on this ROCm build (a status buffer read after a replay
// returned stale data unless the host synchronised first).
__global__ void vg_fill_bytes_kernel(unsigned char* p, size_t n, unsigned char v);
__global__ void vg_copy2d_kernel(unsigned char* dst, size_t dpitch, const unsigned char* src,
                                 size_t spitch, size_t width, size_t height);
hipError_t vg_memset(void* p, int value, size_t bytes, hipStream_t s);
hipError_t vg_memcpy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                       size_t height, hipMemcpyKind kind, hipStream_t s);

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- device helpers -------------------------------------------------------------------------

// Wave64 reductions.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (value, index) arg-max with the reference's tie rule: larger value wins; on equal value the
// LOWER index wins (placement_algorithm2.py:62 uses strict '<' scanning upward).  Index -1 is
// "no candidate" and loses to everything.  A NaN value ranks below every number (the reference's
// `delta_st < delta_y` is false for NaN, so a NaN delta is never selected), which keeps key_gt a
// strict order whatever the lane order of a reduction.
struct KeyMax {
  double v;
  long long i;
};

__device__ __forceinline__ bool key_gt(double v1, long long i1, double v2, long long i2) {
  if (i1 < 0) return false;
  if (i2 < 0) return true;
  if (__builtin_isnan(v1)) return __builtin_isnan(v2) && i1 < i2;
  if (__builtin_isnan(v2)) return true;
  return (v1 > v2) || (v1 == v2 && i1 < i2);
}

__device__ __forceinline__ void wave_keymax(double& v, long long& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, 64);
    long long oi = __shfl_xor(i, o, 64);
    if (key_gt(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
}

}  // namespace vgposp

namespace vgposp {
// Optional per-launch timing (vgposp_prof_enable): the library records a hipEvent pair around
// every launch of a named kernel together with its algorithmic flops / bytes.  Off by default.
bool prof_on();
int prof_begin(const char* name, hipStream_t s, double flops, double bytes);
void prof_end(int slot, hipStream_t s);

struct ProfScope {
  int slot;
  hipStream_t s;
  ProfScope(const char* name, hipStream_t st, double flops, double bytes, bool enable = true)
      : slot(enable && prof_on() ? prof_begin(name, st, flops, bytes) : -1), s(st) {}
  ~ProfScope() {
    if (slot >= 0) prof_end(slot, s);
  }
};
}  // namespace vgposp
