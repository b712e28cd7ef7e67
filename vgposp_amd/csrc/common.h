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

// Wave64 butterfly reductions without the LDS crossbar.  Every reduction here is the descending
// xor butterfly (partner lane i ^ o for o = 32, 16, 8, 4, 2, 1; at each step a lane combines its
// value with its partner's), computed with cross-lane VALU ops instead of ds_bpermute (__shfl_xor
// is one LDS-crossbar round trip per 32-bit word per step, and the latency-bound C4 kernels spent
// most of their time in those chains):
//   o = 32, 16: v_permlane32_swap / v_permlane16_swap (CDNA4) with both operands the value, which
//               returns the two halves' (rows') values {own half, other half} in a fixed order;
//   o = 8:      DPP row_ror:8 (rotating a 16-lane row by 8 is lane i ^ 8 exactly);
//   o = 4:      DPP row_ror:4, which is lane i ^ 4 whenever lanes i and i ^ 8 hold the same value —
//               always true after the o = 8 step of a descending butterfly;
//   o = 2, 1:   DPP quad_perm [2,3,0,1] / [1,0,3,2].
// The combining operators used with it (+, min, max, the key arg-max) are commutative, so the
// results are bit-identical to the __shfl_xor butterfly they replace.  Whole waves only.
template <int O>
__device__ __forceinline__ void xor_pair32(unsigned x, unsigned& a, unsigned& b) {
  if constexpr (O == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    a = r[0];
    b = r[1];
  } else if constexpr (O == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    a = r[0];
    b = r[1];
  } else {
    constexpr int CTRL = O == 8 ? 0x128 : O == 4 ? 0x124 : O == 2 ? 0x4E : 0xB1;
    static_assert(O == 8 || O == 4 || O == 2 || O == 1, "butterfly step");
    a = x;
    // (every lane reads a valid source under these controls with all rows and banks enabled, so
    // the mov has no old value to preserve: no zero-initialised destination per step)
    b = (unsigned)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
  }
}

// The two values of a butterfly step for a 64-bit word: {a, b} = {own, partner} (o <= 8) or
// {lower half / even row, upper half / odd row} (o = 32 / 16); either way the step's result is
// op(a, b) for a commutative op.
template <int O, class T>
__device__ __forceinline__ void xor_pair64(T v, T& a, T& b) {
  static_assert(sizeof(T) == 8, "64-bit words");
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  unsigned a0, b0, a1, b1;
  xor_pair32<O>((unsigned)u, a0, b0);
  xor_pair32<O>((unsigned)(u >> 32), a1, b1);
  a = __builtin_bit_cast(T, (unsigned long long)a0 | ((unsigned long long)a1 << 32));
  b = __builtin_bit_cast(T, (unsigned long long)b0 | ((unsigned long long)b1 << 32));
}

template <int O, class Op>
__device__ __forceinline__ double wave_step(double v, Op op) {
  double a, b;
  xor_pair64<O>(v, a, b);
  return op(a, b);
}

// Every lane returns op over the wave's 64 values (op commutative).
template <class Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
  v = wave_step<32>(v, op);
  v = wave_step<16>(v, op);
  v = wave_step<8>(v, op);
  v = wave_step<4>(v, op);
  v = wave_step<2>(v, op);
  return wave_step<1>(v, op);
}

__device__ __forceinline__ double wave_sum(double v) {
  return wave_reduce(v, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ double wave_min(double v) {
  return wave_reduce(v, [](double a, double b) { return fmin(a, b); });
}
__device__ __forceinline__ double wave_max(double v) {
  return wave_reduce(v, [](double a, double b) { return fmax(a, b); });
}

// Lane `src`'s value (src wave-uniform), as a uniform value.
__device__ __forceinline__ double wave_bcast(double v, int src) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
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

// The same order as two unsigned 64-bit words compared lexicographically, so a comparison is
// three integer compares and no branches: v = an order-preserving code of the value (numbers
// >= 2, NaN 1, "no candidate" (index < 0) 0; -0 is taken as +0, which key_gt treats as equal to
// it anyway), i = ~index (a lower index is a larger code; ~(-1) = 0).
struct Key {
  unsigned long long v, i;
};

__device__ __forceinline__ Key key_enc(double v, long long i) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v + 0.0);
  const unsigned long long o = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
  Key k;
  k.i = ~(unsigned long long)i;
  k.v = i < 0 ? 0ull : (__builtin_isnan(v) ? 1ull : o);
  return k;
}

// The value back (0.0 for no candidate, a quiet NaN for NaN).
__device__ __forceinline__ double key_value(const Key& k) {
  if (k.v <= 1ull) return k.v ? __builtin_nan("") : 0.0;
  const unsigned long long u = (k.v >> 63) ? (k.v & 0x7fffffffffffffffull) : ~k.v;
  return __builtin_bit_cast(double, u);
}

__device__ __forceinline__ long long key_index(const Key& k) { return (long long)~k.i; }

__device__ __forceinline__ bool key_enc_gt(const Key& a, const Key& b) {
  return a.v > b.v || (a.v == b.v && a.i > b.i);
}

// k <- c if c > k (component-wise selects: a select of the whole struct can be lowered through
// scratch memory with a dynamic index)
__device__ __forceinline__ void key_take_max(Key& k, const Key& c) {
  const bool g = key_enc_gt(c, k);
  k.v = g ? c.v : k.v;
  k.i = g ? c.i : k.i;
}

template <int O>
__device__ __forceinline__ void wave_keystep(Key& k) {
  Key a, b;
  xor_pair64<O>(k.v, a.v, b.v);
  xor_pair64<O>(k.i, a.i, b.i);
  key_take_max(a, b);
  k = a;
}

// Every lane returns the wave's key maximum (the butterfly of wave_reduce; the order is a strict
// total order on candidates, so the result does not depend on the pairing).
__device__ __forceinline__ Key wave_keymax(Key k) {
  wave_keystep<32>(k);
  wave_keystep<16>(k);
  wave_keystep<8>(k);
  wave_keystep<4>(k);
  wave_keystep<2>(k);
  wave_keystep<1>(k);
  return k;
}

// (value, index) form: every lane returns the wave's arg-max under key_gt (its value as stored,
// except that -0.0 comes back as +0.0 and a NaN as the quiet NaN; with no candidate, index -1 and
// value 0.0).
__device__ __forceinline__ void wave_keymax(double& v, long long& i) {
  const Key k = wave_keymax(key_enc(v, i));
  v = key_value(k);
  i = key_index(k);
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
