// ABI version, the thread-local error channel, and optional per-launch event profiling.
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace vgposp {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

struct ProfRec {
  std::string name;
  hipEvent_t start = nullptr, stop = nullptr;
  double flops = 0, bytes = 0;
  bool used = false;
};

static std::mutex g_prof_mu;
static bool g_prof = false;
static std::vector<ProfRec> g_recs;
static size_t g_nrec = 0;

bool prof_on() { return g_prof; }

int prof_begin(const char* name, hipStream_t s, double flops, double bytes) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (g_nrec == g_recs.size()) {
    ProfRec r;
    if (hipEventCreate(&r.start) != hipSuccess || hipEventCreate(&r.stop) != hipSuccess) return -1;
    g_recs.push_back(r);
  }
  ProfRec& r = g_recs[g_nrec];
  r.name = name;
  r.flops = flops;
  r.bytes = bytes;
  r.used = true;
  (void)hipEventRecord(r.start, s);
  return (int)g_nrec++;
}

void prof_end(int slot, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (slot >= 0 && (size_t)slot < g_recs.size()) (void)hipEventRecord(g_recs[slot].stop, s);
}

}  // namespace vgposp

using namespace vgposp;

extern "C" int vgposp_abi_version(void) { return VGPOSP_ABI_VERSION; }

extern "C" const char* vgposp_last_error(void) { return g_err; }

extern "C" int vgposp_prof_enable(int on) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof = on != 0;
  g_nrec = 0;
  return 0;
}

extern "C" int vgposp_prof_query(const char* name, double* total_ms, int64_t* launches,
                                 double* flops, double* bytes) {
  clear_error();
  VG_CHECK_ARG(name != nullptr, 1);
  std::lock_guard<std::mutex> lk(g_prof_mu);
  double ms = 0, fl = 0, by = 0;
  int64_t cnt = 0;
  for (size_t i = 0; i < g_nrec; ++i) {
    ProfRec& r = g_recs[i];
    // a name also matches its classes: "gemm_f64" covers "gemm_f64[nt,triA]" etc.
    const size_t nl = strlen(name);
    if (r.name != name && !(r.name.size() > nl && r.name.compare(0, nl, name) == 0 && r.name[nl] == '['))
      continue;
    VG_HIP(hipEventSynchronize(r.stop));
    float t = 0.f;
    VG_HIP(hipEventElapsedTime(&t, r.start, r.stop));
    ms += t;
    fl += r.flops;
    by += r.bytes;
    ++cnt;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = cnt;
  if (flops) *flops = fl;
  if (bytes) *bytes = by;
  return 0;
}

// Per-name summary of everything recorded since prof_enable, one "name\tms\tlaunches\tflops\tbytes"
// line per distinct name (sorted by name).  Returns the bytes needed (including the final NUL);
// writes at most `len` bytes into buf (may be NULL to size the buffer).
extern "C" int64_t vgposp_prof_dump(char* buf, size_t len) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  struct Agg { double ms = 0, fl = 0, by = 0; int64_t n = 0; };
  std::map<std::string, Agg> agg;
  for (size_t i = 0; i < g_nrec; ++i) {
    ProfRec& r = g_recs[i];
    if (hipEventSynchronize(r.stop) != hipSuccess) return VGPOSP_E_HIP;
    float t = 0.f;
    if (hipEventElapsedTime(&t, r.start, r.stop) != hipSuccess) return VGPOSP_E_HIP;
    Agg& a = agg[r.name];
    a.ms += t;
    a.fl += r.flops;
    a.by += r.bytes;
    ++a.n;
  }
  std::string out;
  char line[512];
  for (auto& kv : agg) {
    snprintf(line, sizeof(line), "%s\t%.6f\t%lld\t%.6e\t%.6e\n", kv.first.c_str(), kv.second.ms,
             (long long)kv.second.n, kv.second.fl, kv.second.by);
    out += line;
  }
  if (buf && len) {
    size_t n = out.size() < len - 1 ? out.size() : len - 1;
    memcpy(buf, out.data(), n);
    buf[n] = '\0';
  }
  return (int64_t)out.size() + 1;
}

namespace vgposp {

__global__ void vg_fill_bytes_kernel(unsigned char* p, size_t n, unsigned char v) {
  // 8 bytes per thread where aligned, bytes at the ends
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t head = (8 - (reinterpret_cast<uintptr_t>(p) & 7)) & 7;
  if (i < head && i < n) p[i] = v;
  const size_t n8 = n > head ? (n - head) / 8 : 0;
  unsigned long long w = v;
  w |= w << 8;
  w |= w << 16;
  w |= w << 32;
  for (size_t k = i; k < n8; k += (size_t)gridDim.x * blockDim.x)
    reinterpret_cast<unsigned long long*>(p + head)[k] = w;
  const size_t t0 = head + 8 * n8;
  if (t0 + i < n && i < 8) p[t0 + i] = v;
}

__global__ void vg_copy2d_kernel(unsigned char* dst, size_t dpitch, const unsigned char* src,
                                 size_t spitch, size_t width, size_t height) {
  const size_t row = blockIdx.y;
  if (row >= height) return;
  unsigned char* d = dst + row * dpitch;
  const unsigned char* sp = src + row * spitch;
  const bool w8 = ((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(sp) | width) & 7) == 0;
  if (w8) {
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < width / 8;
         k += (size_t)gridDim.x * blockDim.x)
      reinterpret_cast<double*>(d)[k] = reinterpret_cast<const double*>(sp)[k];
  } else {
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < width;
         k += (size_t)gridDim.x * blockDim.x)
      d[k] = sp[k];
  }
}

hipError_t vg_memset(void* p, int value, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((bytes / 8 + 255) / 256 + 1, 4096);
  hipLaunchKernelGGL(vg_fill_bytes_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     static_cast<unsigned char*>(p), bytes, (unsigned char)value);
  return hipGetLastError();
}

hipError_t vg_memcpy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                       size_t height, hipMemcpyKind kind, hipStream_t s) {
  if (kind != hipMemcpyDeviceToDevice)
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, kind, s);
  if (width == 0 || height == 0) return hipSuccess;
  size_t bx = std::min<size_t>((width / 8 + 255) / 256, 64);
  if (bx == 0) bx = 1;
  for (size_t r0 = 0; r0 < height; r0 += 65535) {
    const size_t h = std::min<size_t>(height - r0, 65535);
    hipLaunchKernelGGL(vg_copy2d_kernel, dim3((unsigned)bx, (unsigned)h), dim3(256), 0, s,
                       static_cast<unsigned char*>(dst) + r0 * dpitch,
                       dpitch, static_cast<const unsigned char*>(src) + r0 * spitch, spitch,
                       width, h);
  }
  return hipGetLastError();
}

}  // namespace vgposp
