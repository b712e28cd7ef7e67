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
    if (r.name != name) continue;
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
