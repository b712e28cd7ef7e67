// ABI version and the thread-local error channel of libvgposp.so.
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

}  // namespace vgposp

extern "C" int vgposp_abi_version(void) { return VGPOSP_ABI_VERSION; }

extern "C" const char* vgposp_last_error(void) { return vgposp::g_err; }
