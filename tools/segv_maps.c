/* Diagnostic (not product code): on SIGSEGV / SIGBUS write the faulting address, the interrupted
 * PC and /proc/self/maps to a file, then hand the signal on to the handler that was installed
 * before (the profiler's failure handler, or the default action).
 *
 *   cc -O2 -shared -fPIC tools/segv_maps.c -o tools/_build/libsegvmaps.so
 *   ctypes.CDLL(...).segv_maps_install(b"gpurun_out/segv_maps.txt")   (after the GPU runtime and
 *   any profiler tool are initialised, so this handler runs first)
 *
 * The handler only uses async-signal-safe calls (open / read / write / close / sigaction). */
#define _GNU_SOURCE
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <ucontext.h>
#include <unistd.h>

static char g_path[512];
static struct sigaction g_old_segv, g_old_bus;

static void put(int fd, const char* s) { (void)!write(fd, s, strlen(s)); }

static void put_hex(int fd, unsigned long v) {
  char b[19];
  b[0] = '0';
  b[1] = 'x';
  for (int i = 0; i < 16; ++i) b[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
  b[18] = 0;
  put(fd, b);
}

static void handler(int sig, siginfo_t* si, void* uc) {
  int fd = open(g_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd >= 0) {
    put(fd, sig == SIGSEGV ? "SIGSEGV" : "SIGBUS");
    put(fd, " addr ");
    put_hex(fd, (unsigned long)si->si_addr);
    put(fd, " pc ");
    put_hex(fd, (unsigned long)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP]);
    put(fd, " code ");
    put_hex(fd, (unsigned long)si->si_code);
    put(fd, "\n--- /proc/self/maps ---\n");
    int m = open("/proc/self/maps", O_RDONLY);
    if (m >= 0) {
      char buf[4096];
      ssize_t n;
      while ((n = read(m, buf, sizeof buf)) > 0) (void)!write(fd, buf, (size_t)n);
      close(m);
    }
    close(fd);
  }
  /* hand on: restore the previous disposition and return; the faulting instruction re-executes
   * and raises the signal again under it */
  sigaction(sig, sig == SIGSEGV ? &g_old_segv : &g_old_bus, 0);
}

int segv_maps_install(const char* path) {
  strncpy(g_path, path, sizeof g_path - 1);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGSEGV, &sa, &g_old_segv) != 0) return -1;
  if (sigaction(SIGBUS, &sa, &g_old_bus) != 0) return -2;
  return 0;
}
