// The 65k placement step of bench.py through the C-ABI alone: no PyTorch, so one HIP / HSA runtime
// in the process (/opt/rocm's).  Used to profile the step under rocprofv3 --pmc, where the
// PyTorch process (whose wheel bundles its own ROCm runtime beside the profiler's) hangs or
// crashes.  One step = Sigma = K(X, X) + (noise + 1e-6) I (full), the fused
// Cholesky + inverse (vgposp_greedy_init_ex), k lazy rounds (vgposp_greedy_step) — the calls
// vgposp_amd.placement_algorithm2.GreedyPlacement makes for bench.py's step.
//
//   python3 tools/step65k_data.py tools/_build/x65k.bin        (the bench's grid, numpy only)
//   hipcc -O2 --offload-arch=gfx950 tools/step65k.cpp -Iinclude -Lvgposp_amd -lvgposp \
//         -Wl,-rpath,$PWD/vgposp_amd -o tools/_build/step65k
//   tools/_build/step65k tools/_build/x65k.bin [steps] [k]
// Prints one JSON line: per-step time, the picks, and the library's own GEMM accounting
// (launches, algorithmic flops, event time) of the last step.  Progress goes to stderr through
// unbuffered write(2) at every phase (library loaded, inputs uploaded, init enqueued, init
// synchronised, every 10 rounds), so a profiled run that stalls shows where (verdict r5 item 5).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "vgposp.h"

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                \
    }                                                                         \
  } while (0)
#define CV(x)                                                                          \
  do {                                                                                 \
    int r_ = (x);                                                                      \
    if (r_ != 0) {                                                                     \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, r_, vgposp_last_error()); \
      exit(3);                                                                         \
    }                                                                                  \
  } while (0)

// One progress line on fd 2, unbuffered, with the seconds since start.
static void progress(const char* what, int a = -1) {
  static const auto t0 = std::chrono::steady_clock::now();
  const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  char buf[160];
  const int len = a >= 0 ? snprintf(buf, sizeof buf, "[step65k %8.3f s] %s %d\n", t, what, a)
                         : snprintf(buf, sizeof buf, "[step65k %8.3f s] %s\n", t, what);
  if (len > 0) {
    const ssize_t w = write(2, buf, (size_t)len);
    (void)w;
  }
}

int main(int argc, char** argv) {
  progress("start (library loaded by the dynamic linker)");
  if (argc < 2) {
    fprintf(stderr, "usage: step65k X.bin [steps] [k]\n");
    return 1;
  }
  const int steps = argc > 2 ? atoi(argv[2]) : 1;
  const int k = argc > 3 ? atoi(argv[3]) : 50;
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    perror(argv[1]);
    return 1;
  }
  int64_t hdr[2];
  double ls = 0.0;
  if (fread(hdr, 8, 2, f) != 2 || fread(&ls, 8, 1, f) != 1) return 1;
  const int64_t n = hdr[0], d = hdr[1];
  std::vector<double> X((size_t)(n * d));
  if (fread(X.data(), 8, X.size(), f) != X.size()) return 1;
  fclose(f);
  const double noise = 1e-2 + 1e-6, amp = 1.0;
  double *dX, *dS, *dpar, *dsel_delta;
  int64_t *dsel, *devals;
  int* dinfo;
  void* ws;
  const size_t ws_bytes = vgposp_greedy_workspace_bytes(n, k);
  CK(hipMalloc(&dX, X.size() * 8));
  CK(hipMalloc(&dS, (size_t)n * n * 8));
  CK(hipMalloc(&dpar, 3 * 8));
  CK(hipMalloc(&dsel, (size_t)k * 8));
  CK(hipMalloc(&devals, (size_t)k * 8));
  CK(hipMalloc(&dsel_delta, (size_t)k * 8));
  CK(hipMalloc(&dinfo, 4));
  CK(hipMalloc(&ws, ws_bytes));
  CK(hipMemcpy(dX, X.data(), X.size() * 8, hipMemcpyHostToDevice));
  const double par[3] = {amp, ls, noise};
  CK(hipMemcpy(dpar, par, 3 * 8, hipMemcpyHostToDevice));
  progress("inputs uploaded, buffers allocated");
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto step = [&](int it) {
    CV(vgposp_kernel_matrix(VGPOSP_KERNEL_EQ, dX, n, dX, n, (int)d, dpar, dpar + 1, dpar + 2, 1,
                            VGPOSP_FULL, dS, n, 0, s));
    CV(vgposp_greedy_init_ex(dS, n, n, k, 0.0, 1e-8, INFINITY, dinfo, ws, ws_bytes, s));
    progress("init enqueued, step", it);
    CK(hipStreamSynchronize(s));
    progress("init synchronised, step", it);
    for (int r = 0; r < k; ++r) {
      CV(vgposp_greedy_step(dS, n, n, k, r, 1, dsel, dsel_delta, devals, ws, ws_bytes, s));
      if (r % 10 == 9) {
        CK(hipStreamSynchronize(s));
        progress("rounds done:", r + 1);
      }
    }
  };
  double best = 1e30, total = 0.0;
  for (int it = 0; it < steps; ++it) {
    if (it + 1 == steps) vgposp_prof_enable(1);
    CK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    step(it);
    CK(hipStreamSynchronize(s));
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, dt);
    total += dt;
    fprintf(stderr, "step %d: %.3f s (with the progress synchronisations)\n", it, dt);
  }
  int info = 0;
  std::vector<int64_t> sel(k);
  CK(hipMemcpy(&info, dinfo, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sel.data(), dsel, (size_t)k * 8, hipMemcpyDeviceToHost));
  double ms = 0.0, fl = 0.0, by = 0.0;
  int64_t launches = 0;
  vgposp_prof_query("gemm_f64", &ms, &launches, &fl, &by);
  printf("{\"n\": %lld, \"k\": %d, \"steps\": %d, \"s_per_step_mean\": %.6f, \"s_per_step_min\": %.6f, "
         "\"info\": %d, \"gemm\": {\"launches\": %lld, \"flops\": %.6e, \"event_ms\": %.3f}, \"picks\": [",
         (long long)n, k, steps, total / steps, best, info, (long long)launches, fl, ms);
  for (int r = 0; r < k; ++r) printf("%s%lld", r ? ", " : "", (long long)sel[r]);
  printf("]}\n");
  return 0;
}
