// Bare fp64 MFMA + LDS-fragment stream on gfx950: what fraction of the fp64 MFMA peak the K-loop's
// inner structure can reach with NO global traffic (verdict r5 item 2: locate the GEMM's loss).
// Each wave runs T "K-tiles" of 4 k-slices x 16 v_mfma_f64_16x16x4f64 (a 64 x 64 block per wave,
// the library kernel's geometry), reading its 8 fragments per slice from LDS.  Variants (MODE bits):
//   1  accumulators in AGPRs (asm groups of 4 MFMAs; else the compiler's VGPR accumulators)
//   2  double-buffered fragments (slice s+1 read before slice s's MFMAs)
//   4  s_barrier once per K-tile
//   8  one wave per SIMD (one 256-thread workgroup per CU, else two)
//  16  a 64 x 128 block per wave (32 MFMAs per slice, hipBLASLt's MT128x256 per-wave shape; with 8)
//  32  a 64 x 32 block per wave (8 MFMAs per slice) at FOUR waves per SIMD (four workgroups per CU)
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_lab.hip -o tools/_build/mfma_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl4 __attribute__((ext_vector_type(4)));

template <bool AGPR, int FJ>
__device__ __forceinline__ void mfma_row(dbl4 (&c)[FJ], double a, const double (&b)[FJ]) {
  if (AGPR) {
#pragma unroll
    for (int j = 0; j < FJ; j += 4)
      asm volatile(
          "v_mfma_f64_16x16x4_f64 %0, %4, %5, %0\n\t"
          "v_mfma_f64_16x16x4_f64 %1, %4, %6, %1\n\t"
          "v_mfma_f64_16x16x4_f64 %2, %4, %7, %2\n\t"
          "v_mfma_f64_16x16x4_f64 %3, %4, %8, %3"
          : "+a"(c[j]), "+a"(c[j + 1]), "+a"(c[j + 2]), "+a"(c[j + 3])
          : "v"(a), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]));
  } else {
#pragma unroll
    for (int j = 0; j < FJ; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[j], c[j], 0, 0, 0);
  }
}

template <int FJ>
__device__ __forceinline__ void rd(const double* L, int t, int ks, double (&a)[4], double (&b)[FJ]) {
  const int lane = threadIdx.x & 63;
  // 64 x 32 blocks: 2 buffers x 4 slices x 6 fragments (3 KiB per slice) in 32 KiB
  const double* base = FJ == 2 ? L + (t & 1) * 1536 + ks * 384 + lane
                               : L + (t & 1) * 6144 + ks * 768 + lane;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = base[i * 64];
#pragma unroll
  for (int j = 0; j < FJ; ++j) b[j] = base[256 + j * 64];  // (FJ = 2: 256..383)
}

template <int MODE>
__global__ __launch_bounds__(256, (MODE & 8) ? 1 : (MODE & 32) ? 4 : 2) void lab(double* out, int T) {
  constexpr bool AG = MODE & 1, DB = MODE & 2, BAR = MODE & 4;
  constexpr int FJ = (MODE & 16) ? 8 : (MODE & 32) ? 2 : 4;
  extern __shared__ double lds[];
  double* L = lds;  // 96 KiB: 2 buffers x 4 slices x [A 4 | B 8 fragments], read by all 4 waves
  for (int e = threadIdx.x; e < ((MODE & 32) ? 4096 : 12288); e += 256) L[e] = 1e-3 * ((e * 7) & 31);
  __syncthreads();
  dbl4 acc[4][FJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};
  double fa[2][4], fb[2][FJ];
  if (DB) rd(L, 0, 0, fa[0], fb[0]);
  for (int t = 0; t < T; ++t) {
    if (BAR) __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = DB ? (ks & 1) : 0;
      if (DB) {
        if (ks < 3) rd(L, t, ks + 1, fa[c ^ 1], fb[c ^ 1]);
        else rd(L, t + 1, 0, fa[c ^ 1], fb[c ^ 1]);
      } else {
        rd(L, t, ks, fa[0], fb[0]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) mfma_row<AG, FJ>(acc[i], fa[c][i], fb[c]);
    }
  }
  if (AG) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
static void run(double* out, int T, int cus) {
  const int occ = (MODE & 8) ? 1 : (MODE & 32) ? 4 : 2;
  const int nwg = cus * occ;
  const size_t lds = (MODE & 8) ? 120 * 1024 : (MODE & 32) ? 32 * 1024 : 96 * 1024 - 8192;
  hipFuncSetAttribute((const void*)lab<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(lab<MODE>, dim3(nwg), dim3(256), lds, 0, out, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(lab<MODE>, dim3(nwg), dim3(256), lds, 0, out, T);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double flops = (double)nwg * 4 * T * ((MODE & 16) ? 128 : (MODE & 32) ? 32 : 64) * 2048.0;
  const double tf = flops / (best * 1e-3) / 1e12;
  printf("{\"mode\": %d, \"agpr\": %d, \"dbuf\": %d, \"barrier\": %d, \"waves_per_simd\": %d, "
         "\"wave_tile\": \"64x%d\", \"ms\": %.3f, \"tflops\": %.2f, \"frac\": %.4f}\n",
         MODE, MODE & 1, (MODE >> 1) & 1, (MODE >> 2) & 1, occ, (MODE & 16) ? 128 : (MODE & 32) ? 32 : 64,
         best, tf, tf / 78.6);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 2000;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  double* out;
  hipMalloc(&out, (size_t)cus * 4 * 256 * sizeof(double));
  run<32>(out, T, cus);
  run<34>(out, T, cus);
  run<36>(out, T, cus);
  run<38>(out, T, cus);
  run<0>(out, T, cus);
  run<1>(out, T, cus);
  run<2>(out, T, cus);
  run<3>(out, T, cus);
  run<4>(out, T, cus);
  run<5>(out, T, cus);
  run<6>(out, T, cus);
  run<7>(out, T, cus);
  run<8>(out, T, cus);
  run<9>(out, T, cus);
  run<10>(out, T, cus);
  run<11>(out, T, cus);
  run<15>(out, T, cus);
  run<24>(out, T, cus);
  run<25>(out, T, cus);
  run<27>(out, T, cus);
  run<31>(out, T, cus);
  hipFree(out);
  return 0;
}
