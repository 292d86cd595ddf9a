// Probe: cycles per v_mfma_f32_16x16x32_bf16 in a segment of 32 independent MFMAs (the gemm8p ring's MFMA segment:
// 8 A x 4 B fragments, 32 accumulators), per wave, for several residency layouts:
//   mode 0: 4 waves / WG (one per SIMD), every wave MFMA-only
//   mode 1: 8 waves / WG (two per SIMD), both waves MFMA-only
//   mode 2: 8 waves / WG, waves 4-7 park at barriers while 0-3 compute (ring-style alternation, barrier per segment)
// One workgroup per CU (96 KB of dynamic LDS). Operands: random bf16 bits (fixed per lane) or zeros. Prints mean cycles per MFMA from s_memtime and wall TF/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/mfma_rate_probe.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512, 2) void probe(const unsigned* seed, unsigned long long* cyc, float* sink, int iters) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  bf16x8_t a[8], b[4];
  for (int i = 0; i < 8; ++i) {
    unsigned s = seed[(i * 64 + lane) & 1023];
    for (int e = 0; e < 8; ++e) { unsigned short h = (s >> (e * 3)) & 0x3fff; a[i][e] = __builtin_bit_cast(__bf16, (unsigned short)(h ^ 0x3c00)); }
  }
  for (int j = 0; j < 4; ++j) {
    unsigned s = seed[(j * 64 + lane + 512) & 1023];
    for (int e = 0; e < 8; ++e) { unsigned short h = (s >> (e * 2)) & 0x3fff; b[j][e] = __builtin_bit_cast(__bf16, (unsigned short)(h ^ 0x3c00)); }
  }
  f32x4_t c[8][4];
  for (int i = 0; i < 8; ++i) for (int j = 0; j < 4; ++j) c[i][j] = f32x4_t{0, 0, 0, 0};
  const bool late = wave >= 4;
  if (MODE >= 2 && late) __builtin_amdgcn_s_barrier();
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), tm = 0;
  for (int it = 0; it < iters; ++it) {
    if (MODE >= 2) { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); __builtin_amdgcn_sched_barrier(0); }
    unsigned long long s0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long s1 = __builtin_amdgcn_s_memtime();
    tm += s1 - s0;
    if (MODE >= 2) { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); __builtin_amdgcn_sched_barrier(0); }
  }
  if (MODE >= 2 && !late) __builtin_amdgcn_s_barrier();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) for (int j = 0; j < 4; ++j) s += c[i][j][0] + c[i][j][3];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) {
    cyc[(blockIdx.x * 8 + wave) * 2] = tm;
    cyc[(blockIdx.x * 8 + wave) * 2 + 1] = t1 - t0;
  }
}

int main() {
  const int nblk = 256 * 4, iters = 2000;
  hipFuncSetAttribute((const void*)probe<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  hipFuncSetAttribute((const void*)probe<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  hipFuncSetAttribute((const void*)probe<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  unsigned* dseed; unsigned long long* dcyc; float* dsink;
  hipMalloc(&dseed, 1024 * 4); hipMalloc(&dcyc, nblk * 8 * 2 * 8); hipMalloc(&dsink, nblk * 512 * 4);
  unsigned hs[1024];
  for (int zero = 0; zero < 2; ++zero) {
    srand(7);
    for (int i = 0; i < 1024; ++i) hs[i] = zero ? 0x03000300u : ((unsigned)rand() << 1) ^ rand();
    hipMemcpy(dseed, hs, sizeof(hs), hipMemcpyHostToDevice);
    for (int mode = 0; mode < 3; ++mode) {
      const int threads = mode == 0 ? 256 : 512;
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(nblk), dim3(threads), 96 * 1024, 0, dseed, dcyc, dsink, iters);
        if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(nblk), dim3(threads), 96 * 1024, 0, dseed, dcyc, dsink, iters);
        if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(nblk), dim3(threads), 96 * 1024, 0, dseed, dcyc, dsink, iters);
      };
      launch();
      hipDeviceSynchronize();
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      static unsigned long long hc[256 * 4 * 8 * 2];
      hipMemcpy(hc, dcyc, sizeof(hc), hipMemcpyDeviceToHost);
      const int nw = threads / 64;
      double seg = 0, tot = 0; int n = 0;
      for (int bk = 0; bk < nblk; ++bk) for (int w = 0; w < nw; ++w) { seg += hc[(bk * 8 + w) * 2]; tot += hc[(bk * 8 + w) * 2 + 1]; ++n; }
      seg /= n; tot /= n;
      const double flop = 2.0 * 16 * 16 * 32 * 32 * (double)iters * nw * nblk;
      printf("%s mode %d: MFMA segment %.1f cyc/MFMA; whole loop %.1f cyc per 32-MFMA iteration; wall %.3f ms = %.0f TF/s; clock ~%.2f GHz\n",
             zero ? "zero  " : "random", mode, seg / (32.0 * iters), tot / iters, ms, flop / (ms * 1e-3) / 1e12,
             tot / (ms * 1e-3) / 1e9 / 1.0);
    }
  }
  return 0;
}
