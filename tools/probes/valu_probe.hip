// Probe: VALU issue cost on gfx950 of the instruction mix of the selective-scan recurrence
// (scan.hip): v_fma_f32 vs v_pk_fma_f32 vs v_pk_mul_f32 vs v_exp_f32, one and four waves per SIMD.
// Each lane runs NIT iterations of 8 independent chains of the instruction under test (inline asm,
// so the compiler neither packs nor unpacks them). Cycles per wave-instruction = elapsed shader
// cycles (s_memtime) / instructions issued by one wave, reported for the given waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define NIT 2048

template <int OP>
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* cyc) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = {a1, a0}, p5 = {a3, a2}, p6 = {a5, a4},
     p7 = {a7, a6};
  const float m = 0.999f, c = 1e-4f;
  const f2 m2 = {m, m}, c2 = {c, c};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < NIT; ++i) {
    if (OP == 0) {           // v_fma_f32 x 8
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a4) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a5) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a6) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a7) : "v"(m), "v"(c));
    } else if (OP == 1) {    // v_pk_fma_f32 x 8
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p0) : "v"(m2), "v"(c2));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p1) : "v"(m2), "v"(c2));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p2) : "v"(m2), "v"(c2));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p3) : "v"(m2), "v"(c2));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p4) : "v"(m2), "v"(c2));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p5) : "v"(m2), "v"(c2));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p6) : "v"(m2), "v"(c2));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p7) : "v"(m2), "v"(c2));
    } else if (OP == 2) {    // v_pk_mul_f32 x 8
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p0) : "v"(m2));
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p1) : "v"(m2));
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p2) : "v"(m2));
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p3) : "v"(m2));
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p4) : "v"(m2));
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p5) : "v"(m2));
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p6) : "v"(m2));
      asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p7) : "v"(m2));
    } else if (OP == 3) {    // v_exp_f32 x 8
      asm volatile("v_exp_f32 %0, %0" : "+v"(a0));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a1));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a2));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a3));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a4));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a5));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a6));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a7));
    } else if (OP == 4) {    // v_mul_f32 x 8
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a0) : "v"(m));
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a1) : "v"(m));
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a2) : "v"(m));
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a3) : "v"(m));
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a4) : "v"(m));
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a5) : "v"(m));
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a6) : "v"(m));
      asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a7) : "v"(m));
    } else {                 // mixed: 2 exp + 4 fma (the scan's ratio)
      asm volatile("v_exp_f32 %0, %0" : "+v"(a0));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(m), "v"(c));
      asm volatile("v_exp_f32 %0, %0" : "+v"(a3));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a4) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a5) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a6) : "v"(m), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a7) : "v"(m), "v"(c));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.x + p2.x + p3.x + p4.y + p5.y + p6.y + p7.y;
  if (s == 12345.f) out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(const char* name, int waves_per_simd) {
  float* out;
  unsigned long long* cyc;
  const int nblk = 256 * waves_per_simd;    // 256 CUs; 256 threads = 4 waves = one per SIMD per block
  hipMalloc(&out, 1024 * sizeof(float));
  hipMalloc(&cyc, nblk * sizeof(unsigned long long));
  hipLaunchKernelGGL(probe<OP>, dim3(nblk), dim3(256), 0, 0, out, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<OP>, dim3(nblk), dim3(256), 0, 0, out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[4096];
  hipMemcpy(h, cyc, nblk * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < nblk; ++i) avg += h[i];
  avg /= nblk;
  const double insts = 8.0 * NIT;
  // s_memtime ticks at the shader clock (MI355X_MICROARCH.md); per SIMD `waves_per_simd` waves share issue
  printf("%-12s waves/SIMD %d: %.2f cycles per wave-instruction (per-wave view), %.2f per instruction per SIMD, "
         "kernel %.3f ms\n", name, waves_per_simd, avg / insts, avg / insts / waves_per_simd, ms);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w : {1, 2, 4}) {
    run<0>("v_fma_f32", w);
    run<4>("v_mul_f32", w);
    run<1>("v_pk_fma_f32", w);
    run<2>("v_pk_mul_f32", w);
    run<3>("v_exp_f32", w);
    run<5>("2exp+6fma", w);
  }
  return 0;
}
