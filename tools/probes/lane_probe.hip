// Probe: lane layouts the scan kernel relies on (gfx950).
//  1. v_mfma_f32_16x16x1_4b_f32 (__builtin_amdgcn_mfma_f32_16x16x1f32): which lane supplies the row (A) and
//     the column (B) of every accumulator register of every lane (4 blocks of 16x16 outer products).
//  2. v_permlane32_swap / v_permlane16_swap: which lane's value each lane holds afterwards.
// Prints compact tables; the scan's layout assumptions are asserted at the end (PASS / FAIL).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void mfma_layout(float* rowsrc, float* colsrc) {
  const int l = threadIdx.x;
  f32x16 z = {};
  // A = lane + 1, B = 1: D = A of the lane that supplied the row
  f32x16 r = __builtin_amdgcn_mfma_f32_16x16x1f32((float)(l + 1), 1.0f, z, 0, 0, 0);
  f32x16 c = __builtin_amdgcn_mfma_f32_16x16x1f32(1.0f, (float)(l + 1), z, 0, 0, 0);
  for (int i = 0; i < 16; ++i) {
    rowsrc[l * 16 + i] = r[i] - 1.0f;
    colsrc[l * 16 + i] = c[i] - 1.0f;
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void mfma4_layout(float* rowsrc, float* colsrc) {
  const int l = threadIdx.x;
  f32x4 z = {};
  f32x4 r = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.0f, z, 0, 0, 0);
  f32x4 c = __builtin_amdgcn_mfma_f32_4x4x1f32(1.0f, (float)(l + 1), z, 0, 0, 0);
  for (int i = 0; i < 4; ++i) {
    rowsrc[l * 4 + i] = r[i] - 1.0f;
    colsrc[l * 4 + i] = c[i] - 1.0f;
  }
}

__global__ void permlane(unsigned* o) {
  const unsigned l = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
  o[l * 4 + 0] = a[0];
  o[l * 4 + 1] = a[1];
  o[l * 4 + 2] = b[0];
  o[l * 4 + 3] = b[1];
}

int main() {
  float *dr, *dc;
  unsigned* dp;
  hipMalloc(&dr, 64 * 16 * 4);
  hipMalloc(&dc, 64 * 16 * 4);
  hipMalloc(&dp, 64 * 4 * 4);
  hipLaunchKernelGGL(mfma_layout, dim3(1), dim3(64), 0, 0, dr, dc);
  hipLaunchKernelGGL(permlane, dim3(1), dim3(64), 0, 0, dp);
  float hr[1024], hc[1024];
  unsigned hp[256];
  hipMemcpy(hr, dr, sizeof hr, hipMemcpyDeviceToHost);
  hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
  hipMemcpy(hp, dp, sizeof hp, hipMemcpyDeviceToHost);
  printf("16x16x1_4b: lane: (rowsrc,colsrc) per acc reg\n");
  for (int l = 0; l < 64; l += 5) {
    printf("lane %2d:", l);
    for (int i = 0; i < 16; ++i) printf(" (%2.0f,%2.0f)", hr[l * 16 + i], hc[l * 16 + i]);
    printf("\n");
  }
  // expected: acc[4b + r] of lane l = block b, row 4(l>>4) + r, col l & 15;
  // A of block b row i from lane 16b + i, B of block b col j from lane 16b + j
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int b = 0; b < 4; ++b)
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * b + r;
        const int row = 4 * (l >> 4) + r, col = l & 15;
        if ((int)hr[l * 16 + i] != 16 * b + row || (int)hc[l * 16 + i] != 16 * b + col) ++bad;
      }
  printf("mfma 16x16x1_4b layout assumption: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
  hipLaunchKernelGGL(mfma4_layout, dim3(1), dim3(64), 0, 0, dr, dc);
  hipMemcpy(hr, dr, 64 * 4 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hc, dc, 64 * 4 * 4, hipMemcpyDeviceToHost);
  printf("4x4x1_16b: lane: (rowsrc,colsrc) per acc reg\n");
  for (int l = 0; l < 64; l += 3) {
    printf("lane %2d:", l);
    for (int i = 0; i < 4; ++i) printf(" (%2.0f,%2.0f)", hr[l * 4 + i], hc[l * 4 + i]);
    printf("\n");
  }
  // expected: acc[r] of lane l = block l >> 2, row r, col l & 3; A of block b row i from lane 4b + i,
  // B of block b col j from lane 4b + j
  bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r)
      if ((int)hr[l * 4 + r] != 4 * (l >> 2) + r || (int)hc[l * 4 + r] != l) ++bad;
  printf("mfma 4x4x1_16b layout assumption: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
  printf("permlane32_swap(old=l, src=100+l) -> [0],[1]; permlane16_swap -> [0],[1]\n");
  for (int l = 0; l < 64; l += 7) printf("lane %2d: %3u %3u | %3u %3u\n", l, hp[l * 4], hp[l * 4 + 1], hp[l * 4 + 2], hp[l * 4 + 3]);
  hipFree(dr);
  hipFree(dc);
  hipFree(dp);
  return 0;
}
