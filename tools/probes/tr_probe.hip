// Probe: semantics of ds_read_b64_tr_b16 on gfx950. LDS holds a 16 x 64 matrix of 16-bit
// values M[r][c] = r * 100 + c. Lane 4q+p of each 16-lane group supplies the address of row
// (4g' + q) at column 4p (+16 * (g & 1)); print what each lane receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4_t lds_short4;
__global__ void k(short* out) {
  __shared__ short m[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) m[i] = (short)((i / 64) * 100 + (i % 64));
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 4 * (g >> 1) + q, col = 16 * (g & 1) + 4 * p;
  short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)&m[row * 64 + col]);
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %5d %5d %5d %5d\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
  return 0;
}
