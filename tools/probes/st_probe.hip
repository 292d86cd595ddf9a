// Probe: HBM store throughput of the GEMM epilogue's store pattern vs linear stores (gfx950).
// Output: M x N bf16 (N = 320), 256-row tiles, 512 threads per tile. Patterns:
//   0 linear:  each wave writes consecutive 1 KiB pieces of the tile (whole rows, row-major)
//   1 gemm8p:  4 quadrants (128 rows x 160 cols); wave (wr = w % 4, wc = w / 4) owns 32 rows x 80
//              cols; lane chunk ch -> row ch / 10, 8 cols at (ch % 10) * 8 (16 B per lane)
//   2 column-half: as 1 but a wave's 80 columns span full rows across the two column halves first
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(512) void st_kernel(uint4* out, int M, int pattern) {
  const int N = 320;
  const int tile_m = blockIdx.x * 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint4 v = make_uint4(tid, blockIdx.x, 1, 2);
  char* base = reinterpret_cast<char*>(out);
  if (pattern == 0) {
    const size_t tile_bytes = (size_t)256 * N * 2;
    char* t = base + (size_t)tile_m * N * 2;
    for (size_t off = (size_t)tid * 16; off < tile_bytes; off += 512 * 16)
      if (tile_m + off / (N * 2) < (size_t)M) *reinterpret_cast<uint4*>(t + off) = v;
    return;
  }
  const int wr = wave % 4, wc = wave / 4;
  for (int qm = 0; qm < 2; ++qm)
    for (int qn = 0; qn < 2; ++qn) {
      const int row0 = tile_m + qm * 128 + wr * 32;
      const int col0 = qn * 160 + wc * 80;
      for (int ch = lane; ch < 32 * 10; ch += 64) {
        const int r = ch / 10, c8 = (ch % 10) * 8;
        if (row0 + r < M) *reinterpret_cast<uint4*>(base + ((size_t)(row0 + r) * N + col0 + c8) * 2) = v;
      }
    }
}

int main() {
  const int M = 516096, N = 320;
  void* d;
  hipMalloc(&d, (size_t)M * N * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int pat = 0; pat < 2; ++pat) {
    hipLaunchKernelGGL(st_kernel, dim3(M / 256), dim3(512), 0, 0, (uint4*)d, M, pat);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(st_kernel, dim3(M / 256), dim3(512), 0, 0, (uint4*)d, M, pat);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("pattern %d: %.1f us/launch, %.2f TB/s\n", pat, ms * 100.0f, (double)M * N * 2 / (ms / 10 * 1e-3) / 1e12);
  }
  return 0;
}
