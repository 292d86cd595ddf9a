// Probe: main-loop efficiency of a 4-wave, one-wave-per-SIMD 256x256x64 bf16 GEMM tile on gfx950 (each wave
// a 128x128 quadrant, 64 16x16x32 MFMAs per 32-deep k-step, accumulators past 256 registers so the AGPRs
// hold them), against the 8-wave 4-phase gemm8p kernel's main loop (52 % MFMA busy at 4096^3,
// DESIGN.md §3). A/B staged by LDS-DMA (16-B pieces, the gemm8p XOR swizzle), double-buffered, one barrier
// per K tile. C = A B^T, A (M, K), B (N, K) row-major bf16; C bf16. Diagnostic only.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/gemm4w_probe.hip -o /tmp/gemm4w && /tmp/gemm4w
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <cmath>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

#ifndef PF_KSTEP
#define PF_KSTEP 1     // 1: frags of k-step 1 read while k-step 0's MFMAs run
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <bool STORE>
__global__ __launch_bounds__(256, 1) void gemm4w(const uint16_t* A, const uint16_t* B, uint16_t* C, int M, int N,
                                                 int K, unsigned abytes, unsigned bbytes) {
  constexpr int STAGE = 2 * 256 * 128;          // A 256 rows x 128 B + B 256 rows x 128 B
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave & 1, wc = wave >> 1;
  // XCD-aware tile order, n fastest
  const int ntn = gridDim.x, nwg = gridDim.x * gridDim.y, bid = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int tile_n = (lin % ntn) * 256, tile_m = (lin / ntn) * 256;
  const auto ra = rsrc(A, abytes), rb = rsrc(B, bbytes);
  // DMA: wave w issues pieces w + 4u (u 0..7) of A and of B; piece = 8 rows x 64 k
  const int lrow = lane >> 3, cch = (lane & 7) ^ lrow;
  unsigned aoff[8], boff[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int r = (wave + 4 * u) * 8 + lrow;
    aoff[u] = ((unsigned)(tile_m + r) * K + cch * 8) * 2u;
    boff[u] = ((unsigned)(tile_n + r) * K + cch * 8) * 2u;
  }
  auto stage = [&](int kt, int buf) {
    char* s = smem + buf * STAGE;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(s + (wave + 4 * u) * 1024), 16,
                                               aoff[u] + (unsigned)kt * 128u, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(s + 32768 + (wave + 4 * u) * 1024), 16,
                                               boff[u] + (unsigned)kt * 128u, 0, 0, 0);
    }
  };
  const int fr = lane & 15, fq = lane >> 4, fkey = lane & 7;
  const int sw[2] = {((0 + fq) ^ fkey) << 4, ((4 + fq) ^ fkey) << 4};
  const int a_row = (wr * 128 + fr) * 128, b_row = (wc * 128 + fr) * 128;
  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t af[2][8], bfr[2][8];
  auto rd = [&](int buf, int ks, int slot) {
    const char* s = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 8; ++i) af[slot][i] = *reinterpret_cast<const bf16x8_t*>(s + a_row + i * 2048 + sw[ks]);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      bfr[slot][j] = *reinterpret_cast<const bf16x8_t*>(s + 32768 + b_row + j * 2048 + sw[ks]);
  };
  auto mma = [&](int slot) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[slot][i], bfr[slot][j], acc[i][j], 0, 0, 0);
  };
  const int nk = K / 64;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#if PF_KSTEP == 2
  // hand-interleaved body: the next K tile's 16 LDS-DMA pieces and k-step 1's 16 fragment reads are spread
  // one each between groups of 4 of k-step 0's 64 MFMAs (sched_group_barrier), k-step 1's MFMAs follow
  auto body = [&](int cur, bool more, int kt) {
    rd(cur, 0, 0);
    if (more) stage(kt + 1, cur ^ 1);
    rd(cur, 1, 1);
    mma(0);
    mma(1);
    // ordering hints for the region: 8 ds_read, then repeat {4 MFMA, 1 DS read, 1 VMEM} x 16
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);   // k-step 0 fragments first
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read (k-step 1)
      if (more) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 VMEM (DMA)
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);   // k-step 1 MFMAs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int kt = 0; kt + 1 < nk; ++kt) body(kt & 1, true, kt);
  body((nk - 1) & 1, false, nk - 1);
#else
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    rd(cur, 0, 0);
    if (PF_KSTEP) {
      rd(cur, 1, 1);
      mma(0);
      mma(1);
    } else {
      mma(0);
      rd(cur, 1, 0);
      mma(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#endif
  if (!STORE) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  // c[i][j][r] = C[row 16 i + 4 fq + r][col 16 j + fr]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = tile_m + wr * 128 + 16 * i + 4 * fq + r, col = tile_n + wc * 128 + 16 * j + fr;
        C[(size_t)row * N + col] = __bfloat16_as_ushort(__float2bfloat16(acc[i][j][r]));
      }
}

static float bf2f(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }
static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7fff + ((u >> 16) & 1); return u >> 16; }

int main() {
  // correctness at 512 x 512 x 256
  {
    const int M = 512, N = 512, K = 256;
    std::vector<uint16_t> a(M * K), b(N * K), c(M * N);
    srand(1);
    for (auto& x : a) x = f2bf((rand() / (float)RAND_MAX - 0.5f));
    for (auto& x : b) x = f2bf((rand() / (float)RAND_MAX - 0.5f));
    uint16_t *da, *db, *dc;
    hipMalloc(&da, a.size() * 2); hipMalloc(&db, b.size() * 2); hipMalloc(&dc, c.size() * 2);
    hipMemcpy(da, a.data(), a.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), b.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(gemm4w<true>, dim3(N / 256, M / 256), dim3(256), 0, 0, da, db, dc, M, N, K,
                       (unsigned)(a.size() * 2), (unsigned)(b.size() * 2));
    hipMemcpy(c.data(), dc, c.size() * 2, hipMemcpyDeviceToHost);
    double err = 0, ref2 = 0;
    for (int m = 0; m < M; m += 7)
      for (int n = 0; n < N; n += 5) {
        double s = 0;
        for (int k = 0; k < K; ++k) s += (double)bf2f(a[m * K + k]) * bf2f(b[n * K + k]);
        err += (bf2f(c[m * N + n]) - s) * (bf2f(c[m * N + n]) - s);
        ref2 += s * s;
      }
    printf("check 512x512x256: rel-L2 %.3e\n", sqrt(err / ref2));
    hipFree(da); hipFree(db); hipFree(dc);
  }
  const int shapes[][3] = {{4096, 4096, 4096}, {8192, 8192, 8192}, {48384, 10240, 1280}, {193536, 5120, 640},
                           {48384, 1280, 1280}, {193536, 640, 640}};
  for (auto& s : shapes) {
    const int M = s[0], N = s[1], K = s[2];
    uint16_t *da, *db, *dc;
    hipMalloc(&da, (size_t)M * K * 2); hipMalloc(&db, (size_t)N * K * 2); hipMalloc(&dc, (size_t)M * N * 2);
    hipMemset(da, 0x3c, (size_t)M * K * 2); hipMemset(db, 0x3c, (size_t)N * K * 2);
    for (int st = 0; st < 2; ++st) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      auto launch = [&]() {
        if (st) hipLaunchKernelGGL(gemm4w<true>, dim3(N / 256, M / 256), dim3(256), 0, 0, da, db, dc, M, N, K,
                                   (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2));
        else hipLaunchKernelGGL(gemm4w<false>, dim3(N / 256, M / 256), dim3(256), 0, 0, da, db, dc, M, N, K,
                                (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2));
      };
      launch();
      hipEventRecord(e0);
      const int it = 10;
      for (int i = 0; i < it; ++i) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= it;
      printf("%6d x %6d x %5d %s: %8.1f us  %7.1f TF/s\n", M, N, K, st ? "with store" : "main loop ", ms * 1e3,
             2.0 * M * N * K / (ms * 1e-3) / 1e12);
    }
    hipFree(da); hipFree(db); hipFree(dc);
  }
  return 0;
}
