// Probe: a 4-wave, one-wave-per-SIMD 256x256 bf16 GEMM main loop with 128x128 wave tiles (a third fewer LDS bytes
// per MFMA than gemm8p's 8-wave layout: 16 ds_read_b128 per 64 MFMAs instead of 12 per 32), fed by a 4-slot ring
// of 32-deep sub-tiles three deep (slot s+1 read into the second fragment register set during sub-tile s's MFMAs,
// s+2 landed, s+3 in flight), one barrier per sub-tile, no stagger. C = A B^T, A (M, K), B (N, K) row-major bf16.
// Diagnostic only: main loop + plain stores; --check runs a host reference.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/gemm4r_probe.hip -o tools/probes/gemm4r_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

#ifndef IL
#define IL 1      // 1: pin the interleave (2 ds_read + 1 DMA per 8 MFMAs) with sched_group_barrier
#endif
#ifndef ASM_MFMA
#define ASM_MFMA 1
#endif
#ifndef REGSTAGE
#define REGSTAGE 0  // 1: buffer_load_dwordx4 into VGPRs (iteration s) + ds_write_b128 into the slot (iteration s + 1)
#endif
#ifndef DMAPOS
#define DMAPOS 0  // 0: one piece before each group of 8 MFMAs, 1: all 8 before group 0, 2: one piece mid-group
#endif
#ifndef NSLOT
#define NSLOT 4   // ring slots (32 KB each); DMA runs NSLOT - 1 sub-tiles ahead
#endif
#ifndef DIAG
#define DIAG 0    // 1: no vmcnt wait, 2: no DMA in the loop, 4: no fragment reads in the loop, 8: no barrier
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <bool STORE>
__global__ __launch_bounds__(256, 1) void gemm4r(const uint16_t* A, const uint16_t* B, uint16_t* C, int M, int N,
                                                 int K, unsigned abytes, unsigned bbytes) {
  constexpr int SLOT = 512 * 64;                 // 256 A rows + 256 B rows, 64 B each
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave & 1, wc = wave >> 1;
  // XCD-aware bijective tile order, n fastest
  const int ntn = gridDim.x, nwg = gridDim.x * gridDim.y, bid = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int tile_n = (lin % ntn) * 256, tile_m = (lin / ntn) * 256;
  const auto ra = rsrc(A, abytes), rb = rsrc(B, bbytes);
  // DMA pieces: 16 rows x 64 B; wave w issues A pieces w + 4u and B pieces w + 4u (u = 0..3)
  const int lrow = lane >> 2;
  const int cch = (lane & 3) ^ ((0x78 >> (2 * (lane >> 4))) & 3);
  unsigned ao[4], bo[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (wave + 4 * u) * 16 + lrow;
    ao[u] = ((unsigned)(tile_m + r) * K + cch * 8) * 2u;
    bo[u] = ((unsigned)(tile_n + r) * K + cch * 8) * 2u;
  }
  auto stage = [&](int st) {
    char* s = smem + (st % NSLOT) * SLOT;
    const int so = st * 64;                      // 32 bf16 = 64 B of K per sub-tile
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(s + (wave + 4 * u) * 1024), 16, ao[u], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(s + 256 * 64 + (wave + 4 * u) * 1024), 16, bo[u], so,
                                               0, 0);
    }
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int frag = fr * 64 + ((fq ^ ((0x78 >> (2 * (fr >> 2))) & 3)) << 4);
  const int a_base = wr * 128 * 64 + frag, b_base = 256 * 64 + wc * 128 * 64 + frag;
  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t fa[2][8], fb[2][8];
  auto rd = [&](int st, bf16x8_t (&a)[8], bf16x8_t (&b)[8]) {
    const char* s = smem + (st % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8_t*>(s + a_base + i * 1024);
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const bf16x8_t*>(s + b_base + j * 1024);
  };
  const int ns = K / 32;
  v4u sg[2][8];
#if REGSTAGE
  // prologue: sub-tiles 0, 1 written; 2 loaded into sg[1] (written in iteration 0); fragments of 0 in registers
  auto ldp = [&](int t, v4u (&d)[8]) {
#pragma unroll
    for (int g = 0; g < 8; ++g)
      d[g] = (g & 1) ? __builtin_amdgcn_raw_buffer_load_b128(rb, bo[g >> 1], t * 64, 0)
                     : __builtin_amdgcn_raw_buffer_load_b128(ra, ao[g >> 1], t * 64, 0);
  };
  auto wrp = [&](int t, const v4u (&d)[8]) {
    char* w = smem + (t % NSLOT) * SLOT;
#pragma unroll
    for (int g = 0; g < 8; ++g)
      *reinterpret_cast<v4u*>(w + (g & 1) * 256 * 64 + (wave + 4 * (g >> 1)) * 1024 + lane * 16) = d[g];
  };
  ldp(0, sg[0]);
  ldp(1, sg[1]);
  wrp(0, sg[0]);
  wrp(1, sg[1]);
  if (ns > 2) ldp(2, sg[1]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#else
  // prologue: sub-tiles 0, 1 landed; 2 in flight; fragments of 0 in registers
  stage(0);
  stage(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 2; t < NSLOT - 1; ++t)
    if (t < ns) stage(t);
#endif
  rd(0, fa[0], fb[0]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // one 32-deep sub-tile: per group g of 8 MFMAs (A row-fragment g against the 8 B fragments) two fragment reads of
  // sub-tile st + 1 and one DMA piece of sub-tile st + NSLOT - 1; FULL: steady state, no guards (tail peeled)
  // ASM_MFMA: accumulators pinned to AGPRs, fragments to VGPRs (the allocator otherwise shuffles them)
  auto mfma = [](f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
#if ASM_MFMA
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
#else
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
  };
  auto body = [&](auto full, int st, bf16x8_t (&ca)[8], bf16x8_t (&cb)[8], bf16x8_t (&na)[8], bf16x8_t (&nb)[8],
                  v4u (&cg)[8], v4u (&pg)[8]) {
    constexpr bool FULL = decltype(full)::value;
    const bool wr_next = REGSTAGE && (FULL || st + 2 < ns);
    char* wsw = smem + ((st + 2) % NSLOT) * SLOT;
    const bool rd_next = FULL ? !(DIAG & 4) : (st + 1 < ns && !(DIAG & 4));
    const bool more = FULL ? !(DIAG & 2) : (st + NSLOT - 1 < ns && !(DIAG & 2));
    const char* rs = smem + ((st + 1) % NSLOT) * SLOT;
    char* ws = smem + ((st + NSLOT - 1) % NSLOT) * SLOT;
    const int so = (st + NSLOT - 1) * 64;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (rd_next) {
        if (g < 4) {
          na[2 * g] = *reinterpret_cast<const bf16x8_t*>(rs + a_base + (2 * g) * 1024);
          na[2 * g + 1] = *reinterpret_cast<const bf16x8_t*>(rs + a_base + (2 * g + 1) * 1024);
        } else {
          nb[2 * g - 8] = *reinterpret_cast<const bf16x8_t*>(rs + b_base + (2 * g - 8) * 1024);
          nb[2 * g - 7] = *reinterpret_cast<const bf16x8_t*>(rs + b_base + (2 * g - 7) * 1024);
        }
      }
#if REGSTAGE
      if (wr_next) {   // piece g of sub-tile st + 2, loaded one iteration ago
        const int u = g >> 1;
        *reinterpret_cast<v4u*>(wsw + (g & 1) * 256 * 64 + (wave + 4 * u) * 1024 + lane * 16) = pg[g];
      }
      if (more) {
        const int u = g >> 1;
        cg[g] = (g & 1) ? __builtin_amdgcn_raw_buffer_load_b128(rb, bo[u], so, 0)
                        : __builtin_amdgcn_raw_buffer_load_b128(ra, ao[u], so, 0);
      }
#else
      auto piece = [&](int pg) {
        const int u = pg >> 1;
        if (pg & 1)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(ws + 256 * 64 + (wave + 4 * u) * 1024), 16, bo[u],
                                                   so, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(ws + (wave + 4 * u) * 1024), 16, ao[u], so, 0, 0);
      };
      if (more && DMAPOS == 0) piece(g);
      if (more && DMAPOS == 1 && g == 0)
        for (int pg = 0; pg < 8; ++pg) piece(pg);
#endif
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mfma(acc[g][j], ca[g], cb[j]);
#if !REGSTAGE
        if (more && DMAPOS == 2 && j == 3) piece(g);
#endif
      }
#if IL
      if constexpr (FULL) {
        if (!(DIAG & 4)) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS read
        if (DMAPOS == 0 && !(DIAG & 2)) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM
        if (DMAPOS == 1 && g == 0 && !(DIAG & 2)) __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);
        if (DMAPOS == 2 && !(DIAG & 2)) {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);                  // MFMA
        }
      }
#endif
    }
    __builtin_amdgcn_s_setprio(0);
    // sub-tile st + 2 landed before the barrier that precedes its reads; the reads of st + 1 done before the MFMAs
    // that use them (next iteration)
    if (DIAG & 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else if (REGSTAGE) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else if (more && NSLOT == 5) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
    else if (more) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (!(DIAG & 8)) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  int st = 0;
  for (; st + NSLOT < ns; st += 2) {
    body(T_{}, st, fa[0], fb[0], fa[1], fb[1], sg[0], sg[1]);
    body(T_{}, st + 1, fa[1], fb[1], fa[0], fb[0], sg[1], sg[0]);
  }
  for (; st < ns; st += 2) {   // ns even (host check)
    body(F_{}, st, fa[0], fb[0], fa[1], fb[1], sg[0], sg[1]);
    body(F_{}, st + 1, fa[1], fb[1], fa[0], fb[0], sg[1], sg[0]);
  }
  if (!STORE) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = tile_m + wr * 128 + 16 * i + 4 * fq + r, col = tile_n + wc * 128 + 16 * j + fr;
        C[(size_t)row * N + col] = __builtin_bit_cast(uint16_t, (__bf16)acc[i][j][r]);
      }
}

static float bf2f(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }
static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7fff + ((u >> 16) & 1); return u >> 16; }

int main(int argc, char** argv) {
  {
    // correctness at 512 x 512 x 320 (K a multiple of 32, odd sub-tile count)
    const int M = 512, N = 512, K = 384;
    std::vector<uint16_t> a(M * K), b(N * K), c(M * N);
    srand(1);
    for (auto& x : a) x = f2bf(rand() / (float)RAND_MAX - 0.5f);
    for (auto& x : b) x = f2bf(rand() / (float)RAND_MAX - 0.5f);
    uint16_t *da, *db, *dc;
    hipMalloc(&da, a.size() * 2); hipMalloc(&db, b.size() * 2); hipMalloc(&dc, c.size() * 2);
    hipMemcpy(da, a.data(), a.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), b.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(gemm4r<true>, dim3(N / 256, M / 256), dim3(256), 0, 0, da, db, dc, M, N, K,
                       (unsigned)(a.size() * 2), (unsigned)(b.size() * 2));
    hipMemcpy(c.data(), dc, c.size() * 2, hipMemcpyDeviceToHost);
    double err = 0, ref2 = 0;
    for (int m = 0; m < M; m += 3)
      for (int n = 0; n < N; n += 5) {
        double s = 0;
        for (int k = 0; k < K; ++k) s += (double)bf2f(a[m * K + k]) * bf2f(b[n * K + k]);
        err += (bf2f(c[m * N + n]) - s) * (bf2f(c[m * N + n]) - s);
        ref2 += s * s;
      }
    printf("check 512x512x384: rel-L2 %.3e\n", sqrt(err / ref2));
    hipFree(da); hipFree(db); hipFree(dc);
  }
  const int shapes[][3] = {{8192, 8192, 8192}, {4096, 4096, 4096}, {48384, 10240, 1280}, {193536, 5120, 640},
                           {48384, 1280, 1280}, {48384, 1280, 5120}};
  for (auto& s : shapes) {
    const int M = s[0], N = s[1], K = s[2];
    uint16_t *da, *db, *dc;
    hipMalloc(&da, (size_t)M * K * 2); hipMalloc(&db, (size_t)N * K * 2); hipMalloc(&dc, (size_t)M * N * 2);
    {
      // random bf16 in [-1, 1) (zero / constant operands raise the clock: guide §5.4 rule 25)
      std::vector<uint16_t> h(1 << 20);
      srand(3);
      for (auto& x : h) x = f2bf(rand() / (float)RAND_MAX * 2.f - 1.f);
      for (size_t o = 0; o < (size_t)M * K; o += h.size())
        hipMemcpy(da + o, h.data(), std::min(h.size(), (size_t)M * K - o) * 2, hipMemcpyHostToDevice);
      for (size_t o = 0; o < (size_t)N * K; o += h.size())
        hipMemcpy(db + o, h.data(), std::min(h.size(), (size_t)N * K - o) * 2, hipMemcpyHostToDevice);
    }
    for (int st = 0; st < 2; ++st) {
      auto launch = [&]() {
        if (st) hipLaunchKernelGGL(gemm4r<true>, dim3(N / 256, M / 256), dim3(256), 0, 0, da, db, dc, M, N, K,
                                   (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2));
        else hipLaunchKernelGGL(gemm4r<false>, dim3(N / 256, M / 256), dim3(256), 0, 0, da, db, dc, M, N, K,
                                (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2));
      };
      launch();
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      const int it = 10;
      hipEventRecord(e0);
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
