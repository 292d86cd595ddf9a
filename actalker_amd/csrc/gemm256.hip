// bf16 MFMA GEMM, 256-row tiles, 8 waves (gfx950). Same operand loaders and fused epilogues as the
// 128x128 kernel in gemm.hip (see gemm_common.h); picked by acth_gemm for the large-M shapes of the
// UNet (every level-0..2 Linear / conv), where a 128x128 tile is L2->CU bandwidth bound:
// a 128x128x64 step moves 32 KB for 2.1 MFLOP (64 FLOP/B), a 256x256 step 64 KB for 8.4 MFLOP
// (128 FLOP/B), against ~72 FLOP/B that one CU needs to keep its matrix pipes busy from L2.
//
// Tiles (template <BN, WM, WN>): BM = 256 rows, BN = 256 or 160 columns (160 divides the C = 320 /
// 640 / 960 projections exactly), 8 waves arranged WM x WN, each wave owning a (256/WM) x (BN/WN)
// sub-tile of v_mfma_f32_16x16x32_bf16 accumulators (8x4 or 4x5 of them).
// K loop: BK = 64, two LDS stages (A 32 KB + B up to 32 KB each). Both operands move HBM/L2 -> LDS
// by LDS-DMA (buffer_load_dwordx4 ... lds), 1 KiB = 8 rows x 128 B per wave-instruction; the
// per-lane SOURCE address carries the im2col / concat / upsample remap and the XOR swizzle
// (16-B chunk ^ (row & 7)) that makes the fragment reads (ds_read_b128 of 16 rows x 16 B per
// lane group) bank-conflict free. Stage k+1's DMA is issued before stage k's MFMAs, so each K step
// (2048 MFMA cycles per SIMD) covers the next tile's load latency; one vmcnt(0) + barrier per step.
// Epilogue: each wave transposes its accumulators through a private LDS slab, 32 rows at a time,
// so every lane owns 8 consecutive columns of a row (16-byte coalesced bias / residual / output).
#include "gemm_common.h"

using namespace gemm;

#define G_BM 256
#define G_BK 64
#define PERSIST_BLOCKS 256   // MI355X CUs

// pixel (row of the A source) feeding output row `ri` at conv/temporal tap `tap`, or -1 when the
// tap falls into zero padding / outside the frame window
template <int AMODE>
__device__ __forceinline__ int tap_pixel(const ActhGemmDesc& p, int m, const RowInfo& ri, int tap) {
  if (!ri.ok) return -1;
  if (AMODE == 0) return m;
  if (AMODE == 1) {
    const int ky = tap / 3, kx = tap - ky * 3;
    int iy, ix;
    if (p.upsample) {
      iy = ri.y + ky - 1; ix = ri.x + kx - 1;
      if (iy < 0 || ix < 0 || iy >= 2 * p.H || ix >= 2 * p.W) return -1;
      iy >>= 1; ix >>= 1;
    } else {
      iy = ri.y * p.conv_stride + ky - 1; ix = ri.x * p.conv_stride + kx - 1;
      if (iy < 0 || ix < 0 || iy >= p.H || ix >= p.W) return -1;
    }
    return (ri.b * p.H + iy) * p.W + ix;
  }
  const int f = ri.y + tap - 1;
  if (f < 0 || f >= p.F) return -1;
  return m + (tap - 1) * p.S;
}

template <int BN_, int WM_, int WN_, int AMODE>
__global__ __launch_bounds__(512, 2) void gemm256_kernel(const ActhGemmDesc p, unsigned a_bytes,
                                                         unsigned a2_bytes, unsigned b_bytes, int vec_ok) {
  constexpr int WTM = G_BM / WM_, WTN = BN_ / WN_;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = G_BM * 128;
  constexpr int B_BYTES = BN_ * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NB_INSTR = BN_ / 8;             // B-tile DMA wave-instructions per stage
  constexpr int NB_J = (NB_INSTR + 7) / 8;
  constexpr int EPI_LD = WTN + 4;               // fp32 row stride of a wave's 16-row epilogue slab
  static_assert(WM_ * WN_ == 8, "8 waves");
  static_assert(WTN % 16 == 0 && WTM % 16 == 0, "tile shape");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
  static_assert(8 * 16 * EPI_LD * 4 <= STAGE, "epilogue slab fits in one stage buffer");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN_, wn = wave % WN_;

  // ---- persistent tile schedule -------------------------------------------------------------
  // Tiles are numbered m-major / n-fastest. Block ids are dealt round-robin over the 8 XCDs (b and
  // b + 8 share an L2), so XCD x owns the contiguous tile range [lo_x, hi_x) (bijective split) and
  // its blocks walk it with stride (blocks on x): the tiles that share an A panel run together on
  // one L2. With at most one tile per block (small grids) this degenerates to the plain remap.
  const int ntn = (p.N + BN_ - 1) / BN_;
  const int ntiles = ntn * ((p.M + G_BM - 1) / G_BM);
  const int nblk = gridDim.x;
  const int xcd = blockIdx.x & 7;
  const int q = ntiles >> 3, rr = ntiles & 7;
  const int lo = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  const int hi = lo + q + (xcd < rr ? 1 : 0);
  const int bpx = (nblk - xcd + 7) >> 3;        // blocks on this XCD
  int tile = lo + (int)(blockIdx.x >> 3);
  if (tile >= hi) return;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t ra2 = make_rsrc(p.A2 ? p.A2 : p.A, p.A2 ? a2_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);

  // DMA instruction i (0..31 for A) fills tile rows [8i, 8i+8); wave w issues i = 8j + w.
  // Lane -> (row 8i + lane/8, physical 16-B slot lane%8) holding logical K chunk slot ^ (row & 7).
  const int lrow = lane >> 3;
  const int cch = (lane & 7) ^ lrow;
  // Staging state of the tile whose K tiles are being loaded (one K step ahead of the MFMAs, so at
  // a tile's last K step it already belongs to the next tile). A: per row a byte offset of
  // (source pixel, this lane's K chunk) in each source, >= OOB when the row / tap is padding;
  // recomputed only when the conv tap changes (every Cin/64 K tiles).
  RowInfo ri[4];
  int arow[4];
  unsigned aoff[4], aoff2[4], boff[NB_J];
  int s_tap = 0, s_c0 = 0;
  const bool two_src = p.A2 != nullptr;
  const int cin = AMODE == 0 ? 0x7fffffff : p.Cin;
  auto set_tap = [&](int tap) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pix = tap_pixel<AMODE>(p, arow[j], ri[j], tap);
      aoff[j] = pix < 0 ? OOB : ((unsigned)pix * p.lda + cch * 8) * 2u;
      aoff2[j] = pix < 0 ? OOB : ((unsigned)pix * p.lda2 + cch * 8) * 2u;
    }
  };
  auto init_tile = [&](int t) {
    const int tm = (t / ntn) * G_BM, tn = (t % ntn) * BN_;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      arow[j] = tm + (j * 8 + wave) * 8 + lrow;
      ri[j] = row_info(p, arow[j]);
    }
    set_tap(0);
    s_tap = 0; s_c0 = 0;
#pragma unroll
    for (int j = 0; j < NB_J; ++j) {
      const int brow = tn + (j * 8 + wave) * 8 + lrow;
      boff[j] = brow < p.N ? ((unsigned)brow * p.ldb + cch * 8) * 2u : OOB;
    }
  };

  const int nk = (p.K + G_BK - 1) / G_BK;
  const int kfull = p.K / G_BK;                 // K tiles without a ragged tail

  // stage() is called for kt = 0, 1, 2, ... of one tile in order
  auto stage = [&](int kt, int buf) {
    const int k0 = kt * G_BK;
    char* sA = smem + buf * STAGE;
    char* sB = sA + A_BYTES;
    const int c0 = AMODE == 0 ? k0 : s_c0;
    if (AMODE != 0) {
      if (s_c0 == 0 && s_tap > 0) set_tap(s_tap);   // uniform: first K tile of a new tap
      s_c0 += G_BK;
      if (s_c0 == cin) { s_c0 = 0; ++s_tap; }
    }
    const bool second = two_src && c0 >= p.K1;
    const bool tail = kt >= kfull;              // ragged K tile: lanes past K read zeros
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lds_void* dst = (lds_void*)(sA + (j * 8 + wave) * 1024);
      unsigned off = second ? aoff2[j] + (unsigned)(c0 - p.K1) * 2u : aoff[j] + (unsigned)c0 * 2u;
      if (tail && k0 + cch * 8 >= p.K) off = OOB;
      if (second) __builtin_amdgcn_raw_ptr_buffer_load_lds(ra2, dst, 16, off, 0, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, dst, 16, off, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NB_J; ++j) {
      const int i = j * 8 + wave;
      if (NB_INSTR % 8 == 0 || i < NB_INSTR) {
        unsigned off = boff[j] + (unsigned)k0 * 2u;
        if (tail && k0 + cch * 8 >= p.K) off = OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(sB + i * 1024), 16, off, 0, 0, 0);
      }
    }
  };

  // fragment rows: wave base + 16 t + lane%16; the swizzle key row & 7 == lane & 7
  const int fr = lane & 15, fkey = lane & 7, fq = lane >> 4;
  const int a_base = (wm * WTM + fr) * 128;
  const int b_base = (wn * WTN + fr) * 128;
  const bool geglu = p.act == 2;

  f32x4_t acc[TM][TN];
  init_tile(tile);
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (;;) {
    const int tile_m = (tile / ntn) * G_BM, tile_n = (tile % ntn) * BN_;
    const int next = tile + bpx < hi ? tile + bpx : -1;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};

    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) {
        stage(kt + 1, cur ^ 1);
      } else if (next >= 0) {
        init_tile(next);                        // next tile's first K tile lands during this epilogue
        stage(0, cur ^ 1);
      }
      const char* sA = smem + cur * STAGE;
      const char* sB = sA + A_BYTES;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int sw = ((4 * s + fq) ^ fkey) << 4;
        bf16x8_t af[TM], bfr[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(sB + b_base + j * 16 * 128 + sw);
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8_t*>(sA + a_base + i * 16 * 128 + sw);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
      // next K tile landed (this wave's DMAs) and every wave is done reading `cur`
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      cur ^= 1;
    }

    // ---- epilogue: per-wave 16-row slab inside the stage buffer just consumed -------------------
    if (p.tile & 0x100) {                        // diagnostic: main loop only (keeps acc live)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
      if (next < 0) break;
      __builtin_amdgcn_s_barrier();
      tile = next;
      continue;
    }
    float* et = reinterpret_cast<float*>(smem + (cur ^ 1) * STAGE) + wave * (16 * EPI_LD);
    const int col0 = tile_n + wn * WTN;          // first weight column of this wave
    const int row0 = tile_m + wm * WTM;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) et[(fq * 4 + r) * EPI_LD + j * 16 + fr] = acc[i][j][r];
      // the slab is private to this wave and LDS ops of one wave complete in order
      const int rbase = row0 + i * 16;
      if (geglu) {
        // two (hidden 16 | gate 16) granule pairs per wave -> 32 outputs: 16 rows x 4 chunks
        if (WTN == 64 && col0 < p.N) {
          const int r = lane >> 2, oc = (lane & 3) * 8;
          const int hc = 32 * (oc >> 4) + (oc & 15);
          const int row = rbase + r;
          if (row < p.M)
            epilogue_geglu8(p, row, col0 + hc, col0 + hc + 16, col0 / 2 + oc, &et[r * EPI_LD + hc],
                            &et[r * EPI_LD + hc + 16], vec_ok);
        }
      } else {
        constexpr int CPR = WTN / 8;             // 8-column chunks per row
        for (int ch = lane; ch < 16 * CPR; ch += 64) {
          const int r = ch / CPR, c8 = (ch - r * CPR) * 8;
          const int row = rbase + r, ocol = col0 + c8;
          if (row < p.M && ocol < p.N) {
            float v[8];
            const float4 x0 = *reinterpret_cast<const float4*>(&et[r * EPI_LD + c8]);
            const float4 x1 = *reinterpret_cast<const float4*>(&et[r * EPI_LD + c8 + 4]);
            v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
            epilogue8(p, row, ocol, v, vec_ok);
          }
        }
      }
    }
    if (next < 0) break;
    // every wave's slab reads are done before the next tile's second K tile overwrites the buffer
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    tile = next;
  }
}

template <int BN_, int WM_, int WN_>
static void launch_mode(const ActhGemmDesc* d, dim3 grid, unsigned a_bytes, unsigned a2_bytes, unsigned b_bytes,
                        int vec_ok, hipStream_t stream) {
  if (d->amode == 1)
    hipLaunchKernelGGL((gemm256_kernel<BN_, WM_, WN_, 1>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes, b_bytes,
                       vec_ok);
  else if (d->amode == 2)
    hipLaunchKernelGGL((gemm256_kernel<BN_, WM_, WN_, 2>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes, b_bytes,
                       vec_ok);
  else
    hipLaunchKernelGGL((gemm256_kernel<BN_, WM_, WN_, 0>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes, b_bytes,
                       vec_ok);
}

// launched by acth_gemm (gemm.hip) after its argument checks
int gemm256_launch(const ActhGemmDesc* d, int tile, unsigned a_bytes, unsigned a2_bytes, unsigned b_bytes,
                   int vec_ok, hipStream_t stream) {
  // persistent grid: one 512-thread workgroup per CU (the 128+ KB of LDS admits one), each walking
  // its XCD's tile range
  const long long mt = (d->M + G_BM - 1) / G_BM;
  const int bn = tile == 2 ? 256 : 160;
  const long long ntiles = mt * ((d->N + bn - 1) / bn);
  if (ntiles >= (1ll << 31)) return ACTH_EINVAL;
  const unsigned nblk = (unsigned)(ntiles < PERSIST_BLOCKS ? ntiles : PERSIST_BLOCKS);
  if (tile == 2) {
    launch_mode<256, 2, 4>(d, dim3(nblk), a_bytes, a2_bytes, b_bytes, vec_ok, stream);
  } else if (tile == 3) {
    if (d->act == 2) return ACTH_EINVAL;         // GEGLU granules need 64-column wave tiles
    launch_mode<160, 4, 2>(d, dim3(nblk), a_bytes, a2_bytes, b_bytes, vec_ok, stream);
  } else {
    return ACTH_EINVAL;
  }
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
