// bf16 MFMA GEMM with implicit-conv A loaders and fused epilogues (gfx950).
//
// C[M,N] = epilogue( A[M,K] . B[N,K]^T )
//   * B is a weight matrix stored like nn.Linear.weight: (N, K) row-major, bf16.
//   * A is produced by one of three loaders (all NHWC / token-major activations):
//       dense     : A[m, k] = src[m*lda + k]                      (nn.Linear, 1x1 conv)
//       conv3x3   : A[m, (ky*3+kx)*Cin + c] = img[b, y*s+ky-1, x*s+kx-1, c]   (ResBlock convs,
//                   Downsample2D with s=2, Upsample2D with a nearest-x2 source remap)
//       temporal3 : A[m, kf*Cin + c] = x[(b,f+kf-1,s), c]          (Conv3d kernel (3,1,1))
//     each loader can read its K range from two tensors (channel concat of UNet skips).
//   * epilogue: alpha*acc + bias[n] + rowbias[row/rb_div, n] + R[rmap(row), n],
//     optional SiLU / GELU / GEGLU (h * gelu(g) on interleaved 32-column granules),
//     optional AlphaBlender mix with a second tensor, fp32 or bf16 output, row remap.
//
// Tiling: 128x128x64 workgroup tile, 4 waves (2x2), each wave 64x64 = 2x2 tiles of
// v_mfma_f32_32x32x16_bf16. Operands are register-staged global->LDS (the loaders
// transform addresses, so LDS-DMA's lane-linear destination does not fit), double-buffered,
// one barrier per K-tile. LDS rows padded to 72 bf16 (144 B) so every ds_read_b128
// lane group of 16 rows hits 16 distinct 16-B bank slots.
#include "common.h"


#define BM 128
#define BN 128
#define BKT 64
#define LDSK 72

namespace {

struct RowInfo { int b, y, x; bool ok; };

__device__ __forceinline__ uint4 load_a_chunk(const ActhGemmDesc& p, int m, const RowInfo& ri,
                                              int k0, int kc) {
  uint4 z = make_uint4(0, 0, 0, 0);
  if (!ri.ok) return z;
  const int k = k0 + kc * 8;
  if (k >= p.K) return z;
  if (p.amode == 0) {
    if (k < p.K1) return *reinterpret_cast<const uint4*>((const bf16_t*)p.A + (size_t)m * p.lda + k);
    return *reinterpret_cast<const uint4*>((const bf16_t*)p.A2 + (size_t)m * p.lda2 + (k - p.K1));
  }
  const int tap = k0 / p.Cin;               // uniform over the K tile (Cin % 64 == 0)
  const int c = k - tap * p.Cin;
  size_t pix;
  if (p.amode == 1) {
    const int ky = tap / 3, kx = tap - ky * 3;
    int iy, ix;
    if (p.upsample) {
      iy = ri.y + ky - 1; ix = ri.x + kx - 1;
      if (iy < 0 || ix < 0 || iy >= 2 * p.H || ix >= 2 * p.W) return z;
      iy >>= 1; ix >>= 1;
    } else {
      iy = ri.y * p.conv_stride + ky - 1; ix = ri.x * p.conv_stride + kx - 1;
      if (iy < 0 || ix < 0 || iy >= p.H || ix >= p.W) return z;
    }
    pix = ((size_t)ri.b * p.H + iy) * p.W + ix;
  } else {
    const int f = ri.y + tap - 1;             // ri.y holds the frame index
    if (f < 0 || f >= p.F) return z;
    pix = (size_t)m + (ptrdiff_t)(tap - 1) * p.S;
  }
  if (c < p.K1) return *reinterpret_cast<const uint4*>((const bf16_t*)p.A + pix * p.lda + c);
  return *reinterpret_cast<const uint4*>((const bf16_t*)p.A2 + pix * p.lda2 + (c - p.K1));
}

}  // namespace

__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(const ActhGemmDesc p) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * BM * LDSK];
  bf16_t* sA = smem;                       // [2][BM][LDSK]
  bf16_t* sB = smem + 2 * BM * LDSK;       // [2][BN][LDSK]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tile_n = blockIdx.x * BN;
  const int tile_m = blockIdx.y * BM;

  const int kc = tid & 7;       // 16-byte chunk within a 64-wide K tile
  const int r0 = tid >> 3;      // first of four rows handled by this thread (stride 32)

  RowInfo ri[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = tile_m + r0 + 32 * i;
    ri[i].ok = m < p.M;
    ri[i].b = 0; ri[i].y = 0; ri[i].x = 0;
    if (p.amode == 1) {
      const int hw = p.Ho * p.Wo;
      ri[i].b = m / hw;
      const int rem = m - ri[i].b * hw;
      ri[i].y = rem / p.Wo;
      ri[i].x = rem - ri[i].y * p.Wo;
    } else if (p.amode == 2) {
      ri[i].y = (m / p.S) % p.F;
    }
  }

  const int nk = (p.K + BKT - 1) / BKT;
  uint4 ra[4], rb[4];

  auto gload = [&](int kt) {
    const int k0 = kt * BKT;
#pragma unroll
    for (int i = 0; i < 4; ++i) ra[i] = load_a_chunk(p, tile_m + r0 + 32 * i, ri[i], k0, kc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = tile_n + r0 + 32 * i;
      const int k = k0 + kc * 8;
      rb[i] = (n < p.N && k < p.K)
                  ? *reinterpret_cast<const uint4*>((const bf16_t*)p.B + (size_t)n * p.ldb + k)
                  : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<uint4*>(&sA[(buf * BM + r0 + 32 * i) * LDSK + kc * 8]) = ra[i];
      *reinterpret_cast<uint4*>(&sB[(buf * BN + r0 + 32 * i) * LDSK + kc * 8]) = rb[i];
    }
  };

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  gload(0);
  lstore(0);
  __syncthreads();

  const int r32 = lane & 31, hh = lane >> 5;
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kt + 1);
    const bf16_t* a_base = sA + (cur * BM + wm * 64 + r32) * LDSK + hh * 8;
    const bf16_t* b_base = sB + (cur * BN + wn * 64 + r32) * LDSK + hh * 8;
#pragma unroll
    for (int kk = 0; kk < BKT / 16; ++kk) {
      const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(a_base + kk * 16);
      const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(a_base + 32 * LDSK + kk * 16);
      const bf16x8_t b0 = *reinterpret_cast<const bf16x8_t*>(b_base + kk * 16);
      const bf16x8_t b1 = *reinterpret_cast<const bf16x8_t*>(b_base + 32 * LDSK + kk * 16);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---------------- epilogue ----------------
  if (p.act == 2) {
    // GEGLU: subtile j=0 holds the "hidden" half, j=1 the "gate" half of a 64-col granule
    const int hcol = tile_n + wn * 64 + r32;
    const int gcol = hcol + 32;
    const int ocol = (tile_n + wn * 64) / 2 + r32;
    if (gcol >= p.N) return;
    const float hb = p.bias ? p.bias[hcol] : 0.0f;
    const float gb = p.bias ? p.bias[gcol] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tile_m + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (row >= p.M) continue;
        const float hv = acc[i][0][r] * p.alpha + hb;
        const float gv = acc[i][1][r] * p.alpha + gb;
        const float v = hv * gelu_erf(gv);
        const size_t prow = (size_t)(row / p.orow_div) * p.orow_stride + (row % p.orow_div) + p.orow_off;
        if (p.out_f32) ((float*)p.C)[prow * p.ldc + ocol] = v;
        else ((bf16_t*)p.C)[prow * p.ldc + ocol] = f2bf(v);
      }
    return;
  }

#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = tile_n + wn * 64 + j * 32 + r32;
    if (col >= p.N) continue;
    const float bcol = p.bias ? p.bias[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tile_m + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (row >= p.M) continue;
        float v = acc[i][j][r] * p.alpha + bcol;
        if (p.rowbias) v += p.rowbias[(size_t)(row / p.rb_div) * p.ldrb + col];
        if (p.R) {
          size_t rrow = row;
          if (p.rmap) rrow = (size_t)p.rmap[(row / p.r_div) % p.r_mod] * p.r_div + (row % p.r_div);
          v += bf2f(((const bf16_t*)p.R)[rrow * p.ldr + col]);
        }
        if (p.act == 1) v = silu_f(v);
        else if (p.act == 3) v = gelu_erf(v);
        if (p.MIX) v = p.mix_alpha * bf2f(((const bf16_t*)p.MIX)[(size_t)row * p.ldmix + col]) +
                       (1.0f - p.mix_alpha) * v;
        const size_t prow = (size_t)(row / p.orow_div) * p.orow_stride + (row % p.orow_div) + p.orow_off;
        if (p.out_f32) ((float*)p.C)[prow * p.ldc + col] = v;
        else ((bf16_t*)p.C)[prow * p.ldc + col] = f2bf(v);
      }
  }
}

extern "C" int acth_gemm(const ActhGemmDesc* d, hipStream_t stream) {
  if (!d || !d->A || !d->B || !d->C) return ACTH_EINVAL;
  if (d->M < 0 || d->N <= 0 || d->K <= 0) return ACTH_EINVAL;
  if (d->M == 0) return ACTH_OK;
  if (d->K % 8 || d->K1 % 8 || d->lda % 8 || (d->A2 && d->lda2 % 8) || d->ldb % 8) return ACTH_EINVAL;
  if (d->amode != 0 && (d->Cin % BKT || d->K % d->Cin)) return ACTH_EINVAL;
  if (d->amode == 1 && d->K != 9 * d->Cin) return ACTH_EINVAL;
  if (d->amode == 2 && (d->K != 3 * d->Cin || d->F <= 0 || d->S <= 0)) return ACTH_EINVAL;
  if (d->act == 2 && d->N % 64) return ACTH_EINVAL;
  if (d->orow_div <= 0 || (d->rowbias && d->rb_div <= 0) || (d->rmap && (d->r_div <= 0 || d->r_mod <= 0)))
    return ACTH_EINVAL;
  dim3 grid((d->N + BN - 1) / BN, (d->M + BM - 1) / BM);
  if (grid.y > 65535) return ACTH_EINVAL;
  hipLaunchKernelGGL(gemm_bf16_kernel, grid, dim3(256), 0, stream, *d);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

extern "C" int acth_gemm_desc_size(void) { return (int)sizeof(ActhGemmDesc); }
