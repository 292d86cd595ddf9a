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
// Structure: 128x128x64 workgroup tile, 4 waves (2x2), each wave 64x64 = 2x2 tiles of
// v_mfma_f32_32x32x16_bf16. Operands move HBM/L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds):
// each wave-instruction fills 1 KiB = 8 tile rows x 128 B; the per-lane SOURCE address carries the
// im2col / concat / upsample remapping and an XOR swizzle (chunk ^ (row & 7)) so the MFMA fragment
// reads (ds_read_b128, 16 rows per lane group) spread over the bank row; lanes whose element is
// outside the tensor (conv zero padding, M/N/K tails) get an offset past the buffer's num_records
// and the hardware range check returns zeros. Two LDS stages: the next K tile's DMA is in flight
// while the current one feeds the MFMAs. The epilogue transposes the accumulators through LDS so
// every thread owns 8 consecutive columns of a row: bias / residual / mix loads and the output
// store are 16-byte and fully coalesced.
#include "common.h"

#define BM 128
#define BN 128
#define BKT 64
#define STAGE_BYTES (2 * BM * BKT * 2)        // A + B tile, bf16
#define EPI_LD 132                            // fp32 row stride of the epilogue tile
#define SMEM_BYTES (BM * EPI_LD * 4)          // >= 2 * STAGE_BYTES

typedef __attribute__((address_space(3))) void lds_void;

namespace {

struct RowInfo { int b, y, x; bool ok; };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

constexpr unsigned OOB = 0x80000000u;     // any offset >= num_records reads as zero

// byte offset of the 8-element chunk at (row m, k) inside its source (A, or A2 when `second`:
// uniform over a K tile because K1 % 64 == 0 is required for two-source operands)
__device__ __forceinline__ unsigned a_offset(const ActhGemmDesc& p, int m, const RowInfo& ri, int k0, int k,
                                             bool second) {
  if (!ri.ok || k >= p.K) return OOB;
  if (p.amode == 0) {
    if (!second) return ((unsigned)m * p.lda + k) * 2u;
    return ((unsigned)m * p.lda2 + (k - p.K1)) * 2u;
  }
  const int tap = k0 / p.Cin;               // uniform over the K tile (Cin % 64 == 0)
  const int c = k - tap * p.Cin;
  unsigned pix;
  if (p.amode == 1) {
    const int ky = tap / 3, kx = tap - ky * 3;
    int iy, ix;
    if (p.upsample) {
      iy = ri.y + ky - 1; ix = ri.x + kx - 1;
      if (iy < 0 || ix < 0 || iy >= 2 * p.H || ix >= 2 * p.W) return OOB;
      iy >>= 1; ix >>= 1;
    } else {
      iy = ri.y * p.conv_stride + ky - 1; ix = ri.x * p.conv_stride + kx - 1;
      if (iy < 0 || ix < 0 || iy >= p.H || ix >= p.W) return OOB;
    }
    pix = ((unsigned)ri.b * p.H + iy) * p.W + ix;
  } else {
    const int f = ri.y + tap - 1;             // ri.y holds the frame index
    if (f < 0 || f >= p.F) return OOB;
    pix = (unsigned)(m + (tap - 1) * p.S);
  }
  if (!second) return (pix * p.lda + c) * 2u;
  return (pix * p.lda2 + (c - p.K1)) * 2u;
}

}  // namespace

__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(const ActhGemmDesc p, unsigned a_bytes,
                                                           unsigned a2_bytes, unsigned b_bytes, int vec_ok) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  // readfirstlane: the wave id is uniform, and proving it keeps the LDS-DMA destination (M0)
  // scalar; otherwise hipcc wraps every DMA in a waterfall loop
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: dispatch deals block ids round-robin over the 8 XCDs, so block b and
  // b + 8 share an L2. Give each XCD a contiguous run of (m, n) tiles (n fastest) so the N tiles that
  // share an A panel are read from one L2 (bijective for any grid size).
  const int ntn = gridDim.x;
  const int nwg = gridDim.x * gridDim.y;
  const int bid = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int tile_n = (lin % ntn) * BN;
  const int tile_m = (lin / ntn) * BM;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t ra2 = make_rsrc(p.A2 ? p.A2 : p.A, p.A2 ? a2_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);

  // this lane's DMA slots: instruction j of wave w fills tile rows [32w + 8j, +8), lane -> (row, slot)
  const int lrow = lane >> 3;                // 0..7
  const int pchunk = lane & 7;               // physical 16-B slot in the 128-B LDS row
  RowInfo ri[4];
  int arow[4], brow[4], cchunk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = wave * 32 + j * 8 + lrow;  // tile row 0..127
    cchunk[j] = pchunk ^ (r & 7);            // logical K chunk this lane fetches
    arow[j] = tile_m + r;
    brow[j] = tile_n + r;
    const int m = arow[j];
    ri[j].ok = m < p.M;
    ri[j].b = 0; ri[j].y = 0; ri[j].x = 0;
    if (p.amode == 1) {
      const int hw = p.Ho * p.Wo;
      ri[j].b = m / hw;
      const int rem = m - ri[j].b * hw;
      ri[j].y = rem / p.Wo;
      ri[j].x = rem - ri[j].y * p.Wo;
    } else if (p.amode == 2) {
      ri[j].y = (m / p.S) % p.F;
    }
  }

  const int nk = (p.K + BKT - 1) / BKT;

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BKT;
    char* sA = smem + buf * STAGE_BYTES;
    char* sB = sA + BM * BKT * 2;
    // A2 (skip-connection half of a channel concat) holds K columns [K1, K): one source per K tile
    const bool second = p.A2 && ((p.amode == 0 ? k0 : k0 % p.Cin) >= p.K1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + cchunk[j] * 8;
      const unsigned off = a_offset(p, arow[j], ri[j], k0, k, second);
      lds_void* dst = (lds_void*)(sA + (wave * 32 + j * 8) * 128);
      if (second) __builtin_amdgcn_raw_ptr_buffer_load_lds(ra2, dst, 16, off, 0, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, dst, 16, off, 0, 0, 0);
      const unsigned boff = (brow[j] < p.N && k < p.K) ? ((unsigned)brow[j] * p.ldb + k) * 2u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(sB + (wave * 32 + j * 8) * 128), 16, boff, 0, 0, 0);
    }
  };

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int r32 = lane & 31, hh = lane >> 5;
  // fragment rows read by this lane and their swizzle keys
  const int ar0 = wm * 64 + r32, ar1 = ar0 + 32;
  const int br0 = wn * 64 + r32, br1 = br0 + 32;

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* sA = smem + cur * STAGE_BYTES;
    const char* sB = sA + BM * BKT * 2;
#pragma unroll
    for (int kk = 0; kk < BKT / 16; ++kk) {
      const int c = kk * 2 + hh;
      const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(sA + ar0 * 128 + ((c ^ (ar0 & 7)) << 4));
      const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(sA + ar1 * 128 + ((c ^ (ar1 & 7)) << 4));
      const bf16x8_t b0 = *reinterpret_cast<const bf16x8_t*>(sB + br0 * 128 + ((c ^ (br0 & 7)) << 4));
      const bf16x8_t b1 = *reinterpret_cast<const bf16x8_t*>(sB + br1 * 128 + ((c ^ (br1 & 7)) << 4));
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
    // next tile landed (this wave's DMAs) and every wave is done reading `cur`
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur ^= 1;
  }

  // ---------------- epilogue: accumulators -> LDS (fp32 [128][EPI_LD]) -> row-contiguous ----------
  float* et = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const int col = wn * 64 + j * 32 + r32;
        et[row * EPI_LD + col] = acc[i][j][r];
      }
  __syncthreads();

  const bool geglu = p.act == 2;
  // each thread: 8 consecutive output columns of a row; 16 (or 8 for GEGLU) threads per row
  const int tpr = geglu ? 8 : 16;
  const int rows_per_pass = 256 / tpr;
  const int cg = tid % tpr;
  for (int r0 = tid / tpr; r0 < BM; r0 += rows_per_pass) {
    const int row = tile_m + r0;
    if (row >= p.M) break;
    const size_t prow = (size_t)(row / p.orow_div) * p.orow_stride + (row % p.orow_div) + p.orow_off;
    float v[8];
    int ocol;
    if (geglu) {
      // output columns [tile_n/2 + 8cg, +8): hidden at tile col 64g + j, gate at 64g + 32 + j
      const int oc = cg * 8;                       // 0..63 within the tile's 64 output columns
      const int g = oc >> 5, j0 = oc & 31;
      const int hc = 64 * g + j0, gc = hc + 32;
      ocol = tile_n / 2 + oc;
      if (tile_n + gc >= p.N) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float hv = et[r0 * EPI_LD + hc + e] * p.alpha + (p.bias ? p.bias[tile_n + hc + e] : 0.0f);
        const float gv = et[r0 * EPI_LD + gc + e] * p.alpha + (p.bias ? p.bias[tile_n + gc + e] : 0.0f);
        v[e] = hv * gelu_erf(gv);
      }
    } else {
      const int c0 = cg * 8;
      ocol = tile_n + c0;
      if (ocol >= p.N) continue;
      const bool full = vec_ok && ocol + 8 <= p.N;
      const float4 x0 = *reinterpret_cast<const float4*>(&et[r0 * EPI_LD + c0]);
      const float4 x1 = *reinterpret_cast<const float4*>(&et[r0 * EPI_LD + c0 + 4]);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= p.alpha;
      if (p.bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (ocol + e < p.N) ? p.bias[ocol + e] : 0.0f;
      }
      if (p.rowbias) {
        const float* rb2 = p.rowbias + (size_t)(row / p.rb_div) * p.ldrb + ocol;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (ocol + e < p.N) ? rb2[e] : 0.0f;
      }
      if (p.R) {
        size_t rrow = row;
        if (p.rmap) rrow = (size_t)p.rmap[(row / p.r_div) % p.r_mod] * p.r_div + (row % p.r_div);
        const bf16_t* rp = (const bf16_t*)p.R + rrow * p.ldr + ocol;
        float t[8];
        if (full) {
          unpack8(*reinterpret_cast<const uint4*>(rp), t);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] = (ocol + e < p.N) ? bf2f(rp[e]) : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
      }
      if (p.act == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = silu_f(v[e]);
      } else if (p.act == 3) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
      }
      if (p.MIX) {
        const bf16_t* mp = (const bf16_t*)p.MIX + (size_t)row * p.ldmix + ocol;
        float t[8];
        if (full) {
          unpack8(*reinterpret_cast<const uint4*>(mp), t);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] = (ocol + e < p.N) ? bf2f(mp[e]) : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = p.mix_alpha * t[e] + (1.0f - p.mix_alpha) * v[e];
      }
      if (!full) {
        for (int e = 0; e < 8 && ocol + e < p.N; ++e) {
          if (p.out_f32) ((float*)p.C)[prow * p.ldc + ocol + e] = v[e];
          else ((bf16_t*)p.C)[prow * p.ldc + ocol + e] = f2bf(v[e]);
        }
        continue;
      }
    }
    if (!vec_ok) {
      for (int e = 0; e < 8; ++e) {
        if (p.out_f32) ((float*)p.C)[prow * p.ldc + ocol + e] = v[e];
        else ((bf16_t*)p.C)[prow * p.ldc + ocol + e] = f2bf(v[e]);
      }
      continue;
    }
    if (p.out_f32) {
      float* cp = (float*)p.C + prow * p.ldc + ocol;
      *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      *reinterpret_cast<uint4*>((bf16_t*)p.C + prow * p.ldc + ocol) = pack8(v);
    }
  }
}

extern "C" int acth_gemm(const ActhGemmDesc* d, hipStream_t stream) {
  if (!d || !d->A || !d->B || !d->C) return ACTH_EINVAL;
  if (d->M < 0 || d->N <= 0 || d->K <= 0) return ACTH_EINVAL;
  if (d->M == 0) return ACTH_OK;
  if (d->K % 8 || d->lda % 8 || (d->A2 && (d->lda2 % 8 || d->K1 % 64)) || d->ldb % 8) return ACTH_EINVAL;
  // 16-byte epilogue vectors need 16-byte aligned rows in C / R / MIX; otherwise scalar path
  const int esz = d->out_f32 ? 4 : 2;
  const int vec_ok = ((size_t)d->C % 16 == 0) && ((d->ldc * esz) % 16 == 0) &&
                     (!d->R || ((size_t)d->R % 16 == 0 && d->ldr % 8 == 0)) &&
                     (!d->MIX || ((size_t)d->MIX % 16 == 0 && d->ldmix % 8 == 0));
  if (d->amode != 0 && (d->Cin % BKT || d->K % d->Cin)) return ACTH_EINVAL;
  if (d->amode == 1 && d->K != 9 * d->Cin) return ACTH_EINVAL;
  if (d->amode == 2 && (d->K != 3 * d->Cin || d->F <= 0 || d->S <= 0)) return ACTH_EINVAL;
  if (d->act == 2 && d->N % 64) return ACTH_EINVAL;
  if (d->orow_div <= 0 || (d->rowbias && d->rb_div <= 0) || (d->rmap && (d->r_div <= 0 || d->r_mod <= 0)))
    return ACTH_EINVAL;
  // operand extents (buffer num_records): rows of each A source and of B
  long long a_rows, a2_rows;
  if (d->amode == 1) a_rows = a2_rows = (long long)(d->M / (d->Ho * d->Wo)) * d->H * d->W;
  else a_rows = a2_rows = d->M;
  const int c1 = d->A2 ? d->K1 : (d->amode == 0 ? d->K : d->Cin);
  const long long a_bytes = ((a_rows - 1) * (long long)d->lda + (d->A2 ? c1 : (d->amode == 0 ? d->K : d->Cin))) * 2;
  const long long a2_bytes = d->A2 ? ((a2_rows - 1) * (long long)d->lda2 +
                                      ((d->amode == 0 ? d->K : d->Cin) - c1)) * 2 : 0;
  const long long b_bytes = ((long long)(d->N - 1) * d->ldb + d->K) * 2;
  if (a_bytes >= 0x80000000LL || a2_bytes >= 0x80000000LL || b_bytes >= 0x80000000LL) return ACTH_EINVAL;
  dim3 grid((d->N + BN - 1) / BN, (d->M + BM - 1) / BM);
  if (grid.y > 65535) return ACTH_EINVAL;
  hipLaunchKernelGGL(gemm_bf16_kernel, grid, dim3(256), 0, stream, *d, (unsigned)a_bytes,
                     (unsigned)a2_bytes, (unsigned)b_bytes, vec_ok);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

extern "C" int acth_gemm_desc_size(void) { return (int)sizeof(ActhGemmDesc); }
