// Normalisation kernels on token-major (rows x C) bf16 activations.
//
//  * acth_layernorm      : nn.LayerNorm over C per token, optional fused "x + rowvec[row/div]"
//                          pre-add (frame position embedding before the temporal block,
//                          TransformerSTmodel.py:4125-4126) that also writes the sum.
//  * acth_groupnorm_*    : nn.GroupNorm(32) with statistics spanning rows_per_stat tokens
//                          (one frame for spatial blocks, a whole F-frame window for
//                          diffusers' TemporalResnetBlock), optional SiLU, optional two-tensor
//                          channel concat input (UNet skip connections).
//  * acth_mamba_combine_ln: SS2D_cond_v10's "xz1[sel] = scan_audio; xz2[sel] = scan_exp;
//                          out_norm(xz1 + xz2)" (mamba_layer.py:1963-1985) in one pass: each
//                          branch's value is either its in_proj row or the sum of its two scan
//                          directions at the token's position in the selected sequence.
#include "common.h"

#define MAXCH 8   // max 16-byte chunks per lane: C <= 64 * 8 * 8 = 4096

// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void layernorm_ragged_kernel(const ActhLayerNormDesc p) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.M) return;
  const int nch = p.C >> 3;
  float v[MAXCH][8];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch) {
      unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)p.x + row * p.ldx + ch * 8), v[i]);
      if (p.add) {
        float a[8];
        unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)p.add + (row / p.add_div) * p.ldadd + ch * 8), a);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] += a[e];
        if (p.sum_out) {
          // round the sum to bf16 as the stored tensor will be, and normalise that value
          const uint4 w = pack8(v[i]);
          *reinterpret_cast<uint4*>((bf16_t*)p.sum_out + row * p.ldsum + ch * 8) = w;
          unpack8(w, v[i]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    }
  }
  const float mean = wave_sum(s) / p.C;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / p.C + p.eps);
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = ch * 8 + e;
        o[e] = (v[i][e] - mean) * rstd * (p.gamma ? p.gamma[c] : 1.0f) + (p.beta ? p.beta[c] : 0.0f);
      }
      *reinterpret_cast<uint4*>((bf16_t*)p.y + row * p.ldy + ch * 8) = pack8(o);
    }
  }
}

// One row per LPR-lane group (64/LPR rows per wave), CPL 16-byte chunks per lane: every lane has
// all of its row's loads in flight at once, which is what a 640-2560-byte row needs to approach
// HBM bandwidth (one row per wave leaves most lanes idle and one load per lane in flight).
template <int LPR, int CPL>
__global__ __launch_bounds__(256) void layernorm_kernel(const ActhLayerNormDesc p) {
  // gamma | beta staged in LDS (dynamic, 2 C floats) when a block holds >= 16 rows (LPR <= 16): their
  // global loads are issued before the row loads and land while the row statistics are reduced, instead
  // of after them (level 0 / 1: -5 / -3 %); with 8 rows per block the staging costs more than it hides
  constexpr bool STAGE = LPR <= 16;
  extern __shared__ float ln_gb[];
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, l = lane - sub * LPR;
  const long long row = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / LPR) + sub;
  const bool ok = row < p.M;
  const long long rr = ok ? row : 0;
  float gbv[(2 * LPR * CPL * 8 + 255) / 256];
#pragma unroll
  for (int k = 0; k < (STAGE ? (2 * LPR * CPL * 8 + 255) / 256 : 0); ++k) {
    const int i = threadIdx.x + 256 * k;
    const int c = i < p.C ? i : i - p.C;
    const float* src = i < p.C ? p.gamma : p.beta;
    gbv[k] = (i < 2 * p.C) ? (src ? src[c] : (i < p.C ? 1.0f : 0.0f)) : 0.0f;
  }
  float v[CPL][8];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
    unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)p.x + rr * p.ldx + (l + LPR * i) * 8), v[i]);
  if constexpr (STAGE) {
#pragma unroll
    for (int k = 0; k < (2 * LPR * CPL * 8 + 255) / 256; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < 2 * p.C) ln_gb[i] = gbv[k];
    }
    __syncthreads();
  }
  if (p.add) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int ch = l + LPR * i;
      float a[8];
      unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)p.add + (rr / p.add_div) * p.ldadd + ch * 8), a);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] += a[e];
      // round the sum to bf16 as the stored tensor will be, and normalise that value
      const uint4 w = pack8(v[i]);
      if (p.sum_out && ok) *reinterpret_cast<uint4*>((bf16_t*)p.sum_out + rr * p.ldsum + ch * 8) = w;
      if (p.sum_out) unpack8(w, v[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[i][e];
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / p.C;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q += d * d; }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q / p.C + p.eps);
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int ch = l + LPR * i;
    float g[8], b[8], o[8];
    if constexpr (STAGE) {
      const float4 g0 = reinterpret_cast<const float4*>(ln_gb + ch * 8)[0];
      const float4 g1 = reinterpret_cast<const float4*>(ln_gb + ch * 8)[1];
      g[0] = g0.x; g[1] = g0.y; g[2] = g0.z; g[3] = g0.w; g[4] = g1.x; g[5] = g1.y; g[6] = g1.z; g[7] = g1.w;
      const float4 b0 = reinterpret_cast<const float4*>(ln_gb + p.C + ch * 8)[0];
      const float4 b1 = reinterpret_cast<const float4*>(ln_gb + p.C + ch * 8)[1];
      b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
    } else {
      if (p.gamma) {
        const float4 g0 = reinterpret_cast<const float4*>(p.gamma + ch * 8)[0];
        const float4 g1 = reinterpret_cast<const float4*>(p.gamma + ch * 8)[1];
        g[0] = g0.x; g[1] = g0.y; g[2] = g0.z; g[3] = g0.w; g[4] = g1.x; g[5] = g1.y; g[6] = g1.z; g[7] = g1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = 1.0f;
      }
      if (p.beta) {
        const float4 b0 = reinterpret_cast<const float4*>(p.beta + ch * 8)[0];
        const float4 b1 = reinterpret_cast<const float4*>(p.beta + ch * 8)[1];
        b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) b[e] = 0.0f;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + b[e];
    *reinterpret_cast<uint4*>((bf16_t*)p.y + row * p.ldy + ch * 8) = pack8(o);
  }
}

template <int LPR>
static void ln_launch(const ActhLayerNormDesc* d, int cpl, hipStream_t stream) {
  const long long rows_per_blk = 4LL * (64 / LPR);
  const dim3 grid((unsigned)((d->M + rows_per_blk - 1) / rows_per_blk));
  switch (cpl) {
    case 1: hipLaunchKernelGGL((layernorm_kernel<LPR, 1>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
    case 2: hipLaunchKernelGGL((layernorm_kernel<LPR, 2>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
    case 3: hipLaunchKernelGGL((layernorm_kernel<LPR, 3>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
    case 4: hipLaunchKernelGGL((layernorm_kernel<LPR, 4>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
    case 5: hipLaunchKernelGGL((layernorm_kernel<LPR, 5>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
    case 6: hipLaunchKernelGGL((layernorm_kernel<LPR, 6>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
    case 7: hipLaunchKernelGGL((layernorm_kernel<LPR, 7>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
    default: hipLaunchKernelGGL((layernorm_kernel<LPR, 8>), grid, dim3(256), LPR <= 16 ? 2 * d->C * sizeof(float) : 0, stream, *d); break;
  }
}

// widths that are not a multiple of 8 (VasaProjModel's 1018-wide output, audio_proj.py:147-150):
// one wave per row, scalar bf16 loads, two-pass mean / variance from registers-free re-reads
__global__ __launch_bounds__(256) void layernorm_scalar_kernel(const ActhLayerNormDesc p) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.M) return;
  const bf16_t* x = (const bf16_t*)p.x + row * p.ldx;
  float s = 0.0f;
  for (int c = lane; c < p.C; c += 64) s += bf2f(x[c]);
  const float mean = wave_sum(s) / p.C;
  float q = 0.0f;
  for (int c = lane; c < p.C; c += 64) { const float d = bf2f(x[c]) - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) / p.C + p.eps);
  bf16_t* y = (bf16_t*)p.y + row * p.ldy;
  for (int c = lane; c < p.C; c += 64) {
    float o = (bf2f(x[c]) - mean) * rstd;
    if (p.gamma) o = o * p.gamma[c] + (p.beta ? p.beta[c] : 0.0f);
    y[c] = f2bf(o);
  }
}

extern "C" int acth_layernorm(const ActhLayerNormDesc* d, hipStream_t stream) {
  if (d && d->M == 0) return ACTH_OK;   // no rows: nothing read or written
  if (d && d->x && d->y && d->C > 0 && (d->C % 8 || d->ldx % 8 || d->ldy % 8) && !d->add && !d->sum_out &&
      d->ldx >= d->C && d->ldy >= d->C) {
    if (d->M == 0) return ACTH_OK;
    hipLaunchKernelGGL(layernorm_scalar_kernel, dim3((unsigned)((d->M + 3) / 4)), dim3(256), 0, stream, *d);
    ACTH_CHECK_LAUNCH();
    return ACTH_OK;
  }
  if (!d || !d->x || !d->y || d->C <= 0 || d->C % 8 || d->C > 64 * 8 * MAXCH) return ACTH_EINVAL;
  if (d->ldx % 8 || d->ldy % 8 || (d->add && (d->ldadd % 8 || d->add_div <= 0)) || (d->sum_out && d->ldsum % 8))
    return ACTH_EINVAL;
  if (d->M == 0) return ACTH_OK;
  // lanes per row: the smallest of 4..64 that leaves at most 8 chunks per lane and divides the row;
  // other widths (and unaligned gamma/beta) take the one-row-per-wave kernel
  const int nch = d->C / 8;
  int lpr = 0;
  for (int c = 4; c <= 64; c *= 2)
    if (nch % c == 0 && nch / c <= 8) { lpr = c; break; }
  if (!lpr || ((size_t)d->gamma | (size_t)d->beta) % 16) {
    hipLaunchKernelGGL(layernorm_ragged_kernel, dim3((unsigned)((d->M + 3) / 4)), dim3(256), 0, stream, *d);
    ACTH_CHECK_LAUNCH();
    return ACTH_OK;
  }
  const int cpl = nch / lpr;
  if (lpr == 4) ln_launch<4>(d, cpl, stream);
  else if (lpr == 8) ln_launch<8>(d, cpl, stream);
  else if (lpr == 16) ln_launch<16>(d, cpl, stream);
  else if (lpr == 32) ln_launch<32>(d, cpl, stream);
  else ln_launch<64>(d, cpl, stream);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// GroupNorm. Rows are tokens; statistics batch = row / rows_per_stat; group = c / (C/G).
// Input may be the channel concat of x (C1 channels) and x2 (C - C1 channels).

// Statistics: each block reduces gs_rows rows of one statistics batch to per-channel fp32 partial
// sums (LDS), folds them in a fixed order to per-group fp64 sums and adds those to fp64
// accumulators (2*G doubles per batch; fp64 sums of fp32 partials are exact in practice, so the
// cross-block atomics do not make the result order-dependent). Apply: each block covers rows of a single batch, turns (mean, rstd, gamma, beta) into a
// per-channel scale/shift once, then streams y = x * a + b (+ SiLU) with 16-byte accesses.
// Thread layout of both: nchl = min(C/8, 256) chunk columns x (256 / nchl) row lanes; a thread
// owns chunk columns cl and cl + nchl (C <= 4096).


__device__ __forceinline__ uint4 gn_load(const ActhGroupNormDesc& p, long long row, int ch) {
  const int c = ch * 8;
  if (c < p.C1) return *reinterpret_cast<const uint4*>((const bf16_t*)p.x + row * p.ldx + c);
  return *reinterpret_cast<const uint4*>((const bf16_t*)p.x2 + row * p.ldx2 + (c - p.C1));
}

// grid: (ceil(rows_per_stat / gs_rows), nstat); gs_rows (rows per block) is
// sized on the host so the grid is one round of resident blocks (>= 64 rows each: the per-block fold
// below is serial, so fewer, fuller blocks keep the pass streaming; 128-row blocks ran at ~3.2 TB/s)
__global__ __launch_bounds__(256) void gn_stats_kernel(const ActhGroupNormDesc p, int gs_rows) {
  // per row lane, per channel partial sums (written once each, reduced in a fixed order below, so
  // the statistics are bit-reproducible): rows_par * 2C <= 8192 floats for C <= 4096
  __shared__ float red[8192];
  const int nch = p.C >> 3;
  const int nchl = nch < 256 ? nch : 256;
  const int rows_par = 256 / nchl;
  const int t = threadIdx.x;
  const int stat = blockIdx.y;
  const long long r_begin = (long long)stat * p.rows_per_stat + (long long)blockIdx.x * gs_rows;
  const long long r_end = min((long long)stat * p.rows_per_stat + p.rows_per_stat, r_begin + gs_rows);
  const int rl = t / nchl, cl = t - rl * nchl;
  if (rl < rows_par) {
    for (int ch = cl; ch < nch; ch += nchl) {
      float s1[8], s2[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] = 0.0f; s2[e] = 0.0f; }
      long long r = r_begin + rl;
      for (; r + 3 * rows_par < r_end; r += 4 * rows_par) {
        uint4 w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = gn_load(p, r + u * rows_par, ch);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float v[8];
          unpack8(w[u], v);
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[e] += v[e]; s2[e] += v[e] * v[e]; }
        }
      }
      for (; r < r_end; r += rows_par) {
        float v[8];
        unpack8(gn_load(p, r, ch), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) { s1[e] += v[e]; s2[e] += v[e] * v[e]; }
      }
      float* dst = red + rl * 2 * p.C + ch * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) { dst[e] = s1[e]; dst[p.C + e] = s2[e]; }
    }
  }
  __syncthreads();
  const int cpg = p.C / p.G;
  if (t < p.G) {
    double a1 = 0.0, a2 = 0.0;
    for (int r = 0; r < rows_par; ++r)
      for (int c = t * cpg; c < (t + 1) * cpg; ++c) { a1 += red[r * 2 * p.C + c]; a2 += red[r * 2 * p.C + p.C + c]; }
    // this block's partial sums in its own slot (no atomics, no zeroed workspace): gn_apply_kernel adds a
    // statistics batch's slots in block order, so the statistics are bitwise reproducible run to run
    double* part = p.ws + (((size_t)stat * gridDim.x + blockIdx.x) * p.G + t) * 2;
    part[0] = a1;
    part[1] = a2;
  }
}

// y = act(x * a + b [+ res]) for one 8-channel chunk of a row, stored as 16 bytes
__device__ __forceinline__ void gn_finish(const ActhGroupNormDesc& p, long long row, int ch, float* v, const float* sa,
                                          const float* sb) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = v[e] * sa[e] + sb[e];
  if (p.res) {
    float r[8];
    unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)p.res + row * p.ldres + ch * 8), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  }
  if (p.silu == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = silu_f(v[e]);
  } else if (p.silu == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.0f);
  }
  *reinterpret_cast<uint4*>((bf16_t*)p.y + row * p.ldy + ch * 8) = pack8(v);
}

#define GN_MAX_GROUPS 1024
// grid: M / rows_per_blk blocks; every block's rows lie in one statistics batch
__global__ __launch_bounds__(256) void gn_apply_kernel(const ActhGroupNormDesc p, int rows_per_blk, int nblk) {
  const int nch = p.C >> 3;
  const int nchl = nch < 256 ? nch : 256;
  const int rows_par = 256 / nchl;
  const int t = threadIdx.x;
  const int rl = t / nchl, cl = t - rl * nchl;
  const long long row0 = (long long)blockIdx.x * rows_per_blk;
  const int stat = (int)(row0 / p.rows_per_stat);
  const int cpg = p.C / p.G;
  // per-group mean / rstd once per block (one fp64 divide + sqrt per group, not per channel and
  // thread: the per-channel form spent more issue on fp64 divides and square roots than the
  // block's 128 rows of streaming)
  __shared__ float s_mean[GN_MAX_GROUPS], s_rstd[GN_MAX_GROUPS];
  __shared__ double s_a[2][256];
  {
    const double n = (double)cpg * p.rows_per_stat;
    // the nblk stats blocks' partial sums of this batch: lane j of group g adds slots j, j + lanes, ... (at
    // most a few independent loads per thread), then the lanes are folded in lane order -- a fixed order
    const double* part = p.ws + (size_t)stat * nblk * p.G * 2;
    const int lanes = p.G <= 256 ? 256 / p.G : 1;
    if (lanes > 1) {
      const int g = t % p.G, j = t / p.G;
      double a1 = 0.0, a2 = 0.0;
      if (j < lanes)
        for (int k = j; k < nblk; k += lanes) {
          const double* q = part + ((size_t)k * p.G + g) * 2;
          a1 += q[0];
          a2 += q[1];
        }
      s_a[0][t] = a1;
      s_a[1][t] = a2;
      __syncthreads();
    }
    for (int g = t; g < p.G; g += 256) {
      double a1 = 0.0, a2 = 0.0;
      if (lanes > 1) {
        for (int j = 0; j < lanes; ++j) {
          a1 += s_a[0][j * p.G + g];
          a2 += s_a[1][j * p.G + g];
        }
      } else {
        for (int k = 0; k < nblk; ++k) {
          a1 += part[((size_t)k * p.G + g) * 2];
          a2 += part[((size_t)k * p.G + g) * 2 + 1];
        }
      }
      const double mean = a1 / n;
      double var = a2 / n - mean * mean;
      if (var < 0.0) var = 0.0;
      s_mean[g] = (float)mean;
      s_rstd[g] = (float)(1.0 / sqrt(var + (double)p.eps));
    }
  }
  __syncthreads();
  if (rl >= rows_par) return;
  float sa[2][8], sb[2][8];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ch = cl + k * nchl;
    if (ch < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = ch * 8 + e, g = c / cpg;
        sa[k][e] = s_rstd[g] * p.gamma[c];
        sb[k][e] = p.beta[c] - s_mean[g] * sa[k][e];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ch = cl + k * nchl;
    if (ch >= nch) break;
    int r = rl;
    for (; r + 3 * rows_par < rows_per_blk; r += 4 * rows_par) {
      uint4 w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = gn_load(p, row0 + r + u * rows_par, ch);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v[8];
        unpack8(w[u], v);
        gn_finish(p, row0 + r + u * rows_par, ch, v, sa[k], sb[k]);
      }
    }
    for (; r < rows_per_blk; r += rows_par) {
      float v[8];
      unpack8(gn_load(p, row0 + r, ch), v);
      gn_finish(p, row0 + r, ch, v, sa[k], sb[k]);
    }
  }
}

// Row span per statistics block: as many blocks as the chip holds at once (its 32 KB of LDS allow 5 per
// CU), split evenly over the statistics batches, so the pass is one full round of blocks (the former
// power-of-two spans gave 1512 blocks against 1280 slots at every UNet level: a second, 18 % round).
// *nblk: stats blocks per batch (each owns a G x 2 fp64 partial-sum slot of the workspace).
static void gn_split(long long nstat, int rows_per_stat, int* gs_rows, int* nblk) {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, ncu = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || ncu <= 0)
      ncu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gn_stats_kernel, 256, 0) != hipSuccess || per_cu <= 0)
      per_cu = 4;
    slots = ncu * per_cu;
  }
  const long long per_stat = nstat >= slots ? 1 : slots / nstat;
  int g = (int)((rows_per_stat + per_stat - 1) / per_stat);
  if (g < 64) g = 64;
  *gs_rows = g;
  *nblk = (rows_per_stat + g - 1) / g;
}

extern "C" size_t acth_groupnorm_workspace_size(int M, int C, int G, int rows_per_stat) {
  if (rows_per_stat <= 0 || M <= 0 || G <= 0) return 0;
  const long long nstat = M / rows_per_stat;
  if (nstat == 0) return 0;
  int gs_rows = 0, nblk = 0;
  gn_split(nstat, rows_per_stat, &gs_rows, &nblk);
  return (size_t)nstat * nblk * G * 2 * sizeof(double);
}

extern "C" int acth_groupnorm(const ActhGroupNormDesc* d, hipStream_t stream) {
  if (d && d->M == 0) return ACTH_OK;   // no rows: nothing read or written
  if (!d || !d->x || !d->y || !d->ws || !d->gamma || !d->beta) return ACTH_EINVAL;
  if (d->C % 8 || d->C1 % 8 || d->G <= 0 || d->C % d->G || d->rows_per_stat <= 0) return ACTH_EINVAL;
  if (d->M % d->rows_per_stat) return ACTH_EINVAL;
  if (d->C1 < d->C && (!d->x2 || d->ldx2 % 8)) return ACTH_EINVAL;
  if (d->ldx % 8 || d->ldy % 8 || d->C > 4096 || d->silu < 0 || d->silu > 2) return ACTH_EINVAL;
  if (d->G > GN_MAX_GROUPS) return ACTH_EINVAL;
  if (d->res && d->ldres % 8) return ACTH_EINVAL;
  const int nstat = d->M / d->rows_per_stat;
  if (nstat == 0) return ACTH_OK;
  if (nstat > 65535) return ACTH_EINVAL;
  // the workspace (acth_groupnorm_workspace_size bytes) needs no clearing: every slot is written by the stats
  // pass before the apply pass reads it
  int gs_rows = 0, nblk = 0;
  gn_split(nstat, d->rows_per_stat, &gs_rows, &nblk);
  dim3 g1(nblk, nstat);
  hipLaunchKernelGGL(gn_stats_kernel, g1, dim3(256), 0, stream, *d, gs_rows);
  ACTH_CHECK_LAUNCH();
  int rpb = 128;
  while (d->rows_per_stat % rpb) rpb >>= 1;
  // fewer rows per block while the grid would not fill the chip twice over (2048 = 8 resident blocks on
  // each of 256 CUs): the level-1 / level-2 shapes had 1512 / 378 blocks of 128 rows
  while (rpb > 32 && (d->M / rpb) < 4096 && d->rows_per_stat % (rpb >> 1) == 0) rpb >>= 1;
  hipLaunchKernelGGL(gn_apply_kernel, dim3((unsigned)(d->M / rpb)), dim3(256), 0, stream, *d, rpb, nblk);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// Mamba combine + LayerNorm. Per branch: mode 0 = nothing selected (row of x), 1 = every
// token selected in order (scan row b*L + s), 2 = position map pos[s] (-1 = unselected).

// Layout: LPR lanes per row (16 / 32 / 64 by width), so a wave combines 64 / LPR rows at once and
// every lane has up to CPL 16-byte chunks of each source in flight before the first use (the
// one-row-per-wave form it replaces ran at ~1.1 TB/s: one latency round trip per row).
// Row reductions are xor-shuffles inside the row's lane group.
__device__ __forceinline__ const bf16_t* mc_src(const void* x, int ldx, const void* y0, const void* y1, int ldyy,
                                                int L, const int* pos, int mode, long long row, int S,
                                                const bf16_t** second) {
  const long long b = row / S;
  const int s = (int)(row - b * S);
  int j = -1;
  if (mode == 1) j = s;
  else if (mode == 2) j = pos[s];
  if (j < 0) {
    *second = nullptr;
    return (const bf16_t*)x + row * ldx;
  }
  const long long r = b * L + j;
  *second = (const bf16_t*)y1 + r * ldyy;
  return (const bf16_t*)y0 + r * ldyy;
}

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int LPR, int CPL>
__global__ __launch_bounds__(256) void mamba_combine_kernel(const ActhMambaCombineDesc p) {
  constexpr int RPW = 64 / LPR;                  // rows per wave
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, gl = lane % LPR;
  const long long row = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + sub;
  const bool ok = row < p.M;
  const long long rw = ok ? row : 0;
  const int nch = p.C >> 3;
  const bf16_t *a0, *a1, *e0, *e1;
  a0 = mc_src(p.xa, p.ldxa, p.ya0, p.ya1, p.ldya, p.La, p.pos_a, p.mode_a, rw, p.S, &a1);
  e0 = mc_src(p.xe, p.ldxe, p.ye0, p.ye1, p.ldye, p.Le, p.pos_e, p.mode_e, rw, p.S, &e1);
  uint4 ra0[CPL], ra1[CPL], re0[CPL], re1[CPL];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int ch = gl + LPR * i;
    const bool c_ok = ok && ch < nch;
    const uint4 z = make_uint4(0, 0, 0, 0);
    // plain guarded loads: the `cond ? *p : z` form was lowered through a private stack slot
    ra0[i] = z; ra1[i] = z; re0[i] = z; re1[i] = z;
    if (c_ok) {
      ra0[i] = *reinterpret_cast<const uint4*>(a0 + ch * 8);
      re0[i] = *reinterpret_cast<const uint4*>(e0 + ch * 8);
      if (a1) ra1[i] = *reinterpret_cast<const uint4*>(a1 + ch * 8);
      if (e1) re1[i] = *reinterpret_cast<const uint4*>(e1 + ch * 8);
    }
  }
  float v[CPL][8];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    float t0[8], t1[8], t2[8], t3[8];
    unpack8(ra0[i], t0); unpack8(ra1[i], t1); unpack8(re0[i], t2); unpack8(re1[i], t3);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // (y0 + y1) + (x or y0' + y1'): a branch's two scan directions are summed first, as in
      // the reference's y = out[:, 0] + flip(out[:, 1]) before the cross-branch add
      v[i][e] = (t0[e] + t1[e]) + (t2[e] + t3[e]);
      s += v[i][e];
    }
  }
  const float mean = group_sum<LPR>(s) / p.C;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    if (gl + LPR * i < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(group_sum<LPR>(q) / p.C + p.eps);
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int ch = gl + LPR * i;
    if (ch < nch) {
      const float4 g0 = *reinterpret_cast<const float4*>(p.gamma + ch * 8);
      const float4 g1 = *reinterpret_cast<const float4*>(p.gamma + ch * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(p.beta + ch * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(p.beta + ch * 8 + 4);
      const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + bb[e];
      *reinterpret_cast<uint4*>((bf16_t*)p.y + row * p.ldy + ch * 8) = pack8(o);
    }
  }
}

extern "C" int acth_mamba_combine_ln(const ActhMambaCombineDesc* d, hipStream_t stream) {
  if (d && d->M == 0) return ACTH_OK;   // no rows: nothing read or written
  if (!d || !d->y || !d->gamma || !d->beta) return ACTH_EINVAL;
  if (d->C % 8 || d->C > 64 * 8 * 6 || d->S <= 0 || d->M % d->S) return ACTH_EINVAL;
  if (((size_t)d->gamma | (size_t)d->beta) & 15) return ACTH_EINVAL;
  const int modes[2] = {d->mode_a, d->mode_e};
  const void* xs[2] = {d->xa, d->xe};
  const void* ys[2] = {d->ya0, d->ye0};
  const void* ys1[2] = {d->ya1, d->ye1};
  const int* ps[2] = {d->pos_a, d->pos_e};
  for (int i = 0; i < 2; ++i) {
    if (modes[i] < 0 || modes[i] > 2) return ACTH_EINVAL;
    if (modes[i] != 1 && !xs[i]) return ACTH_EINVAL;
    if (modes[i] != 0 && (!ys[i] || !ys1[i])) return ACTH_EINVAL;
    if (modes[i] == 2 && !ps[i]) return ACTH_EINVAL;
  }
  if (d->M == 0) return ACTH_OK;
  const int nch = d->C / 8;
  // lanes per row: the smallest group that keeps a lane at <= 6 chunks per source
  const int lpr = nch <= 16 * 6 ? 16 : nch <= 32 * 6 ? 32 : 64;
  const long long rows_per_blk = 4LL * (64 / lpr);
  const unsigned nblk = (unsigned)((d->M + rows_per_blk - 1) / rows_per_blk);
  if (lpr == 16) {
    if (nch <= 16 * 2) hipLaunchKernelGGL((mamba_combine_kernel<16, 2>), dim3(nblk), dim3(256), 0, stream, *d);
    else hipLaunchKernelGGL((mamba_combine_kernel<16, 6>), dim3(nblk), dim3(256), 0, stream, *d);
  } else if (lpr == 32) {
    hipLaunchKernelGGL((mamba_combine_kernel<32, 6>), dim3(nblk), dim3(256), 0, stream, *d);
  } else {
    hipLaunchKernelGGL((mamba_combine_kernel<64, 6>), dim3(nblk), dim3(256), 0, stream, *d);
  }
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// Row softmax y = softmax(scale * x) of fp32 score rows into bf16 probabilities: the middle of the
// materialised single-head (head_dim 512) attention of the VAE mid blocks (diffusers Attention with
// upcast_softmax=True, AttnProcessor2_0), where S x S scores per frame fit HBM easily and the two
// contractions run on the MFMA GEMM. One block per row; fp32 max / sum; three passes over the row
// (max, sum of exponentials, write), the row (<= 36 KB at S = 9216) staying in L2 between passes.
__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = is_max ? fmaxf(r, sh[i]) : r + sh[i];
  return r;
}

__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* x, int ldx, bf16_t* y, int ldy, int cols,
                                                           float scale_log2) {
  __shared__ float sh[4];
  const float* xr = x + (long long)blockIdx.x * ldx;
  bf16_t* yr = y + (long long)blockIdx.x * ldy;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < cols; c += 256) m = fmaxf(m, xr[c]);
  m = block_reduce(m, sh, true) * scale_log2;
  float s = 0.0f;
  for (int c = threadIdx.x; c < cols; c += 256) s += __builtin_amdgcn_exp2f(fmaf(xr[c], scale_log2, -m));
  s = block_reduce(s, sh, false);
  const float inv = 1.0f / s;
  for (int c = threadIdx.x; c < cols; c += 256) yr[c] = f2bf(__builtin_amdgcn_exp2f(fmaf(xr[c], scale_log2, -m)) * inv);
}

extern "C" int acth_softmax_rows(const float* x, int ldx, void* y, int ldy, int rows, int cols, float scale,
                                 hipStream_t stream) {
  if (!x || !y || rows < 0 || cols <= 0 || ldx < cols || ldy < cols || !(scale > 0.0f)) return ACTH_EINVAL;
  if (rows == 0) return ACTH_OK;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)rows), dim3(256), 0, stream, x, ldx, (bf16_t*)y, ldy, cols,
                     scale * 1.4426950408889634f);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
