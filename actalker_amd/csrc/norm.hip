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

__global__ __launch_bounds__(256) void layernorm_kernel(const ActhLayerNormDesc p) {
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

extern "C" int acth_layernorm(const ActhLayerNormDesc* d, hipStream_t stream) {
  if (!d || !d->x || !d->y || d->C <= 0 || d->C % 8 || d->C > 64 * 8 * MAXCH) return ACTH_EINVAL;
  if (d->ldx % 8 || d->ldy % 8 || (d->add && (d->ldadd % 8 || d->add_div <= 0)) || (d->sum_out && d->ldsum % 8))
    return ACTH_EINVAL;
  if (d->M == 0) return ACTH_OK;
  const long long nblk = ((long long)d->M + 3) / 4;
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)nblk), dim3(256), 0, stream, *d);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// GroupNorm. Rows are tokens; statistics batch = row / rows_per_stat; group = c / (C/G).
// Input may be the channel concat of x (C1 channels) and x2 (C - C1 channels).

#define GN_ROWS 256

__device__ __forceinline__ uint4 gn_load(const ActhGroupNormDesc& p, long long row, int ch) {
  const int c = ch * 8;
  if (c < p.C1) return *reinterpret_cast<const uint4*>((const bf16_t*)p.x + row * p.ldx + c);
  return *reinterpret_cast<const uint4*>((const bf16_t*)p.x2 + row * p.ldx2 + (c - p.C1));
}

// grid: (ceil(rows_per_stat / GN_ROWS), nstat)
__global__ __launch_bounds__(256) void gn_stats_kernel(const ActhGroupNormDesc p) {
  const int nch = p.C >> 3;
  const int stat = blockIdx.y;
  const long long r_begin = (long long)stat * p.rows_per_stat + (long long)blockIdx.x * GN_ROWS;
  const long long r_end = min((long long)stat * p.rows_per_stat + p.rows_per_stat,
                              r_begin + GN_ROWS);
  // thread -> (chunk, row lane); when nch > 256 a thread owns chunks t, t+256, ...
  int lanes_per_row, rows_par;
  if (nch <= 256) { rows_par = 256 / nch; lanes_per_row = nch; }
  else { rows_par = 1; lanes_per_row = 256; }
  const int t = threadIdx.x;
  if (t >= rows_par * lanes_per_row) return;
  const int rl = t / lanes_per_row, cl = t - rl * lanes_per_row;
  for (int ch = cl; ch < nch; ch += lanes_per_row) {
    float s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] = 0.0f; s2[e] = 0.0f; }
    for (long long r = r_begin + rl; r < r_end; r += rows_par) {
      float v[8];
      unpack8(gn_load(p, r, ch), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] += v[e]; s2[e] += v[e] * v[e]; }
    }
    double* acc = p.ws + ((size_t)stat * p.C + ch * 8) * 2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      atomicAdd(acc + 2 * e, (double)s1[e]);
      atomicAdd(acc + 2 * e + 1, (double)s2[e]);
    }
  }
}

// one thread per (stat, group): mean / rstd as floats after the per-channel double sums
__global__ void gn_finalize_kernel(const ActhGroupNormDesc p, int nstat) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nstat * p.G) return;
  const int stat = idx / p.G, g = idx - stat * p.G;
  const int cpg = p.C / p.G;
  double s1 = 0.0, s2 = 0.0;
  for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
    s1 += p.ws[((size_t)stat * p.C + c) * 2];
    s2 += p.ws[((size_t)stat * p.C + c) * 2 + 1];
  }
  const double n = (double)cpg * p.rows_per_stat;
  const double mean = s1 / n;
  double var = s2 / n - mean * mean;
  if (var < 0.0) var = 0.0;
  float* st = reinterpret_cast<float*>(p.ws + (size_t)nstat * p.C * 2);
  st[idx * 2] = (float)mean;
  st[idx * 2 + 1] = (float)(1.0 / sqrt(var + (double)p.eps));
}

__global__ __launch_bounds__(256) void gn_apply_kernel(const ActhGroupNormDesc p, int nstat) {
  const int nch = p.C >> 3;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)p.M * nch) return;
  const long long row = idx / nch;
  const int ch = (int)(idx - row * nch);
  const int stat = (int)(row / p.rows_per_stat);
  const int cpg = p.C / p.G;
  const float* st = reinterpret_cast<const float*>(p.ws + (size_t)nstat * p.C * 2);
  float v[8];
  unpack8(gn_load(p, row, ch), v);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = ch * 8 + e;
    const int g = c / cpg;
    const float mean = st[(stat * p.G + g) * 2], rstd = st[(stat * p.G + g) * 2 + 1];
    float o = (v[e] - mean) * rstd * p.gamma[c] + p.beta[c];
    if (p.silu) o = silu_f(o);
    v[e] = o;
  }
  *reinterpret_cast<uint4*>((bf16_t*)p.y + row * p.ldy + ch * 8) = pack8(v);
}

extern "C" size_t acth_groupnorm_workspace_size(int M, int C, int G, int rows_per_stat) {
  if (rows_per_stat <= 0) return 0;
  const size_t nstat = (size_t)M / rows_per_stat;
  return nstat * C * 2 * sizeof(double) + nstat * G * 2 * sizeof(float);
}

extern "C" int acth_groupnorm(const ActhGroupNormDesc* d, hipStream_t stream) {
  if (!d || !d->x || !d->y || !d->ws || !d->gamma || !d->beta) return ACTH_EINVAL;
  if (d->C % 8 || d->C1 % 8 || d->G <= 0 || d->C % d->G || d->rows_per_stat <= 0) return ACTH_EINVAL;
  if (d->M % d->rows_per_stat) return ACTH_EINVAL;
  if (d->C1 < d->C && (!d->x2 || d->ldx2 % 8)) return ACTH_EINVAL;
  if (d->ldx % 8 || d->ldy % 8 || d->C > 8 * 512) return ACTH_EINVAL;
  const int nstat = d->M / d->rows_per_stat;
  if (nstat == 0) return ACTH_OK;
  if (nstat > 65535) return ACTH_EINVAL;
  if (hipMemsetAsync(d->ws, 0, (size_t)nstat * d->C * 2 * sizeof(double), stream) != hipSuccess)
    return ACTH_ELAUNCH;
  dim3 g1((d->rows_per_stat + GN_ROWS - 1) / GN_ROWS, nstat);
  hipLaunchKernelGGL(gn_stats_kernel, g1, dim3(256), 0, stream, *d);
  ACTH_CHECK_LAUNCH();
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((nstat * d->G + 127) / 128), dim3(128), 0, stream, *d, nstat);
  ACTH_CHECK_LAUNCH();
  const long long n = (long long)d->M * (d->C / 8);
  hipLaunchKernelGGL(gn_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, *d, nstat);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// Mamba combine + LayerNorm. Per branch: mode 0 = nothing selected (row of x), 1 = every
// token selected in order (scan row b*L + s), 2 = position map pos[s] (-1 = unselected).

__device__ __forceinline__ void mc_branch(const void* x, int ldx, const void* y0, const void* y1, int ldyy,
                                          int L, const int* pos, int mode, long long row, int S, int ch,
                                          float* v) {
  const long long b = row / S;
  const int s = (int)(row - b * S);
  int j = -1;
  if (mode == 1) j = s;
  else if (mode == 2) j = pos[s];
  if (j < 0) {
    unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)x + row * ldx + ch * 8), v);
  } else {
    const long long r = b * L + j;
    float a[8], c[8];
    unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)y0 + r * ldyy + ch * 8), a);
    unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)y1 + r * ldyy + ch * 8), c);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = a[e] + c[e];
  }
}

__global__ __launch_bounds__(256) void mamba_combine_kernel(const ActhMambaCombineDesc p) {
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
      float a[8], e2[8];
      mc_branch(p.xa, p.ldxa, p.ya0, p.ya1, p.ldya, p.La, p.pos_a, p.mode_a, row, p.S, ch, a);
      mc_branch(p.xe, p.ldxe, p.ye0, p.ye1, p.ldye, p.Le, p.pos_e, p.mode_e, row, p.S, ch, e2);
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[i][e] = a[e] + e2[e]; s += v[i][e]; }
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
        o[e] = (v[i][e] - mean) * rstd * p.gamma[c] + p.beta[c];
      }
      *reinterpret_cast<uint4*>((bf16_t*)p.y + row * p.ldy + ch * 8) = pack8(o);
    }
  }
}

extern "C" int acth_mamba_combine_ln(const ActhMambaCombineDesc* d, hipStream_t stream) {
  if (!d || !d->y || !d->gamma || !d->beta) return ACTH_EINVAL;
  if (d->C % 8 || d->C > 64 * 8 * MAXCH || d->S <= 0 || d->M % d->S) return ACTH_EINVAL;
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
  const long long nblk = ((long long)d->M + 3) / 4;
  hipLaunchKernelGGL(mamba_combine_kernel, dim3((unsigned)nblk), dim3(256), 0, stream, *d);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
