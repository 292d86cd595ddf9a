// Small memory-bound kernels around the UNet and the sampler loop.
//
//  * acth_timestep_embedding : diffusers/TransformerSTmodel get_timestep_embedding
//                              (TransformerSTmodel.py:43-96), bf16 output
//  * acth_nchw_to_tokens / acth_tokens_to_nchw : (B, C, H, W) <-> (B*H*W, C) layout change
//  * acth_im2col(3x3)        : explicit im2col for convs with Cin % 64 != 0 (conv_in: Cin = 8, 7x7 stems)
//  * acth_maxpool2d          : nn.MaxPool2d on NHWC rows (VASA ResNet stems)
//  * acth_gather_rows        : Mamba token selection xz[:, idx] (mamba_layer.py:1963)
//  * acth_frame_mean         : spatial2time context pooling, mean over frames
//                              (TransformerSTmodel.py:4037-4052)
//  * acth_window_input       : pipeline window slice + 4-way CFG concat + scale_model_input +
//                              image-latent channel concat (pipeline:686-719)
//  * acth_cfg_euler_accum    : 4-way guidance + v-prediction Euler step + window accumulate
//                              (pipeline:731-751, EulerDiscreteScheduler.step)
//  * acth_div_counter        : latents_all = pred_latents / counter (pipeline:755-756)
//  * acth_gather_blocks      : batch-element row blocks copied out by index (the UNet's CFG-prefix expand)
#include "common.h"

__global__ void temb_kernel(const float* t, int n, int dim, int flip, float shift, float scale,
                            float max_period, bf16_t* out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * dim) return;
  const int i = idx / dim, j = idx - i * dim;
  const int half = dim / 2;
  float v = 0.0f;
  if (j < 2 * half) {
    // position j in [sin | cos] order, optionally flipped to [cos | sin]
    int jj = j;
    if (flip) jj = (j < half) ? j + half : j - half;
    const int f = jj < half ? jj : jj - half;
    const float expo = -logf(max_period) * (float)f / ((float)half - shift);
    const float arg = scale * t[i] * expf(expo);
    v = jj < half ? sinf(arg) : cosf(arg);
  }
  out[idx] = f2bf(v);
}

extern "C" int acth_timestep_embedding(const float* t, int n, int dim, int flip_sin_to_cos,
                                       float downscale_freq_shift, float scale, float max_period,
                                       void* out, hipStream_t stream) {
  if (!t || !out || n <= 0 || dim <= 1) return ACTH_EINVAL;
  const int tot = n * dim;
  hipLaunchKernelGGL(temb_kernel, dim3((tot + 255) / 256), dim3(256), 0, stream, t, n, dim,
                     flip_sin_to_cos, downscale_freq_shift, scale, max_period, (bf16_t*)out);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// in_dtype/out_dtype: 0 = bf16, 1 = fp32
__device__ __forceinline__ float ld_any(const void* p, size_t i, int dt) {
  return dt ? ((const float*)p)[i] : bf2f(((const bf16_t*)p)[i]);
}
__device__ __forceinline__ void st_any(void* p, size_t i, int dt, float v) {
  if (dt) ((float*)p)[i] = v; else ((bf16_t*)p)[i] = f2bf(v);
}

__global__ void nchw_to_tokens_kernel(const void* x, int in_dt, void* y, int out_dt, int ldy,
                                      int B, int C, int HW) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)B * C * HW) return;
  // idx enumerates the output (b, s, c) so stores are coalesced
  const int c = (int)(idx % C);
  const long long bs = idx / C;
  const int s = (int)(bs % HW);
  const long long b = bs / HW;
  st_any(y, (size_t)bs * ldy + c, out_dt, ld_any(x, ((size_t)b * C + c) * HW + s, in_dt));
}

extern "C" int acth_nchw_to_tokens(const void* x, int in_dt, void* y, int out_dt, int ldy, int B, int C,
                                   int HW, hipStream_t stream) {
  if (!x || !y || B <= 0 || C <= 0 || HW <= 0 || ldy < C) return ACTH_EINVAL;
  const long long n = (long long)B * C * HW;
  hipLaunchKernelGGL(nchw_to_tokens_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x,
                     in_dt, y, out_dt, ldy, B, C, HW);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

__global__ void tokens_to_nchw_kernel(const void* x, int in_dt, int ldx, void* y, int out_dt, int B, int C,
                                      int HW) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)B * C * HW) return;
  const int s = (int)(idx % HW);
  const long long bc = idx / HW;
  const int c = (int)(bc % C);
  const long long b = bc / C;
  st_any(y, idx, out_dt, ld_any(x, ((size_t)b * HW + s) * ldx + c, in_dt));
}

extern "C" int acth_tokens_to_nchw(const void* x, int in_dt, int ldx, void* y, int out_dt, int B, int C,
                                   int HW, hipStream_t stream) {
  if (!x || !y || B <= 0 || C <= 0 || HW <= 0 || ldx < C) return ACTH_EINVAL;
  const long long n = (long long)B * C * HW;
  hipLaunchKernelGGL(tokens_to_nchw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x,
                     in_dt, ldx, y, out_dt, B, C, HW);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// im2col for a kh x kw / stride / pad conv on NHWC bf16 rows (ld ldx): out[m, (ky*kw+kx)*C + c],
// m = (b*Ho + yo)*Wo + xo, ld = Kpad (columns >= kh*kw*C are zero-filled). Used where Cin is too
// narrow for the implicit-GEMM loader (UNet conv_in: Cin = 8; VASA ResNet stems: 7x7 / stride 2, Cin = 3).
__global__ void im2col_kernel(const bf16_t* x, int ldx, int B, int H, int W, int C, int kh, int kw, int stride,
                              int pad, int Ho, int Wo, bf16_t* out, int Kpad) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long M = (long long)B * Ho * Wo;
  if (idx >= M * Kpad) return;
  const long long m = idx / Kpad;
  const int k = (int)(idx - m * Kpad);
  bf16_t v = 0;
  if (k < kh * kw * C) {
    const int tap = k / C, c = k - tap * C;
    const int ky = tap / kw, kx = tap - ky * kw;
    const long long b = m / ((long long)Ho * Wo);
    const int rem = (int)(m - b * Ho * Wo);
    const int y = (rem / Wo) * stride + ky - pad, xx = (rem % Wo) * stride + kx - pad;
    if (y >= 0 && y < H && xx >= 0 && xx < W) v = x[((b * H + y) * W + xx) * ldx + c];
  }
  out[idx] = v;
}

extern "C" int acth_im2col(const void* x, int ldx, int B, int H, int W, int C, int kh, int kw, int stride, int pad,
                           int Ho, int Wo, void* out, int Kpad, hipStream_t stream) {
  if (!x || !out || B <= 0 || C <= 0 || ldx < C || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0) return ACTH_EINVAL;
  if (Kpad < kh * kw * C || Ho != (H + 2 * pad - kh) / stride + 1 || Wo != (W + 2 * pad - kw) / stride + 1)
    return ACTH_EINVAL;
  const long long n = (long long)B * Ho * Wo * Kpad;
  hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const bf16_t*)x, ldx, B, H, W, C, kh, kw, stride, pad, Ho, Wo, (bf16_t*)out, Kpad);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

extern "C" int acth_im2col3x3(const void* x, int B, int H, int W, int C, void* out, int Kpad,
                              hipStream_t stream) {
  return acth_im2col(x, C, B, H, W, C, 3, 3, 1, 1, H, W, out, Kpad, stream);
}

// ------------------------------------------------------------------------------------------
// nn.MaxPool2d(k, stride, pad) on NHWC bf16 rows (padding never wins: PyTorch pads with -inf);
// one thread per (output pixel, 8-channel chunk), 16-byte loads / stores.
__global__ void maxpool_kernel(const bf16_t* x, int ldx, int B, int H, int W, int C, int k, int stride, int pad,
                               int Ho, int Wo, bf16_t* y, int ldy) {
  const int nch = C >> 3;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)B * Ho * Wo * nch) return;
  const int ch = (int)(t % nch);
  const long long m = t / nch;
  const long long b = m / ((long long)Ho * Wo);
  const int rem = (int)(m - b * Ho * Wo);
  const int yo = rem / Wo, xo = rem - yo * Wo;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = -INFINITY;
  for (int ky = 0; ky < k; ++ky) {
    const int yi = yo * stride + ky - pad;
    if (yi < 0 || yi >= H) continue;
    for (int kx = 0; kx < k; ++kx) {
      const int xi = xo * stride + kx - pad;
      if (xi < 0 || xi >= W) continue;
      float w[8];
      unpack8(*reinterpret_cast<const uint4*>(x + ((b * H + yi) * W + xi) * ldx + ch * 8), w);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], w[e]);
    }
  }
  *reinterpret_cast<uint4*>(y + m * ldy + ch * 8) = pack8(v);
}

extern "C" int acth_maxpool2d(const void* x, int ldx, int B, int H, int W, int C, int k, int stride, int pad,
                              int Ho, int Wo, void* y, int ldy, hipStream_t stream) {
  if (!x || !y || B <= 0 || C % 8 || ldx % 8 || ldy % 8 || k <= 0 || stride <= 0 || pad < 0 || 2 * pad > k)
    return ACTH_EINVAL;
  if (Ho != (H + 2 * pad - k) / stride + 1 || Wo != (W + 2 * pad - k) / stride + 1 || Ho <= 0 || Wo <= 0)
    return ACTH_EINVAL;
  const long long n = (long long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const bf16_t*)x, ldx, B, H, W, C, k, stride, pad, Ho, Wo, (bf16_t*)y, ldy);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// dst[b*Ld + j] = src[b*Ls + idx[j]] for j < n, rows of C bf16 (C % 8 == 0)
__global__ void gather_rows_kernel(const bf16_t* src, int lds, int Ls, const int* idx, int n, bf16_t* dst,
                                   int ldd, int Ld, int nb, int C) {
  const int nch = C >> 3;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)nb * n * nch) return;
  const int ch = (int)(t % nch);
  const long long bj = t / nch;
  const int j = (int)(bj % n);
  const long long b = bj / n;
  *reinterpret_cast<uint4*>(dst + ((size_t)b * Ld + j) * ldd + ch * 8) =
      *reinterpret_cast<const uint4*>(src + ((size_t)b * Ls + idx[j]) * lds + ch * 8);
}

extern "C" int acth_gather_rows(const void* src, int lds, int Ls, const int* idx, int n, void* dst, int ldd,
                                int Ld, int nb, int C, hipStream_t stream) {
  if (!src || !dst || !idx || C % 8 || lds % 8 || ldd % 8 || n < 0 || n > Ld) return ACTH_EINVAL;
  if (n == 0 || nb == 0) return ACTH_OK;
  const long long tot = (long long)nb * n * (C / 8);
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream,
                     (const bf16_t*)src, lds, Ls, idx, n, (bf16_t*)dst, ldd, Ld, nb, C);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// out[b*T + t, c] = mean_f x[(b*F + f)*T + t, c]   (bf16 in, bf16 out, fp32 sum)
__global__ void frame_mean_kernel(const bf16_t* x, int ldx, int B, int F, int T, int C, bf16_t* out,
                                  int ldo) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)B * T * C) return;
  const int c = (int)(idx % C);
  const long long bt = idx / C;
  const int t = (int)(bt % T);
  const long long b = bt / T;
  float s = 0.0f;
  for (int f = 0; f < F; ++f) s += bf2f(x[((b * F + f) * T + t) * ldx + c]);
  out[bt * ldo + c] = f2bf(s / F);
}

extern "C" int acth_frame_mean(const void* x, int ldx, int B, int F, int T, int C, void* out, int ldo,
                               hipStream_t stream) {
  if (!x || !out || B <= 0 || F <= 0 || T <= 0 || C <= 0) return ACTH_EINVAL;
  const long long n = (long long)B * T * C;
  hipLaunchKernelGGL(frame_mean_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const bf16_t*)x, ldx, B, F, T, C, (bf16_t*)out, ldo);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// UNet input for a batch of units (unit u = one CFG branch of one window):
//   out[(u*F + f)*S + s, 0:4] = latents[frame_idx[u*F + f]*S + s, 0:4] * in_scale
//   out[(u*F + f)*S + s, 4:8] = img_lat[(branch[u]*T + frame_idx[u*F + f])*S + s, 0:4]
// latents: fp32 token-major (T*S, 4); img_lat: fp32 (nbranch*T*S, 4); out bf16 (., 8)
__global__ void window_input_kernel(const float* lat, const int* frame_idx, const float* img,
                                    const int* branch, float in_scale, bf16_t* out, int U, int F, int S,
                                    int T) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)U * F * S) return;
  const int s = (int)(idx % S);
  const long long uf = idx / S;
  const int u = (int)(uf / F);
  const float4 a = *reinterpret_cast<const float4*>(lat + ((size_t)frame_idx[uf] * S + s) * 4);
  const float4 g =
      *reinterpret_cast<const float4*>(img + (((size_t)branch[u] * T + frame_idx[uf]) * S + s) * 4);
  float v[8] = {a.x * in_scale, a.y * in_scale, a.z * in_scale, a.w * in_scale, g.x, g.y, g.z, g.w};
  *reinterpret_cast<uint4*>(out + idx * 8) = pack8(v);
}

extern "C" int acth_window_input(const float* lat, const int* frame_idx, const float* img, const int* branch,
                                 float in_scale, void* out, int U, int F, int S, int T, hipStream_t stream) {
  if (!lat || !frame_idx || !img || !branch || !out || U <= 0 || F <= 0 || S <= 0 || T <= 0) return ACTH_EINVAL;
  const long long n = (long long)U * F * S;
  hipLaunchKernelGGL(window_input_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, lat,
                     frame_idx, img, branch, in_scale, (bf16_t*)out, U, F, S, T);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// Guidance + Euler (v-prediction, gamma = 0) + accumulation for one window.
//   eps   = u + g1 (dav - u) + g2 (dv - dav) + g3 (c - dv)         (branch units 0..3)
//   x0    = eps * (-sigma / sqrt(sigma^2+1)) + x / (sigma^2 + 1)
//   x'    = x + (x - x0) / sigma * (sigma_next - sigma)
//   acc[frame_idx[f]] += x' ; cnt[frame_idx[f]] += 1
// noise: fp32 token-major rows of the four branch units: unit_off[k] = first row of branch k.
__global__ void cfg_euler_kernel(const float* noise, const long long* unit_off, const float* lat,
                                 const int* frame_idx, float g1, float g2, float g3, float sigma,
                                 float sigma_next, float* acc, float* cnt, int F, int S) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)F * S * 4) return;
  const int ch = (int)(idx & 3);
  const long long fs = idx >> 2;
  const int f = (int)(fs / S), s = (int)(fs % S);
  const size_t off = ((size_t)f * S + s) * 4 + ch;
  const float u = noise[unit_off[0] * 4 + off];
  const float dav = noise[unit_off[1] * 4 + off];
  const float dv = noise[unit_off[2] * 4 + off];
  const float c = noise[unit_off[3] * 4 + off];
  const float eps = u + g1 * (dav - u) + g2 * (dv - dav) + g3 * (c - dv);
  const size_t li = ((size_t)frame_idx[f] * S + s) * 4 + ch;
  const float x = lat[li];
  const float s2 = sigma * sigma + 1.0f;
  const float x0 = eps * (-sigma / sqrtf(s2)) + x / s2;
  const float xn = x + (x - x0) / sigma * (sigma_next - sigma);
  acc[li] += xn;
  if (ch == 0 && s == 0) cnt[frame_idx[f]] += 1.0f;
}

extern "C" int acth_cfg_euler_accum(const float* noise, const long long* unit_off, const float* lat,
                                    const int* frame_idx, float g1, float g2, float g3, float sigma,
                                    float sigma_next, float* acc, float* cnt, int F, int S,
                                    hipStream_t stream) {
  if (!noise || !unit_off || !lat || !frame_idx || !acc || !cnt || F <= 0 || S <= 0 || sigma == 0.0f)
    return ACTH_EINVAL;
  const long long n = (long long)F * S * 4;
  hipLaunchKernelGGL(cfg_euler_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, noise,
                     unit_off, lat, frame_idx, g1, g2, g3, sigma, sigma_next, acc, cnt, F, S);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

__global__ void div_counter_kernel(const float* acc, const float* cnt, float* out, int T, int S) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)T * S * 4) return;
  const int t = (int)(idx / ((long long)S * 4));
  out[idx] = acc[idx] / cnt[t];
}

extern "C" int acth_div_counter(const float* acc, const float* cnt, float* out, int T, int S,
                                hipStream_t stream) {
  if (!acc || !cnt || !out || T <= 0 || S <= 0) return ACTH_EINVAL;
  const long long n = (long long)T * S * 4;
  hipLaunchKernelGGL(div_counter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, acc, cnt,
                     out, T, S);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// dst block i = src block idx[i] (blocks of n16 16-byte vectors): the UNet's CFG-prefix sharing copies the
// distinct batch elements' rows out to the full batch (one launch per copy, 16-byte loads and stores; each
// thread issues its four loads before its four stores)
__global__ void gather_blocks_kernel(const uint4* __restrict__ src, const int* __restrict__ idx,
                                     uint4* __restrict__ dst, long long n16) {
  const int b = blockIdx.y;
  const uint4* s = src + (long long)idx[b] * n16;
  uint4* d = dst + (long long)b * n16;
  const long long i0 = (long long)blockIdx.x * 1024 + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i0 + 256 * k < n16) v[k] = s[i0 + 256 * k];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i0 + 256 * k < n16) d[i0 + 256 * k] = v[k];
}

extern "C" int acth_gather_blocks(const void* src, int n_src, const int* idx, int n, long long block_bytes,
                                  void* dst, hipStream_t stream) {
  if (n < 0 || n > 65535 || n_src <= 0 || block_bytes < 0 || block_bytes % 16) return ACTH_EINVAL;
  if (n == 0 || block_bytes == 0) return ACTH_OK;   // no work: the (possibly empty) buffers are not touched
  if (!src || !idx || !dst || ((uintptr_t)src | (uintptr_t)dst) % 16) return ACTH_EINVAL;
  const long long n16 = block_bytes / 16;
  const long long gx = (n16 + 1023) / 1024;
  if (gx > 0x7fffffffLL) return ACTH_EINVAL;
  hipLaunchKernelGGL(gather_blocks_kernel, dim3((unsigned)gx, (unsigned)n), dim3(256), 0, stream,
                     (const uint4*)src, idx, (uint4*)dst, n16);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

extern "C" int acth_version(void) { return 1; }

// the activation dtype this library was compiled for (common.h ACTH_F16): 0 bf16, 1 fp16
extern "C" int acth_act_dtype(void) { return ACTH_F16 ? 1 : 0; }
