// Direct (non-GEMM) 3-tap / 3x3 convolutions for the narrow-channel layers around the denoising
// loop, where an MFMA implicit GEMM would pad K or N to its 64-wide tiles many times over:
//   * PoseGuider (src/models/audio_adapter/pose_guider.py:28-73): InflatedConv3d 3->16->32->96->256
//     at full / half / quarter resolution (Cin = 3, 16, 32, 96);
//   * AutoencoderKLTemporalDecoder conv_out 128->3 and time_conv_out Conv3d(3, 3, (3,1,1))
//     (diffusers 0.29.2 TemporalDecoder, called from pipeline decode_latents :235-262).
// These layers are HBM-bound (<= 2.3 kFLOP per output element, a few hundred bytes per pixel),
// so the kernel is organised for coalesced NHWC reads, not for matrix cores: one output pixel
// per lane, CG output channels per block, the block's weight slice for 32 input channels staged
// in LDS and read as wave-uniform float4 broadcasts.
#include "common.h"

namespace {

constexpr int CCH = 32;   // input channels per LDS weight chunk

__device__ __forceinline__ long long in_row(const ActhConvDirectDesc& p, long long m, int tap, bool& ok) {
  if (p.mode == 0) {
    const int HWo = p.Ho * p.Wo;
    const long long b = m / HWo;
    const int r = (int)(m - b * HWo);
    const int yo = r / p.Wo, xo = r - (r / p.Wo) * p.Wo;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int lo = p.pad0 ? 0 : 1;          // pad0: F.pad(0, 1, 0, 1) + padding 0 (Downsample2D padding=0)
    const int yi = yo * p.stride - lo + ky, xi = xo * p.stride - lo + kx;
    ok = (yi >= 0) && (yi < p.H) && (xi >= 0) && (xi < p.W);
    return (b * p.H + yi) * p.W + xi;
  }
  const long long bf = m / p.S;
  const int f = (int)(bf % p.F);
  const int fi = f + tap - 1;
  ok = (fi >= 0) && (fi < p.F);
  return m + (long long)(tap - 1) * p.S;
}

template <int CG, bool VEC>
__global__ __launch_bounds__(256) void conv_direct_kernel(const ActhConvDirectDesc p, long long Mout) {
  __shared__ float wsm[9 * CCH * CG];
  const int taps = p.mode == 0 ? 9 : 3;
  const long long m = (long long)blockIdx.x * 256 + threadIdx.x;
  const bool live = m < Mout;
  const int co0 = blockIdx.y * CG;
  float acc[CG];
#pragma unroll
  for (int j = 0; j < CG; ++j) acc[j] = 0.0f;
  long long rows[9];
  bool oks[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    oks[t] = false;
    rows[t] = 0;
    if (t < taps && live) rows[t] = in_row(p, m, t, oks[t]);
  }
  const bf16_t* x = (const bf16_t*)p.x;
  for (int c0 = 0; c0 < p.Cin; c0 += CCH) {
    __syncthreads();
    for (int i = threadIdx.x; i < taps * CCH * CG; i += 256) {
      const int j = i % CG, c = (i / CG) % CCH, t = i / (CG * CCH);
      const int ci = c0 + c, co = co0 + j;
      wsm[i] = (ci < p.Cin && co < p.Cout) ? p.w[((long long)t * p.Cin + ci) * p.Cout + co] : 0.0f;
    }
    __syncthreads();
    const int nc = min(CCH, p.Cin - c0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t >= taps || !oks[t]) continue;
      const bf16_t* src = x + rows[t] * p.ldx + c0;
      float xv[CCH];
      if (VEC) {
#pragma unroll
        for (int q = 0; q < CCH / 8; ++q) {
          if (q * 8 < nc) {
            unpack8(reinterpret_cast<const uint4*>(src)[q], xv + q * 8);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[q * 8 + e] = 0.0f;
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < CCH; ++c) xv[c] = c < nc ? bf2f(src[c]) : 0.0f;
      }
      const float* wt = wsm + t * CCH * CG;
#pragma unroll
      for (int c = 0; c < CCH; ++c) {
#pragma unroll
        for (int j = 0; j < CG; j += 4) {
          const float4 w4 = *reinterpret_cast<const float4*>(wt + c * CG + j);
          acc[j] = fmaf(xv[c], w4.x, acc[j]);
          acc[j + 1] = fmaf(xv[c], w4.y, acc[j + 1]);
          acc[j + 2] = fmaf(xv[c], w4.z, acc[j + 2]);
          acc[j + 3] = fmaf(xv[c], w4.w, acc[j + 3]);
        }
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int j = 0; j < CG; ++j) {
    const int co = co0 + j;
    float v = acc[j] + ((p.bias && co < p.Cout) ? p.bias[co] : 0.0f);
    if (p.act == 1) v = silu_f(v);
    else if (p.act == 3) v = gelu_erf(v);
    acc[j] = v;
  }
  const bool full = co0 + CG <= p.Cout;
  if (p.out_f32) {
    float* y = (float*)p.y + m * p.ldy + co0;
#pragma unroll
    for (int j = 0; j < CG; ++j)
      if (full || co0 + j < p.Cout) y[j] = acc[j];
  } else {
    bf16_t* y = (bf16_t*)p.y + m * p.ldy + co0;
    if (VEC && full && CG % 8 == 0) {
#pragma unroll
      for (int j = 0; j < CG; j += 8) reinterpret_cast<uint4*>(y)[j / 8] = pack8(acc + j);
    } else {
#pragma unroll
      for (int j = 0; j < CG; ++j)
        if (full || co0 + j < p.Cout) y[j] = f2bf(acc[j]);
    }
  }
}

}  // namespace

extern "C" int acth_conv_direct(const ActhConvDirectDesc* d, hipStream_t stream) {
  if (d && d->B == 0) return ACTH_OK;   // empty batch: nothing read or written
  if (!d || !d->x || !d->w || !d->y) return ACTH_EINVAL;
  if (d->Cin <= 0 || d->Cout <= 0 || d->ldx < d->Cin || d->ldy < d->Cout) return ACTH_EINVAL;
  if (d->act != 0 && d->act != 1 && d->act != 3) return ACTH_EINVAL;
  long long Mout;
  if (d->mode == 0) {
    if (d->B <= 0 || d->H <= 0 || d->W <= 0 || (d->stride != 1 && d->stride != 2)) return ACTH_EINVAL;
    const int padsum = d->pad0 ? 1 : 2;
    if (d->H + padsum < 3 || d->W + padsum < 3) return ACTH_EINVAL;
    if (d->Ho != (d->H + padsum - 3) / d->stride + 1 || d->Wo != (d->W + padsum - 3) / d->stride + 1)
      return ACTH_EINVAL;
    Mout = (long long)d->B * d->Ho * d->Wo;
  } else if (d->mode == 1) {
    if (d->B <= 0 || d->F <= 0 || d->S <= 0) return ACTH_EINVAL;
    Mout = (long long)d->B * d->F * d->S;
  } else {
    return ACTH_EINVAL;
  }
  if (Mout == 0) return ACTH_OK;
  const bool vec = (d->Cin % 8 == 0) && (d->ldx % 8 == 0) && ((size_t)d->x % 16 == 0) &&
                   (d->out_f32 || ((d->ldy % 8 == 0) && ((size_t)d->y % 16 == 0)));
  const int cg = d->Cout <= 4 ? 4 : 16;
  dim3 grid((unsigned)((Mout + 255) / 256), (unsigned)((d->Cout + cg - 1) / cg));
  if (grid.x == 0 || (Mout + 255) / 256 > 0x7fffffffLL) return ACTH_EINVAL;
  if (cg == 4) {
    if (vec) hipLaunchKernelGGL((conv_direct_kernel<4, true>), grid, dim3(256), 0, stream, *d, Mout);
    else hipLaunchKernelGGL((conv_direct_kernel<4, false>), grid, dim3(256), 0, stream, *d, Mout);
  } else {
    if (vec) hipLaunchKernelGGL((conv_direct_kernel<16, true>), grid, dim3(256), 0, stream, *d, Mout);
    else hipLaunchKernelGGL((conv_direct_kernel<16, false>), grid, dim3(256), 0, stream, *d, Mout);
  }
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
