// Shared device helpers for the ACTalker denoising-path kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include "../../include/actalker_hip.h"

// Activation precision. The kernels are written once over a 16-bit activation type and built twice
// (Makefile): libactalker_hip.so with bf16 activations (ACTH_F16 = 0, the default path) and
// libactalker_hip_f16.so with fp16 activations (ACTH_F16 = 1: the reference's shipped weight_dtype,
// config/inference.yaml:66). Weights, activations and 16-bit MFMA operands share that type; accumulation,
// statistics and the sampler state stay fp32 in both builds. The names below keep "bf16" for the 16-bit
// activation type in either build (`bf16_t` is its raw bits in HBM).
#ifndef ACTH_F16
#define ACTH_F16 0
#endif
typedef uint16_t bf16_t;                                          // raw 16-bit activation bits in HBM
#if ACTH_F16
typedef _Float16 act16_t;
#else
typedef __bf16 act16_t;
#endif
typedef act16_t bf16x8_t __attribute__((ext_vector_type(8)));     // MFMA A/B fragment
typedef float f32x16_t __attribute__((ext_vector_type(16)));      // 32x32 MFMA accumulator
typedef float f32x4_t __attribute__((ext_vector_type(4)));        // 16x16 MFMA accumulator

// the 16-bit MFMAs over the activation type (fp16 runs at the bf16 rate on gfx950)
__device__ __forceinline__ f32x4_t mfma16x16x32(bf16x8_t a, bf16x8_t b, f32x4_t c) {
#if ACTH_F16
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}

__device__ __forceinline__ f32x16_t mfma32x32x16(bf16x8_t a, bf16x8_t b, f32x16_t c) {
#if ACTH_F16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}

// the two 16-bit values packed in a 32-bit word as floats (low half, high half)
__device__ __forceinline__ float lo16f(uint32_t w) {
#if ACTH_F16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu));
#else
  return __uint_as_float(w << 16);
#endif
}

__device__ __forceinline__ float hi16f(uint32_t w) {
#if ACTH_F16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
#else
  return __uint_as_float(w & 0xffff0000u);
#endif
}

#define ACTH_CHECK_LAUNCH()                                  \
  do {                                                       \
    if (hipGetLastError() != hipSuccess) return ACTH_ELAUNCH; \
  } while (0)

__device__ __forceinline__ float bf2f(bf16_t v) {
#if ACTH_F16
  return (float)__builtin_bit_cast(_Float16, v);
#else
  return __uint_as_float(((uint32_t)v) << 16);
#endif
}

__device__ __forceinline__ bf16_t f2bf(float f) {
#if ACTH_F16
  return __builtin_bit_cast(uint16_t, (_Float16)f);             // RNE
#else
  // lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __bfloat16_as_ushort(__float2bfloat16(f));
#endif
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }

// erf(x) by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 for all x): one v_rcp + one v_exp and
// seven FMAs, about half the VALU issue of ocml's erff; far below bf16 output resolution.
__device__ __forceinline__ float erf_as(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(fmaf(-p, e, 1.0f), x);
}

__device__ __forceinline__ float gelu_erf(float x) {
  // exact (erf) GELU, as torch.nn.functional.gelu(approximate="none")
  return 0.5f * x * (1.0f + erf_as(x * 0.70710678118654752f));
}

// Two GELUs in packed f32x2 arithmetic, no transcendental: erf(z) = z * P(z^2) on z clamped to
// [-3.3, 3.3] (erf(3.3) = 1 - 3.1e-6), P a degree-11 Chebyshev fit in z^2 evaluated by Horner with
// v_pk_fma_f32. |erf error| <= 4.3e-5 in fp32 (|GELU error| <= 1.0e-4 at |x| ~ 4, i.e. < 1 % of a
// bf16 ulp there), against two quarter-rate transcendentals + 7 scalar FMAs per value in gelu_erf:
// the GEGLU epilogue of the K = 320 / 640 GEMMs is VALU-bound on this math.
typedef float float2_pk __attribute__((ext_vector_type(2)));

// The same GELU from the degree-8 erf fit of ffn.hip (erf(g / sqrt 2) = gc * Q(gc^2), gc = g clamped to
// +-2.95 sqrt 2, |GELU error| <= 7.4e-5): 12 packed ops per pair instead of 16.
__device__ __forceinline__ float2_pk gelu_pk8(float2_pk x) {
  constexpr float c[9] = {0.7977727652f, -0.1326450109f, 0.01961599849f, -0.002216302557f, 1.874310692e-04f,
                          -1.138649350e-05f, 4.631291688e-07f, -1.116308557e-08f, 1.195545885e-10f};
  float2_pk gc;
  gc.x = __builtin_amdgcn_fmed3f(x.x, -4.171930f, 4.171930f);
  gc.y = __builtin_amdgcn_fmed3f(x.y, -4.171930f, 4.171930f);
  const float2_pk v = gc * gc;
  float2_pk r = {c[8], c[8]};
#pragma unroll
  for (int k = 7; k >= 0; --k) r = __builtin_elementwise_fma(r, v, (float2_pk){c[k], c[k]});
  const float2_pk hx = x * (float2_pk){0.5f, 0.5f};
  return __builtin_elementwise_fma(hx, gc * r, hx);
}

__device__ __forceinline__ float2_pk gelu_pk(float2_pk x) {
  constexpr float c[12] = {1.128378868e+00f, -3.761171401e-01f, 1.127940044e-01f, -2.678386122e-02f,
                           5.143333692e-03f, -8.073762292e-04f, 1.023587902e-04f, -1.013244946e-05f,
                           7.433642963e-07f, -3.751234701e-08f, 1.150420870e-09f, -1.604821484e-11f};
  float2_pk z = x * (float2_pk){0.70710678118654752f, 0.70710678118654752f};
  z.x = __builtin_amdgcn_fmed3f(z.x, -3.3f, 3.3f);
  z.y = __builtin_amdgcn_fmed3f(z.y, -3.3f, 3.3f);
  const float2_pk u = z * z;
  float2_pk r = {c[11], c[11]};
#pragma unroll
  for (int k = 10; k >= 0; --k) r = __builtin_elementwise_fma(r, u, (float2_pk){c[k], c[k]});
  const float2_pk hx = x * (float2_pk){0.5f, 0.5f};
  return __builtin_elementwise_fma(hx, z * r, hx);
}

#ifndef GEGLU_GELU
#define GEGLU_GELU gelu_pk8
#endif

__device__ __forceinline__ float softplus_f(float x) {
  // torch.nn.functional.softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(__expf(x));
}

// unpack 8 16-bit activations held in a uint4 into floats
__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  f[0] = lo16f(v.x); f[1] = hi16f(v.x);
  f[2] = lo16f(v.y); f[3] = hi16f(v.y);
  f[4] = lo16f(v.z); f[5] = hi16f(v.z);
  f[6] = lo16f(v.w); f[7] = hi16f(v.w);
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef act16_t bf16x2_t __attribute__((ext_vector_type(2)));

// two floats -> packed 16-bit pair (low = a) in ONE v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32 (RNE); two scalar
// f2bf conversions + shift + or cost three extra VALU per pair in every epilogue
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// packed pair of ones, and dot2 accumulation over packed 16-bit pairs (v_dot2_f32_bf16 / v_dot2c_f32_f16)
__device__ __forceinline__ bf16x2_t one2_16() { return (bf16x2_t){(act16_t)1.0f, (act16_t)1.0f}; }

__device__ __forceinline__ float dot2acc(bf16x2_t a, bf16x2_t b, float c) {
#if ACTH_F16
  return __builtin_amdgcn_fdot2(a, b, c, false);
#else
  return __builtin_amdgcn_fdot2_f32_bf16(a, b, c, false);
#endif
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
