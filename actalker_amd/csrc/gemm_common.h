// Shared pieces of the bf16 MFMA GEMM kernels (gemm.hip: 128x128 tile, gemm256.hip: 256-row tiles):
// the implicit-conv A-operand addressing used by the LDS-DMA loaders and the fused epilogue.
#pragma once
#include "common.h"

typedef __attribute__((address_space(3))) void lds_void;

namespace gemm {

struct RowInfo { int b, y, x; bool ok; };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

constexpr unsigned OOB = 0x80000000u;     // any offset >= num_records reads as zero

// Decompose output row m into (image, y, x) for the conv loader or the frame index for the
// temporal loader.
__device__ __forceinline__ RowInfo row_info(const ActhGemmDesc& p, int m) {
  RowInfo ri;
  ri.ok = m < p.M;
  ri.b = 0; ri.y = 0; ri.x = 0;
  if (p.amode == 1) {
    const int hw = p.Ho * p.Wo;
    ri.b = m / hw;
    const int rem = m - ri.b * hw;
    ri.y = rem / p.Wo;
    ri.x = rem - ri.y * p.Wo;
  } else if (p.amode == 2) {
    ri.y = (m / p.S) % p.F;
  }
  return ri;
}

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

// does K tile starting at k0 read from A2 (the skip-connection half of a channel concat)?
__device__ __forceinline__ bool second_source(const ActhGemmDesc& p, int k0) {
  return p.A2 && ((p.amode == 0 ? k0 : k0 % p.Cin) >= p.K1);
}

// v[e] += src[e] for e < 8 (or e < n when !vec): two float4 loads when 16-byte aligned
__device__ __forceinline__ void add8(float* v, const float* src, bool vec, int n) {
  if (vec) {
    const float4 a = reinterpret_cast<const float4*>(src)[0];
    const float4 b = reinterpret_cast<const float4*>(src)[1];
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += e < n ? src[e] : 0.0f;
  }
}

// n / d for 0 <= n < 2^22 and d >= 1: float reciprocal estimate (within 2 of the quotient for a
// reciprocal good to 2 ulp), corrected by two remainder checks; ~12 VALU instead of a
// ~40-instruction integer division sequence per output chunk
__device__ __forceinline__ int udiv22(int n, int d) {
  int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
  int r = n - q * d;
  q += (r >= d) - (r < 0);
  r = n - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

__device__ __forceinline__ size_t out_row(const ActhGemmDesc& p, int row) {
  if (p.orow_div >= p.M) return (size_t)row + p.orow_off;      // no row remap (uniform)
  const int q = udiv22(row, p.orow_div);
  return (size_t)q * p.orow_stride + (row - q * p.orow_div) + p.orow_off;
}

__device__ __forceinline__ void store8(const ActhGemmDesc& p, size_t prow, int ocol, const float* v, bool full,
                                       int vec_ok) {
  if (full && vec_ok) {
    if (p.out_f32) {
      float* cp = (float*)p.C + prow * p.ldc + ocol;
      *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      *reinterpret_cast<uint4*>((bf16_t*)p.C + prow * p.ldc + ocol) = pack8(v);
    }
    return;
  }
  for (int e = 0; e < 8 && ocol + e < p.N; ++e) {
    if (p.out_f32) ((float*)p.C)[prow * p.ldc + ocol + e] = v[e];
    else ((bf16_t*)p.C)[prow * p.ldc + ocol + e] = f2bf(v[e]);
  }
}

// Operands of the non-GEGLU epilogue that come from HBM (residual row, AlphaBlender mix row),
// loaded ahead of the stores that precede their use (gemm8p.hip).
struct EpiPre { uint4 r, mix; };

__device__ __forceinline__ size_t residual_row(const ActhGemmDesc& p, int row) {
  if (!p.rmap) return (size_t)row;
  const int q = udiv22(row, p.r_div);
  return (size_t)p.rmap[q - udiv22(q, p.r_mod) * p.r_mod] * p.r_div + (row - q * p.r_div);
}

// 16-byte residual / mix chunks of (row, [ocol, ocol+8)) for the vector path. The loads are
// unconditional per lane (an invalid or partial chunk reads row 0 / column 0 instead and is never
// used), so the prefetched registers do not live across divergent branches.
__device__ __forceinline__ uint4 epi_load_r(const ActhGemmDesc& p, int row, int ocol, bool ok) {
  const bool use = ok && ocol + 8 <= p.N;
  const int rr = use ? row : 0, cc = use ? ocol : 0;
  return *reinterpret_cast<const uint4*>((const bf16_t*)p.R + residual_row(p, rr) * p.ldr + cc);
}

__device__ __forceinline__ uint4 epi_load_mix(const ActhGemmDesc& p, int row, int ocol, bool ok) {
  const bool use = ok && ocol + 8 <= p.N;
  const int rr = use ? row : 0, cc = use ? ocol : 0;
  return *reinterpret_cast<const uint4*>((const bf16_t*)p.MIX + (size_t)rr * p.ldmix + cc);
}

__device__ __forceinline__ void epi_prefetch(const ActhGemmDesc& p, int row, int ocol, bool ok, EpiPre& e) {
  if (p.R) e.r = epi_load_r(p, row, ocol, ok);
  if (p.MIX) e.mix = epi_load_mix(p, row, ocol, ok);
}

// Epilogue after alpha / bias / row bias: residual, SiLU / GELU, AlphaBlender mix, store. The
// vector path takes the residual / mix chunks from e (epi_prefetch); the scalar path loads them.
__device__ __forceinline__ void epilogue8_tail(const ActhGemmDesc& p, int row, int ocol, float* v, int vec_ok,
                                               const EpiPre& e) {
  const bool full = ocol + 8 <= p.N;
  const bool vec = full && vec_ok;
  if (p.R) {
    float t[8];
    if (vec) {
      unpack8(e.r, t);
    } else {
      const bf16_t* rp = (const bf16_t*)p.R + residual_row(p, row) * p.ldr + ocol;
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = (ocol + k < p.N) ? bf2f(rp[k]) : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += t[k];
  }
  if (p.act == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = silu_f(v[k]);
  } else if (p.act == 3) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = gelu_erf(v[k]);
  } else if (p.act == 4) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.0f);
  }
  if (p.MIX) {
    float t[8];
    if (vec) {
      unpack8(e.mix, t);
    } else {
      const bf16_t* mp = (const bf16_t*)p.MIX + (size_t)row * p.ldmix + ocol;
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = (ocol + k < p.N) ? bf2f(mp[k]) : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p.mix_alpha * t[k] + (1.0f - p.mix_alpha) * v[k];
  }
  store8(p, out_row(p, row), ocol, v, full, vec_ok);
}

// Non-GEGLU epilogue of 8 consecutive output columns [ocol, ocol+8) of output row `row`;
// v holds the raw accumulators. Applies alpha, bias, row bias, residual (row-remapped),
// SiLU / GELU, AlphaBlender mix, and stores (16-byte vectors when aligned).
__device__ __forceinline__ void epilogue8(const ActhGemmDesc& p, int row, int ocol, float* v, int vec_ok) {
  const bool full = ocol + 8 <= p.N;
  const bool vec = full && vec_ok;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= p.alpha;
  if (p.bias) add8(v, p.bias + ocol, full && !((size_t)(p.bias + ocol) & 15), p.N - ocol);
  if (p.rowbias) {
    const float* rb2 = p.rowbias + (size_t)udiv22(row, p.rb_div) * p.ldrb + ocol;
    add8(v, rb2, full && !((size_t)rb2 & 15), p.N - ocol);
  }
  if (p.R) {
    size_t rrow = row;
    if (p.rmap) {
      const int q = udiv22(row, p.r_div);
      rrow = (size_t)p.rmap[q - udiv22(q, p.r_mod) * p.r_mod] * p.r_div + (row - q * p.r_div);
    }
    const bf16_t* rp = (const bf16_t*)p.R + rrow * p.ldr + ocol;
    float t[8];
    if (vec) {
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
  } else if (p.act == 4) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.0f);
  }
  if (p.MIX) {
    const bf16_t* mp = (const bf16_t*)p.MIX + (size_t)row * p.ldmix + ocol;
    float t[8];
    if (vec) {
      unpack8(*reinterpret_cast<const uint4*>(mp), t);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = (ocol + e < p.N) ? bf2f(mp[e]) : 0.0f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p.mix_alpha * t[e] + (1.0f - p.mix_alpha) * v[e];
  }
  store8(p, out_row(p, row), ocol, v, full, vec_ok);
}

// GEGLU epilogue: hidden h[8] at weight columns [hcol, hcol+8) and gate g[8] at [gcol, gcol+8)
// (16-column granules, modules.pack_geglu); writes h * gelu(g) at output column `ocol`.
__device__ __forceinline__ void epilogue_geglu8(const ActhGemmDesc& p, int row, int hcol, int gcol, int ocol,
                                                const float* h, const float* g, int vec_ok) {
  float v[8], hv[8], gv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { hv[e] = h[e] * p.alpha; gv[e] = g[e] * p.alpha; }
  if (p.bias) {
    add8(hv, p.bias + hcol, !((size_t)(p.bias + hcol) & 15), 8);
    add8(gv, p.bias + gcol, !((size_t)(p.bias + gcol) & 15), 8);
  }
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const float2_pk gg = GEGLU_GELU((float2_pk){gv[e], gv[e + 1]});
    v[e] = hv[e] * gg.x;
    v[e + 1] = hv[e + 1] * gg.y;
  }
  store8(p, out_row(p, row), ocol, v, true, vec_ok);
}


}  // namespace gemm
