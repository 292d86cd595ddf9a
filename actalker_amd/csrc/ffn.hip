// Fused GEGLU feed-forward for the level-0 transformer blocks (C = 320): diffusers FeedForward(geglu)
// as used by BasicTransformerBlock.ff and TemporalBasicTransformerBlock.ff_in / .ff (attention.py:
// 223-343, 418-473):
//     y = W2 (h * gelu(g)) + b2 [+ residual] [AlphaBlender: a * mix + (1 - a) * (...)],
//     [h | g] = W1 x + b1,  W1: (2I, C), W2: (C, I), I = 4C.
// Two GEMMs and a 4C-wide hidden tensor per token become one kernel whose hidden activations never
// reach HBM -- the structure of flash attention (S = K Q^T -> P -> O += V^T P^T):
//   * a workgroup owns 128 tokens: 4 wave pairs x 32 tokens (two 16-token groups). A wave's 32
//     token rows of x live in VGPRs for the whole kernel as the up projection's B operand;
//   * the hidden dimension is walked in chunks of 32 gated units (64 rows of W1 = two 16-row
//     (hidden | gate) granules of modules.pack_geglu; 32 columns of W2), double-buffered in LDS by
//     LDS-DMA. Wave `half` of a pair computes granule `half` of the chunk for the pair's 32 tokens,
//     H^T = W1g x^T (v_mfma_f32_16x16x32_bf16; every W1 fragment read feeds two MFMAs), gates it in
//     registers (lane (t, q) holds units 4q..4q+3 of both the hidden and the gate fragment) and
//     swaps the 4 gated units per token with its partner through LDS; then it accumulates output
//     channels [160*half, +160) of O^T += W2c H^T for the 32 tokens. A lane's 4 + 4 units are the
//     down projection's B operand directly, W2's K order permuted to match at pack time (within each
//     32-column block, column 8q + j <- unit 4q + j (j < 4) or 16 + 4q + (j - 4)) and scaled by 0.5;
//   * software pipeline, one barrier per chunk: iteration c runs up(c), down(c-1), gate(c), so the
//     gate VALU has independent MFMAs to overlap; W1(c+1) and W2(c) are in flight meanwhile;
//   * epilogue: O^T fragments -> per-wave LDS slab (token-major) -> + b2, residual, mix -> 16-byte
//     row stores.
// Numerics match the two-kernel path: fp32 accumulation, the gated hidden rounded to bf16 before the
// down projection (as the GEGLU GEMM's bf16 output was); GELU by the degree-8 erf fit below.
// LDS images (conflict-free ds_read_b128 for the gfx950 lane groups): W1 chunk 64 rows x C/8 16-byte
// chunks, chunk index XOR (row & 7) inside 8-chunk groups; W2 chunk C rows x 4 chunks, chunk index
// XOR ((row >> 1) & 2).
#include <type_traits>

#include "common.h"

typedef __attribute__((address_space(3))) void lds_void;

namespace {

// erf(g / sqrt 2) = gc * Q(gc^2), gc = g clamped to +-2.95 sqrt 2 (erf(2.95) = 1 - 4e-5), Q a degree-8
// least-squares fit evaluated by 8 scalar FMAs: |GELU error| <= 7.4e-5 in fp32 over all g (below a
// tenth of a bf16 ulp of the output). Scalar on purpose: packed-f32 VALU beside MFMAs costs more
// issue cycles than the two scalar instructions it replaces.
__device__ __forceinline__ float erf_scaled(float g) {
  constexpr float c[9] = {0.7977727652f, -0.1326450109f, 0.01961599849f, -0.002216302557f, 1.874310692e-04f,
                          -1.138649350e-05f, 4.631291688e-07f, -1.116308557e-08f, 1.195545885e-10f};
  const float gc = __builtin_amdgcn_fmed3f(g, -4.171930f, 4.171930f);
  const float v = gc * gc;
  float r = c[8];
#pragma unroll
  for (int k = 7; k >= 0; --k) r = fmaf(r, v, c[k]);
  return gc * r;
}

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

}  // namespace

// In-kernel phase stamps (diagnostics only, off unless acth_debug_ffn_stamps enabled them): s_memtime
// per workgroup at entry, after the prologue, after chunks 0 / 10 / 30, after the loop, at the end.
#define FFN_STAMP_WGS 8192
#define FFN_NSTAMP 8
__device__ unsigned long long g_ffn_stamps[FFN_STAMP_WGS * FFN_NSTAMP];
__device__ int g_ffn_stamp_on;

template <int C>
__global__ __launch_bounds__(512, 1) void ffn_geglu_kernel(const ActhFfnDesc p, unsigned w1_bytes,
                                                           unsigned w2_bytes) {
  constexpr int I = 4 * C;                // hidden units
  constexpr int KS = C / 32;              // k steps of the up projection
  constexpr int HF = C / 32;              // output fragments (16 channels) per wave: half of C / 16
  constexpr int HC = 32;                  // gated units per chunk
  constexpr int NCH = I / HC;             // chunks
  constexpr int W1R = 2 * HC;             // W1 rows per chunk
  constexpr int W1CH = C / 8;             // 16-byte chunks per W1 row
  constexpr int W1B = W1R * C * 2;        // bytes of a W1 chunk image
  constexpr int W2B = C * HC * 2;         // bytes of a W2 chunk image (C rows x 64 B)
  constexpr int HXB = 8 * 2 * 64 * 8;     // gated-unit exchange: [pair 4][tg 2][half 2][lane 64] x 8 B
  constexpr int NI1 = W1B / 1024, NI2 = W2B / 1024;   // DMA wave-instructions per chunk
  constexpr int NI1W = (NI1 + 7) / 8, NI2W = (NI2 + 7) / 8;
  static_assert(C % 32 == 0 && HF % 2 == 0 && W1CH % 8 == 0 && W1B % 1024 == 0 && W2B % 1024 == 0, "shape");
  static_assert(2 * (W1B + W2B + HXB) + (2 * I + C) * 4 <= 160 * 1024, "LDS");
  // Every buffer is its own LDS object and the chunk loop is unrolled by two so each access names
  // its buffer at compile time: the compiler then knows an LDS-DMA write into one buffer never
  // aliases a read of another and inserts no vmcnt(0) in front of fragment reads.
  __shared__ __attribute__((aligned(16))) char w1s0[W1B], w1s1[W1B], w2s0[W2B], w2s1[W2B], hxs0[HXB], hxs1[HXB];
  __shared__ __attribute__((aligned(16))) float sb1[2 * I], sb2[C];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pr = wave >> 1, half = wave & 1;
  const bool stamps = g_ffn_stamp_on && blockIdx.x < FFN_STAMP_WGS;
  auto stamp = [&](int k) {
    if (stamps && tid == 0) g_ffn_stamps[blockIdx.x * FFN_NSTAMP + k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const int t16 = lane & 15, q = lane >> 4;
  const int tok0 = blockIdx.x * 128 + pr * 32;             // the pair's first token

  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.w1), (short)0, (int)w1_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r2 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.w2), (short)0, (int)w2_bytes, 0x00020000);

  // ---- DMA source offsets of this lane's 16-byte chunk of each image instruction
  unsigned o1[NI1W], o2[NI2W];
#pragma unroll
  for (int u = 0; u < NI1W; ++u) {
    const int pc = (wave + 8 * u) * 64 + lane;
    const int row = pc / W1CH, pch = pc - row * W1CH;
    const int lch = (pch & ~7) | ((pch ^ row) & 7);
    o1[u] = ((unsigned)row * p.ldw1 + lch * 8) * 2u;
  }
#pragma unroll
  for (int u = 0; u < NI2W; ++u) {
    const int pc = (wave + 8 * u) * 64 + lane;
    const int row = pc >> 2, pch = pc & 3;
    const int lch = pch ^ ((row >> 1) & 2);
    o2[u] = ((unsigned)row * p.ldw2 + lch * 8) * 2u;
  }
  auto stage_w1 = [&](int ch, auto par) {
    char* d = decltype(par)::value ? w1s1 : w1s0;
    const unsigned b = (unsigned)ch * W1R * p.ldw1 * 2u;
#pragma unroll
    for (int u = 0; u < NI1W; ++u)
      if (NI1 % 8 == 0 || wave + 8 * u < NI1)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, (lds_void*)(d + (wave + 8 * u) * 1024), 16, (int)(o1[u] + b), 0,
                                                 0, 0);
  };
  auto stage_w2 = [&](int ch, auto par) {
    char* d = decltype(par)::value ? w2s1 : w2s0;
    const unsigned b = (unsigned)ch * HC * 2u;
#pragma unroll
    for (int u = 0; u < NI2W; ++u)
      if (NI2 % 8 == 0 || wave + 8 * u < NI2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r2, (lds_void*)(d + (wave + 8 * u) * 1024), 16, (int)(o2[u] + b), 0,
                                                 0, 0);
  };

  // ---- the pair's 2 x 16 token rows of x, as the up projection's B operand for every k step
  bf16x8_t xf[2][KS];
#pragma unroll
  for (int tg = 0; tg < 2; ++tg) {
    const int tok = tok0 + tg * 16 + t16;
    const bf16_t* xr = (const bf16_t*)p.x + (size_t)(tok < p.M ? tok : 0) * p.ldx + 8 * q;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 v = *reinterpret_cast<const uint4*>(xr + 32 * ks);
      if (tok >= p.M) v = make_uint4(0, 0, 0, 0);
      xf[tg][ks] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  for (int i = tid; i < 2 * I; i += 512) sb1[i] = p.b1 ? p.b1[i] : 0.0f;
  for (int i = tid; i < C; i += 512) sb2[i] = p.b2 ? p.b2[i] : 0.0f;
  stage_w1(0, std::false_type{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(1);

  f32x4_t acc[2][HF];
#pragma unroll
  for (int tg = 0; tg < 2; ++tg)
#pragma unroll
    for (int f = 0; f < HF; ++f) acc[tg][f] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};

  // fragment-read lane offsets. W1 image: row half*32 + 16 i + t16, logical chunk 4 s + q stored at
  // (4 s & ~7) | ((4 s + q) ^ row) & 7 = 8 (s >> 1) + (4 (s & 1) ^ key), key = q ^ (t16 & 7).
  // W2 image: row half*C/2 + 16 f + t16, chunk q ^ ((t16 >> 1) & 2).
  const int key = q ^ (t16 & 7);
  const int a1e = (half * 32 + t16) * (W1CH * 16) + key * 16;
  const int a1o = (half * 32 + t16) * (W1CH * 16) + (4 ^ key) * 16;
  const int a2 = (half * (C / 2) + t16) * 64 + (q ^ ((t16 >> 1) & 2)) * 16;
  const int hx_w = ((pr * 2) * 2 + half) * 512 + lane * 8;   // + tg * 1024: this wave's exchange slot
  const int hx_r = (pr * 2) * 2 * 512 + lane * 8;            // + tg * 1024 + partner * 512

  // one chunk iteration: up(c) [UP], down(c-1) [DN], gate(c) [UP]. The fragment reads run 3 slots
  // ahead of their MFMAs (a slot = one up k step, 4 MFMAs, or one down fragment, 2 MFMAs) and
  // sched_barriers pin that order, so LDS latency hides under the MFMAs of the slots between.
  auto body = [&](int c, auto up_c, auto dn_c, auto par_c) {
    constexpr bool UP = decltype(up_c)::value, DN = decltype(dn_c)::value, PAR = decltype(par_c)::value;
    constexpr int NS = KS + HF;
    using Par = std::integral_constant<bool, PAR>;
    using NPar = std::integral_constant<bool, !PAR>;
    if (UP && c + 1 < NCH) stage_w1(c + 1, NPar{});
    if (UP) stage_w2(c, Par{});
    const char* s1 = PAR ? w1s1 : w1s0;
    const char* s2 = PAR ? w2s0 : w2s1;                      // W2 of chunk c - 1
    const char* hxr = (PAR ? hxs0 : hxs1) + hx_r;
    f32x4_t u[2][2];
    if constexpr (UP) {
      const float* bb = sb1 + c * W1R + half * 32 + 4 * q;
      const f32x4_t bh = *reinterpret_cast<const f32x4_t*>(bb);
      const f32x4_t bg = *reinterpret_cast<const f32x4_t*>(bb + 16);
      u[0][0] = u[1][0] = bh;
      u[0][1] = u[1][1] = bg;
    }
    bf16x8_t fr[4][2], hb[2];
    auto load = [&](auto s_c) {
      constexpr int s = decltype(s_c)::value;
      if constexpr (s < KS) {
        if constexpr (UP) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
            fr[s & 3][i] = *reinterpret_cast<const bf16x8_t*>(s1 + ((s & 1) ? a1o : a1e) + i * 16 * (W1CH * 16) +
                                                              (s >> 1) * 128);
        }
      } else if constexpr (s < NS) {
        if constexpr (DN) {
          fr[s & 3][0] = *reinterpret_cast<const bf16x8_t*>(s2 + a2 + (s - KS) * 1024);
        }
      }
    };
    static_for<0, 3>(load);
    static_for<0, NS>([&](auto s_c) {
      constexpr int s = decltype(s_c)::value;
      load(std::integral_constant<int, s + 3>{});
      if constexpr (DN && s == (KS >= 4 ? KS - 4 : 0)) {
#pragma unroll
        for (int tg = 0; tg < 2; ++tg) {
          const uint2 lo = *reinterpret_cast<const uint2*>(hxr + tg * 1024);
          const uint2 hi = *reinterpret_cast<const uint2*>(hxr + tg * 1024 + 512);
          hb[tg] = __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
        }
      }
      if constexpr (s < KS) {
        if constexpr (UP) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            u[0][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[s & 3][i], xf[0][s], u[0][i], 0, 0, 0);
            u[1][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[s & 3][i], xf[1][s], u[1][i], 0, 0, 0);
          }
        }
      } else {
        if constexpr (DN) {
          constexpr int f = s - KS;
          acc[0][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[s & 3][0], hb[0], acc[0][f], 0, 0, 0);
          acc[1][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[s & 3][0], hb[1], acc[1][f], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (UP) {
      // GEGLU gate of granule `half` (b1 entered as the accumulators' initial value); lane (t, q) holds
      // units 4q + r of its token in each group. Stored: 2 h gelu(g) = h g (1 + erf(g / sqrt 2)),
      // the factor 2 undone by W2's pack-time 0.5 (exact: both are powers of two).
      char* hx = (PAR ? hxs1 : hxs0) + hx_w;
#pragma unroll
      for (int tg = 0; tg < 2; ++tg) {
        float s4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = u[tg][1][r], hg = u[tg][0][r] * g;
          s4[r] = fmaf(hg, erf_scaled(g), hg);
        }
        *reinterpret_cast<uint2*>(hx + tg * 1024) = make_uint2(pack2(s4[0], s4[1]), pack2(s4[2], s4[3]));
      }
    }
    // W1(c+1), W2(c) landed, gated units of chunk c visible, everyone done with the buffers the
    // next iteration re-stages
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  static_assert(NCH % 2 == 0, "chunk loop unrolled by two");
  body(0, std::true_type{}, std::false_type{}, std::false_type{});
  stamp(2);
  for (int c = 1; c + 1 < NCH; c += 2) {
    body(c, std::true_type{}, std::true_type{}, std::true_type{});
    body(c + 1, std::true_type{}, std::true_type{}, std::false_type{});
    if (c + 1 == 10) stamp(3);
    if (c + 1 == 30) stamp(4);
  }
  body(NCH - 1, std::true_type{}, std::true_type{}, std::true_type{});
  body(NCH, std::false_type{}, std::true_type{}, std::false_type{});
  stamp(5);

  // ---- epilogue per token group: O^T -> per-wave fp32 slab [16 tokens][C/2 + 4] -> token rows of
  // 8-channel chunks (+ b2, residual, AlphaBlender mix) -> 16-byte stores
  constexpr int HALF = C / 2, LD = HALF, CPR = HALF / 8, NCK = 16 * CPR / 64;
  static_assert(4 * 16 * LD * 4 <= W1B && 16 * CPR % 64 == 0 && (HALF / 4) % 8 == 0, "epilogue slab");
  float* const sl = reinterpret_cast<float*>(wave < 4 ? w1s0 : w1s1) + (wave & 3) * (16 * LD);
  // 16-byte column chunk k of slab row r lives at chunk (k & ~7) | ((k ^ r) & 7): conflict-free
  auto slab = [&](int r, int k) { return &sl[r * LD + (((k & ~7) | ((k ^ r) & 7)) << 2)]; };
#pragma unroll
  for (int tg = 0; tg < 2; ++tg) {
    const int trow0 = tok0 + tg * 16;
    uint4 rr[NCK], mm[NCK];
#pragma unroll
    for (int k = 0; k < NCK; ++k) {
      const int ck = lane + 64 * k, tr = ck / CPR, c8 = (ck - tr * CPR) * 8;
      const int tk = trow0 + tr < p.M ? trow0 + tr : 0;
      const int col = half * HALF + c8;
      rr[k] = p.res ? *reinterpret_cast<const uint4*>((const bf16_t*)p.res + (size_t)tk * p.ldres + col)
                    : make_uint4(0, 0, 0, 0);
      mm[k] = p.mix ? *reinterpret_cast<const uint4*>((const bf16_t*)p.mix + (size_t)tk * p.ldmix + col)
                    : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int f = 0; f < HF; ++f)
      *reinterpret_cast<f32x4_t*>(slab(t16, f * 4 + q)) = acc[tg][f];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < NCK; ++k) {
      const int ck = lane + 64 * k, tr = ck / CPR, c8 = (ck - tr * CPR) * 8;
      const float4 x0 = *reinterpret_cast<const float4*>(slab(tr, c8 / 4));
      const float4 x1 = *reinterpret_cast<const float4*>(slab(tr, c8 / 4 + 1));
      const int col = half * HALF + c8;
      const float4 b0 = *reinterpret_cast<const float4*>(&sb2[col]);
      const float4 b1 = *reinterpret_cast<const float4*>(&sb2[col + 4]);
      float v[8] = {x0.x + b0.x, x0.y + b0.y, x0.z + b0.z, x0.w + b0.w,
                    x1.x + b1.x, x1.y + b1.y, x1.z + b1.z, x1.w + b1.w};
      if (p.res) {
        float t[8];
        unpack8(rr[k], t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
      }
      if (p.mix) {
        float t[8];
        unpack8(mm[k], t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = p.mix_alpha * t[e] + (1.0f - p.mix_alpha) * v[e];
      }
      if (trow0 + tr < p.M)
        *reinterpret_cast<uint4*>((bf16_t*)p.y + (size_t)(trow0 + tr) * p.ldy + col) = pack8(v);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // slab reads done before the next group's writes
  }
  stamp(6);
}

extern "C" int acth_geglu_ffn(const ActhFfnDesc* d, hipStream_t stream) {
  if (!d || !d->x || !d->w1 || !d->w2 || !d->y) return ACTH_EINVAL;
  if (d->C != 320 || d->M < 0) return ACTH_EINVAL;
  if (d->M == 0) return ACTH_OK;
  if (d->ldx % 8 || d->ldw1 % 8 || d->ldw2 % 8 || d->ldy % 8 || d->ldx < d->C || d->ldw1 < d->C ||
      d->ldw2 < 4 * d->C || d->ldy < d->C)
    return ACTH_EINVAL;
  if ((d->res && (d->ldres % 8 || d->ldres < d->C)) || (d->mix && (d->ldmix % 8 || d->ldmix < d->C)))
    return ACTH_EINVAL;
  if (((size_t)d->x | (size_t)d->y | (size_t)d->res | (size_t)d->mix | (size_t)d->w1 | (size_t)d->w2) & 15)
    return ACTH_EINVAL;
  const long long w1_bytes = ((long long)(8 * d->C - 1) * d->ldw1 + d->C) * 2;
  const long long w2_bytes = ((long long)(d->C - 1) * d->ldw2 + 4 * d->C) * 2;
  if (w1_bytes >= 0x80000000LL || w2_bytes >= 0x80000000LL) return ACTH_EINVAL;
  const unsigned nblk = (unsigned)((d->M + 127) / 128);
  hipLaunchKernelGGL((ffn_geglu_kernel<320>), dim3(nblk), dim3(512), 0, stream, *d, (unsigned)w1_bytes,
                     (unsigned)w2_bytes);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

extern "C" int acth_debug_ffn_stamps(unsigned long long* host_dst, int n_wgs, int enable) {
  if (!host_dst) {
    const int on = enable ? 1 : 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ffn_stamp_on), &on, sizeof(on), 0, hipMemcpyHostToDevice) == hipSuccess
               ? ACTH_OK : ACTH_ELAUNCH;
  }
  if (n_wgs <= 0 || n_wgs > FFN_STAMP_WGS) return ACTH_EINVAL;
  if (hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_ffn_stamps), (size_t)n_wgs * FFN_NSTAMP * sizeof(unsigned long long),
                          0, hipMemcpyDeviceToHost) != hipSuccess)
    return ACTH_ELAUNCH;
  return ACTH_OK;
}
