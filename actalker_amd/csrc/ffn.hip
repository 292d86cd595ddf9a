// Fused GEGLU feed-forward for the level-0 transformer blocks (C = 320): diffusers FeedForward(geglu)
// as used by BasicTransformerBlock.ff and TemporalBasicTransformerBlock.ff_in / .ff (attention.py:
// 223-343, 418-473):
//     y = W2 (h * gelu(g)) + b2 [+ residual] [AlphaBlender: a * mix + (1 - a) * (...)],
//     [h | g] = W1 x + b1,  W1: (2I, C), W2: (C, I), I = 4C.
// Two GEMMs and a 4C-wide hidden tensor per token become one kernel whose hidden activations never
// reach HBM -- the structure of flash attention (S = K Q^T -> P -> O += V^T P^T):
//   * a workgroup owns 128 tokens: 4 wave pairs x 32 tokens. A wave's 32 token rows of x live in
//     VGPRs for the whole kernel as the up projection's B operand (v_mfma_f32_32x32x16_bf16: 32x32
//     fragments hold the MFMA shadow at 8 of 32 issue cycles, against 8 of 16 for 16x16x32);
//   * the hidden dimension is walked in chunks of 32 gated units (64 rows of W1 = two 32-row
//     [hidden 16 | gate 16] granules of modules.pack_geglu; 32 columns of W2), double-buffered in
//     LDS by LDS-DMA. Wave `half` of a pair computes granule `half` for the pair's 32 tokens,
//     H^T = W1g x^T (one 32x32 fragment: lane (t, hi) holds hidden rows 8 jb + 4 hi + r and the gate
//     rows 16 higher, so the gate is lane-local), gates it in registers, keeps its 8 gated units and
//     swaps them with its partner through LDS; then it accumulates output channels
//     [C/2 * half, +C/2) of O^T += W2c H^T for the 32 tokens. A lane's 8 units are the down
//     projection's B operand as they stand: W2's K order is permuted at pack time to match (within
//     each 16-unit granule, column 8 hi + e <- unit 8 (e / 4) + 4 hi + e % 4) and scaled by 0.5;
//   * software pipeline, one barrier per chunk: iteration c runs up(c), then down(c-1) with gate(c)
//     interleaved into its MFMA slots; W1(c+1) and W2(c) are in flight meanwhile. Measured (in-kernel
//     stamps, tools/ffn_stamps.py): the LDS-DMA issue of the 60 KB weight chunk (~65 cycles per 1 KB
//     piece) is the largest cost after the MFMAs -- the price of 128 tokens per weight pass, which is
//     what the VGPR (x rows, O^T accumulators) and LDS (double-buffered chunks) budgets allow;
//   * epilogue: O^T fragments -> per-wave LDS slab (token-major) -> + b2, residual, mix -> 16-byte
//     row stores;
//   * optional input LayerNorm (norm3 / norm_in, attention.py:330-331, 449-452) on the x rows in VGPRs:
//     fp32 statistics (bf16 dot2) across the lane pair (hi = 0 / 1 hold the two channel halves), applied
//     after the prologue barrier with gamma / beta from LDS -- the LN kernel's output write and the
//     FFN's re-read of it leave HBM; optional frame-embedding row add (x + pos_emb[frame]) before it.
// Numerics match the two-kernel path: fp32 accumulation, the gated hidden rounded to bf16 before the
// down projection (as the GEGLU GEMM's bf16 output was); GELU by the degree-8 erf fit below.
// LDS images (conflict-free ds_read_b128 of 32-row fragments for the gfx950 lane groups): W1 chunk
// 64 rows x C/8 16-byte chunks, chunk index XOR ((row >> 1) & 7) inside 8-chunk groups; W2 chunk C
// rows x 4 chunks, chunk index XOR ((row >> 2) & 3).
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
  constexpr int KS = C / 16;              // k steps (16) of the up projection
  constexpr int HF = C / 64;              // output fragments (32 channels) per wave: half of C / 32
  constexpr int HC = 32;                  // gated units per chunk (two 16-unit granules)
  constexpr int NCH = I / HC;             // chunks
  constexpr int W1R = 2 * HC;             // W1 rows per chunk
  constexpr int W1CH = C / 8;             // 16-byte chunks per W1 row
  constexpr int W1B = W1R * C * 2;        // bytes of a W1 chunk image
  constexpr int W2B = C * HC * 2;         // bytes of a W2 chunk image (C rows x 64 B)
  constexpr int HXB = 4 * 2 * 64 * 16;    // gated-unit exchange: [pair 4][half 2][lane 64] x 16 B
  constexpr int NI1 = W1B / 1024, NI2 = W2B / 1024;   // DMA wave-instructions per chunk
  constexpr int NI1W = (NI1 + 7) / 8, NI2W = (NI2 + 7) / 8;
  constexpr int NS = KS + 2 * HF;         // MFMA slots per chunk iteration
  static_assert(C % 64 == 0 && W1CH % 8 == 0 && W1B % 1024 == 0 && W2B % 1024 == 0 && KS % 4 == 0, "shape");
  static_assert(2 * (W1B + W2B + HXB) + (2 * I + 6 * C) * 4 <= 160 * 1024, "LDS");
  // Every buffer is its own LDS object and the chunk loop is unrolled by two so each access names
  // its buffer at compile time: the compiler then knows an LDS-DMA write into one buffer never
  // aliases a read of another and inserts no vmcnt(0) in front of fragment reads.
  __shared__ __attribute__((aligned(16))) char w1s0[W1B], w1s1[W1B], w2s0[W2B], w2s1[W2B], hxs0[HXB], hxs1[HXB];
  // sln: LayerNorm gamma | beta; sadd: the <= 3 add rows the workgroup's 128 tokens touch (add_div % 64 == 0)
  __shared__ __attribute__((aligned(16))) float sb1[2 * I], sb2[C], sln[2 * C], sadd[3 * C];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pr = wave >> 1, half = wave & 1;
  const bool stamps = g_ffn_stamp_on && blockIdx.x < FFN_STAMP_WGS;
  auto stamp = [&](int k) {
    if (stamps && tid == 0) g_ffn_stamps[blockIdx.x * FFN_NSTAMP + k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const int l32 = lane & 31, hi = lane >> 5;
  const int tok0 = blockIdx.x * 128 + pr * 32;             // the pair's first token
  const int tok = tok0 + l32;                              // this lane's token (B-operand column)

  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.w1), (short)0, (int)w1_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r2 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.w2), (short)0, (int)w2_bytes, 0x00020000);

  // ---- DMA source offsets of this lane's 16-byte chunk of each image instruction. W1 image: 64 rows
  // x W1CH chunks, chunk index XOR ((row >> 1) & 7) inside 8-chunk groups; W2 image: C rows x 4
  // chunks, chunk index XOR ((row >> 2) & 3) -- conflict-free ds_read_b128 of 32-row fragments.
  unsigned o1[NI1W], o2[NI2W];
#pragma unroll
  for (int u = 0; u < NI1W; ++u) {
    const int pc = (wave + 8 * u) * 64 + lane;
    const int row = pc / W1CH, pch = pc - row * W1CH;
    const int lch = (pch & ~7) | ((pch ^ (row >> 1)) & 7);
    o1[u] = ((unsigned)row * p.ldw1 + lch * 8) * 2u;
  }
#pragma unroll
  for (int u = 0; u < NI2W; ++u) {
    const int pc = (wave + 8 * u) * 64 + lane;
    const int row = pc >> 2, pch = pc & 3;
    const int lch = pch ^ ((row >> 2) & 3);
    o2[u] = ((unsigned)row * p.ldw2 + lch * 8) * 2u;
  }
  auto stage_w1 = [&](int ch, auto par) {
    char* d = decltype(par)::value ? w1s1 : w1s0;
    const unsigned b = (unsigned)ch * W1R * p.ldw1 * 2u;
#pragma unroll
    for (int u = 0; u < NI1W; ++u)
      if (NI1 % 8 == 0 || wave + 8 * u < NI1)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, (lds_void*)(d + (wave + 8 * u) * 1024), 16, (int)o1[u], (int)b,
                                                 0, 0);
  };
  auto stage_w2 = [&](int ch, auto par) {
    char* d = decltype(par)::value ? w2s1 : w2s0;
    const unsigned b = (unsigned)ch * HC * 2u;
#pragma unroll
    for (int u = 0; u < NI2W; ++u)
      if (NI2 % 8 == 0 || wave + 8 * u < NI2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r2, (lds_void*)(d + (wave + 8 * u) * 1024), 16, (int)o2[u], (int)b,
                                                 0, 0);
  };

  // ---- this lane's token row of x as the up projection's B operand: k step ks holds channels
  // 16 ks + 8 hi .. + 7 [+ the add row, rounded to bf16 as the stored sum; LayerNorm'd below]
  bf16x8_t xf[KS];
  {
    const int tk = tok < p.M ? tok : 0;
    const bf16_t* xr = (const bf16_t*)p.x + (size_t)tk * p.ldx + 8 * hi;
    uint4 xv[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) xv[ks] = *reinterpret_cast<const uint4*>(xr + 16 * ks);
    const int ar0 = p.add ? blockIdx.x * 128 / p.add_div : 0;   // first add row of the workgroup
    if (p.add) {
      const int arl = (min(blockIdx.x * 128 + 127, p.M - 1)) / p.add_div;
      for (int i = tid; i < 3 * C; i += 512) {
        const int r = i / C, c = i - r * C;
        sadd[i] = ar0 + r <= arl ? bf2f(((const bf16_t*)p.add)[(size_t)(ar0 + r) * p.ldadd + c]) : 0.0f;
      }
    }
    // the row loads, the bias / LN parameter staging and W1(0)'s DMA all in flight together: one memory
    // latency for the prologue; the add / LayerNorm arithmetic runs once everything has landed
    for (int i = tid; i < 2 * I; i += 512) sb1[i] = p.b1 ? p.b1[i] : 0.0f;
    for (int i = tid; i < C; i += 512) sb2[i] = p.b2 ? p.b2[i] : 0.0f;
    if (p.ln)
      for (int i = tid; i < 2 * C; i += 512)
        sln[i] = i < C ? (p.ln_g ? p.ln_g[i] : 1.0f) : (p.ln_b ? p.ln_b[i - C] : 0.0f);
    stage_w1(0, std::false_type{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (p.add) {
      const float* ar = sadd + (tk / p.add_div - ar0) * C + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float x8[8];
        unpack8(xv[ks], x8);
        const float4 a0 = *reinterpret_cast<const float4*>(ar + 16 * ks);
        const float4 a1 = *reinterpret_cast<const float4*>(ar + 16 * ks + 4);
        x8[0] += a0.x; x8[1] += a0.y; x8[2] += a0.z; x8[3] += a0.w;
        x8[4] += a1.x; x8[5] += a1.y; x8[6] += a1.z; x8[7] += a1.w;
        xv[ks] = pack8(x8);                                  // rounded to bf16 as the stored sum
      }
    }
    if (tok >= p.M)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xv[ks] = make_uint4(0, 0, 0, 0);
    if (p.ln) {
      // statistics over the lane pair's row (hi = 0 / 1 hold the two channel halves) by bf16 dot2 into fp32:
      // sum and sum of squares straight from the packed row, no unpacked copy of it live (E[x^2] - mean^2,
      // as the attention kernels' LayerNorms)
      const bf16x2_t one2 = one2_16();
      float sm = 0.0f, q = 0.0f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const uint32_t w[4] = {xv[ks].x, xv[ks].y, xv[ks].z, xv[ks].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x2_t v2 = __builtin_bit_cast(bf16x2_t, w[j]);
          sm = dot2acc(v2, one2, sm);
          q = dot2acc(v2, v2, q);
        }
      }
      sm += __shfl_xor(sm, 32, 64);
      q += __shfl_xor(q, 32, 64);
      const float mean = sm * (1.0f / C);
      const float rstd = rsqrtf(fmaxf(q * (1.0f / C) - mean * mean, 0.0f) + p.ln_eps);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int c = 16 * ks + 8 * hi;
        float x8[8];
        unpack8(xv[ks], x8);
        const float4 g0 = *reinterpret_cast<const float4*>(&sln[c]);
        const float4 g1 = *reinterpret_cast<const float4*>(&sln[c + 4]);
        const float4 b0 = *reinterpret_cast<const float4*>(&sln[C + c]);
        const float4 b1 = *reinterpret_cast<const float4*>(&sln[C + c + 4]);
        const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) x8[e] = fmaf((x8[e] - mean) * rstd, g[e], bb[e]);
        xv[ks] = pack8(x8);
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) xf[ks] = __builtin_bit_cast(bf16x8_t, xv[ks]);
  }
  stamp(1);

  // O^T accumulators: fragment f holds channels half*C/2 + 32 f + 8 jb + 4 hi + r (register 4 jb + r)
  // of token tok0 + l32
  f32x16_t acc[HF];
#pragma unroll
  for (int f = 0; f < HF; ++f)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[f][e] = 0.0f;

  // fragment-read lane offsets. W1: row half*32 + l32 (its (row >> 1) & 7 is (l32 >> 1) & 7), logical
  // chunk 2 ks + hi stored at 8 (ks >> 2) + ((2 (ks & 3) + hi) ^ key1): four per-lane offsets by ks & 3.
  const int key1 = (l32 >> 1) & 7, key2 = (l32 >> 2) & 3;
  int a1[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) a1[m] = (half * 32 + l32) * (W1CH * 16) + (((2 * m + hi) ^ key1) * 16);
  // W2: row half*C/2 + 32 f + l32, chunk 2 G + hi (granule G) XOR key2; own granule first
  const int a2own = (half * (C / 2) + l32) * 64 + (((2 * half + hi) ^ key2) * 16);
  const int a2par = (half * (C / 2) + l32) * 64 + (((2 * (half ^ 1) + hi) ^ key2) * 16);
  const int hx_w = (pr * 2 + half) * 1024 + lane * 16;
  const int hx_r = (pr * 2 + (half ^ 1)) * 1024 + lane * 16;

  bf16x8_t hown;                                           // this wave's gated units of the last chunk
  // one chunk iteration: up(c) [UP]; down(c-1) [DN] with gate(c) [UP] interleaved into its slots
  // (independent work: the gate's VALU issues in the MFMA shadow). Fragment reads run 3 slots ahead
  // of their MFMAs; sched_barriers pin the order.
  auto body = [&](int c, auto up_c, auto dn_c, auto par_c) {
    constexpr bool UP = decltype(up_c)::value, DN = decltype(dn_c)::value, PAR = decltype(par_c)::value;
    using Par = std::integral_constant<bool, PAR>;
    using NPar = std::integral_constant<bool, !PAR>;
    if (UP && c + 1 < NCH) stage_w1(c + 1, NPar{});
    if (UP) stage_w2(c, Par{});
    const char* s1 = PAR ? w1s1 : w1s0;
    const char* s2 = PAR ? w2s0 : w2s1;                      // W2 of chunk c - 1
    const char* hxr = (PAR ? hxs0 : hxs1) + hx_r;           // partner's units of chunk c - 1
    char* hxw = (PAR ? hxs1 : hxs0) + hx_w;
    f32x16_t u;
    if constexpr (UP) {
      const float* bb = sb1 + c * W1R + half * 32 + 4 * hi;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const float4 b4 = *reinterpret_cast<const float4*>(bb + 8 * jb);
        u[4 * jb] = b4.x; u[4 * jb + 1] = b4.y; u[4 * jb + 2] = b4.z; u[4 * jb + 3] = b4.w;
      }
    }
    bf16x8_t fr[4], hpar;
    float sg[8];
    auto load = [&](auto s_c) {
      constexpr int s = decltype(s_c)::value;
      if constexpr (s < KS) {
        if constexpr (UP) fr[s & 3] = *reinterpret_cast<const bf16x8_t*>(s1 + a1[s & 3] + (s >> 2) * 128);
      } else if constexpr (s < NS) {
        if constexpr (DN) {
          constexpr int f = (s - KS) >> 1, own = ((s - KS) & 1) == 0;
          fr[s & 3] = *reinterpret_cast<const bf16x8_t*>(s2 + (own ? a2own : a2par) + f * 32 * 64);
        }
      }
    };
    auto gate = [&](int e) {                                 // unit 8 (e / 4) + 4 hi + e % 4 of the granule
      const float h = u[(e >> 2) * 4 + (e & 3)], g = u[8 + (e >> 2) * 4 + (e & 3)], hg = h * g;
      sg[e] = fmaf(hg, erf_scaled(g), hg);
    };
    static_for<0, 3>(load);
    static_for<0, NS>([&](auto s_c) {
      constexpr int s = decltype(s_c)::value;
      load(std::integral_constant<int, s + 3>{});
      // the up projection's MFMA run at raised priority (the partner wave's gate VALU fills its shadow):
      // -1 % per chunk (profiles/r2_step9_ffn_stamps_prio.log)
      if constexpr (s == 0) __builtin_amdgcn_s_setprio(1);
      if constexpr (s == KS) __builtin_amdgcn_s_setprio(0);
      if constexpr (DN && s == KS - 6) hpar = *reinterpret_cast<const bf16x8_t*>(hxr);
      if constexpr (s < KS) {
        if constexpr (UP) u = mfma32x32x16(fr[s & 3], xf[s], u);
      } else {
        if constexpr (DN) {
          constexpr int f = (s - KS) >> 1, own = ((s - KS) & 1) == 0;
          acc[f] = mfma32x32x16(fr[s & 3], own ? hown : hpar, acc[f]);
        }
        if constexpr (UP && DN && s >= KS + 1 && s < KS + 9) gate(s - KS - 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (UP) {
      if constexpr (!DN) {
#pragma unroll
        for (int e = 0; e < 8; ++e) gate(e);
      }
      // stored: 2 h gelu(g) = h g (1 + erf(g / sqrt 2)), the factor 2 undone by W2's pack-time 0.5
      hown = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(sg[0], sg[1]), pack2(sg[2], sg[3]),
                                                     pack2(sg[4], sg[5]), pack2(sg[6], sg[7])));
      *reinterpret_cast<bf16x8_t*>(hxw) = hown;
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

  // ---- epilogue in passes of up to two fragments (64 channels): O^T -> per-wave fp32 slab
  // [32 tokens][64] (16-byte chunk index XOR (row & 7)) -> token rows of 8-channel chunks (+ b2,
  // residual, AlphaBlender mix) -> 16-byte stores
  constexpr int LD = 64;
  static_assert(4 * 32 * LD * 4 <= W1B, "epilogue slab");
  float* const sl = reinterpret_cast<float*>(wave < 4 ? w1s0 : w1s1) + (wave & 3) * (32 * LD);
  auto slab = [&](int r, int k) { return &sl[r * LD + ((k ^ (r & 7)) << 2)]; };
  static_for<0, (HF + 1) / 2>([&](auto p_c) {
    constexpr int P = decltype(p_c)::value;
    constexpr int NFP = (2 * P + 1 < HF) ? 2 : 1;           // fragments in this pass
    constexpr int CPT = NFP * 4;                              // 8-channel chunks per token row
    constexpr int NCK = 32 * CPT / 64;                        // chunks per lane
    const int ch0 = half * (C / 2) + P * 64;
    uint4 rr[NCK], mm[NCK];                                 // mm: the mix row, or the add row (never both)
#pragma unroll
    for (int k = 0; k < NCK; ++k) {
      const int ck = lane + 64 * k, tr = ck / CPT, c8 = (ck - tr * CPT) * 8;
      const int tk = tok0 + tr < p.M ? tok0 + tr : 0;
      rr[k] = p.res ? *reinterpret_cast<const uint4*>((const bf16_t*)p.res + (size_t)tk * p.ldres + ch0 + c8)
                    : make_uint4(0, 0, 0, 0);
      mm[k] = p.mix ? *reinterpret_cast<const uint4*>((const bf16_t*)p.mix + (size_t)tk * p.ldmix + ch0 + c8)
            : p.add ? *reinterpret_cast<const uint4*>((const bf16_t*)p.add + (size_t)(tk / p.add_div) * p.ldadd +
                                                      ch0 + c8)
                    : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int f = 0; f < NFP; ++f)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const f32x16_t& a = acc[2 * P + f];
        *reinterpret_cast<f32x4_t*>(slab(l32, f * 8 + 2 * jb + hi)) =
            f32x4_t{a[4 * jb], a[4 * jb + 1], a[4 * jb + 2], a[4 * jb + 3]};
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < NCK; ++k) {
      const int ck = lane + 64 * k, tr = ck / CPT, c8 = (ck - tr * CPT) * 8;
      const float4 x0 = *reinterpret_cast<const float4*>(slab(tr, c8 / 4));
      const float4 x1 = *reinterpret_cast<const float4*>(slab(tr, c8 / 4 + 1));
      const int col = ch0 + c8;
      const float4 b0 = *reinterpret_cast<const float4*>(&sb2[col]);
      const float4 b1 = *reinterpret_cast<const float4*>(&sb2[col + 4]);
      float v[8] = {x0.x + b0.x, x0.y + b0.y, x0.z + b0.z, x0.w + b0.w,
                    x1.x + b1.x, x1.y + b1.y, x1.z + b1.z, x1.w + b1.w};
      if (p.res) {
        float t[8];
        unpack8(rr[k], t);
        if (p.add) {                                         // residual = bf16(res + add row), as stored
          float a[8];
          unpack8(mm[k], a);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] += a[e];
          unpack8(pack8(t), t);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
      }
      if (p.mix) {
        float t[8];
        unpack8(mm[k], t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = p.mix_alpha * t[e] + (1.0f - p.mix_alpha) * v[e];
      }
      if (tok0 + tr < p.M) *reinterpret_cast<uint4*>((bf16_t*)p.y + (size_t)(tok0 + tr) * p.ldy + col) = pack8(v);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // slab reads done before the next pass's writes
  });
  stamp(6);
}

extern "C" int acth_geglu_ffn(const ActhFfnDesc* d, hipStream_t stream) {
  if (d && d->M == 0) return ACTH_OK;   // no rows: nothing read or written
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
  if (d->add && (d->mix || d->ldadd % 8 || d->ldadd < d->C || d->add_div <= 0 || d->add_div % 64 ||
                 ((size_t)d->add & 15)))
    return ACTH_EINVAL;
  if (d->ln && !(d->ln_eps > 0.0f)) return ACTH_EINVAL;
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
