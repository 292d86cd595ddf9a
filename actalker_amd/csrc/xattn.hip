// Fused IP-adapter cross attention with its surrounding LayerNorms (gfx950): the attn2 of the level-0
// BasicTransformerBlock / TemporalBasicTransformerBlock (attention.py:223-343, 418-473) with the
// reference's IPAdapterAttnProcessor2_0 (attention_processor.py:2747-2934):
//     n  = LN2(h)                                                     (norm2)
//     a  = Wo ( v_id + sa ma[s] softmax_32(q K^T / 8) V + sb mb[s] v_vasa ) + bo,   q = Wq n
//     h' = h + a,   n3 = LN3(h')                                     (norm3: the feed-forward's input)
// ID and VASA are single-key attentions (softmax over one key is 1: the value row itself); only the
// 32-key audio attention is evaluated. Its query and output projections fold into the keys and values
// of each head h (exact algebra, head dim 64):
//     q_h . k_{h,j} / 8 = n . K'_{h,j},        K'_{h,j} = Wq_h^T k_{h,j} / 8            (C wide)
//     Wo sum_h P_h V_h = sum_{h,j} P_{h,j} V'_{h,j},   V'_{h,j} = Wo_h v_{h,j}           (C wide)
// so per token the kernel reads h once and writes h' and n3. The q GEMM, the output GEMM, the LN2 / LN3
// kernels and the q / attention-output tensors of the unfused path (11 activation passes) disappear
// (3 passes remain). K' / V' (H*32 rows per context: one frame, or one window for the temporal block) are
// built per call by acth_ip_fold; the kernel streams one head's K' | V' (2 x 32 x C bf16) per step through
// LDS by LDS-DMA, double-buffered.
//
// Per workgroup 64 tokens of one context = 2 wave pairs x 32 tokens; both waves of a pair compute the
// head's scores for the pair's tokens (the 32x32 S^T = K'_h n^T fragment: v_mfma_f32_32x32x16_bf16, the
// LN2 rows held in VGPRs as the B operand, as ffn.hip holds its x rows), take the softmax in registers
// (lane = token; its 16 keys plus the 16 of lane ^ 32) and accumulate HALF of the output channels each,
// O^T += V'_h^T P^T (P^T is the score accumulator as it stands; V' fragments by transpose reads,
// attention.hip's P.V scheme). The head images stream through a 3-slot LDS ring (K''_0 V'_0 K''_1 ...: two
// chunks in flight while one is read); ~66 KB of LDS and 256 VGPRs x 4 waves let two workgroups share a CU.
// LN2 is folded too (below), so the raw rows of h are the score operand, and they also serve as the
// epilogue's residual through an LDS row tile: h' = h + base + weighted O -> tile -> stored h', LN3 -> n3.
#include <type_traits>

#include "common.h"

typedef __attribute__((address_space(3))) void lds_void;
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4_t lds_short4;
typedef short short8_t __attribute__((ext_vector_type(8)));

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// ------------------------------------------------------------------------------------------ fold
// K''[ctx][h*32 + j][c] = g2[c] K'[.][c],  K' = kscale * sum_d K[ctx*32 + j][64h + d] Wq[64h + d][c]
// gb[ctx][h*32 + j]     = (sum_c K''[.][c] (the stored bf16 values), sum_c b2[c] K'[.][c])   (LN2 folded)
// V'[ctx][h*32 + j][c]  = sum_d V[ctx*32 + j][64h + d] WoT[64h + d][c]      (WoT = Wo^T)
// base[ctx][c] = bo[c] + sum_d vid[ctx][d] WoT[d][c];   vbw[ctx][c] = sum_d vb[ctx][d] WoT[d][c]
// grid (nctx, H + 1), C threads: blocks y < H fold head y (thread: 4 channels x 8 keys, register-blocked,
// the head's K / V slices staged transposed in LDS), y == H the single-key rows. fp32 accumulation.
__global__ __launch_bounds__(1024) void ip_fold_kernel(const ActhIpFoldDesc p) {
  __shared__ __attribute__((aligned(16))) float kt[64][32], vt[64][32], xs[2][8192];
  const int ctx = blockIdx.x, hd = blockIdx.y, t = threadIdx.x;
  const int C = p.C;
  if (hd == p.H) {
    const bf16_t* vi = (const bf16_t*)p.vid + (size_t)ctx * p.ldvid;
    const bf16_t* vv = p.vb ? (const bf16_t*)p.vb + (size_t)ctx * p.ldvb : nullptr;
    xs[0][t] = bf2f(vi[t]);
    xs[1][t] = vv ? bf2f(vv[t]) : 0.0f;
    __syncthreads();
    float a = p.bo ? p.bo[t] : 0.0f, b = 0.0f;
    const bf16_t* w = (const bf16_t*)p.wo + t;                 // WoT[d][t], coalesced over t
    for (int d = 0; d < C; ++d) {
      const float wv = bf2f(w[(size_t)d * p.ldwo]);
      a = fmaf(wv, xs[0][d], a);
      b = fmaf(wv, xs[1][d], b);
    }
    p.base[(size_t)ctx * C + t] = a;
    if (vv) p.vbw[(size_t)ctx * C + t] = b;
    return;
  }
  if (!p.kv) return;
  for (int i = t; i < 32 * 64; i += C) {
    const int j = i >> 6, d = i & 63;
    const bf16_t* row = (const bf16_t*)p.kv + (size_t)(ctx * 32 + j) * p.ldkv;
    kt[d][j] = bf2f(row[64 * hd + d]);
    vt[d][j] = bf2f(row[C + 64 * hd + d]);
  }
  __syncthreads();
  const int ncg = C / 4, cg = t % ncg, jg = t / ncg;         // 4 channels, keys 8 jg .. 8 jg + 7
  float ak[8][4], av[8][4];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) { ak[j][c] = 0.0f; av[j][c] = 0.0f; }
  const bf16_t* wq = (const bf16_t*)p.wq + (size_t)(64 * hd) * p.ldwq + 4 * cg;
  const bf16_t* wo = (const bf16_t*)p.wo + (size_t)(64 * hd) * p.ldwo + 4 * cg;
#pragma unroll 4
  for (int d = 0; d < 64; ++d) {
    const uint2 q2 = *reinterpret_cast<const uint2*>(wq + (size_t)d * p.ldwq);
    const uint2 o2 = *reinterpret_cast<const uint2*>(wo + (size_t)d * p.ldwo);
    const float q4[4] = {lo16f(q2.x), hi16f(q2.x),
                         lo16f(q2.y), hi16f(q2.y)};
    const float o4[4] = {lo16f(o2.x), hi16f(o2.x),
                         lo16f(o2.y), hi16f(o2.y)};
    const float4 k0 = *reinterpret_cast<const float4*>(&kt[d][8 * jg]);
    const float4 k1 = *reinterpret_cast<const float4*>(&kt[d][8 * jg + 4]);
    const float4 v0 = *reinterpret_cast<const float4*>(&vt[d][8 * jg]);
    const float4 v1 = *reinterpret_cast<const float4*>(&vt[d][8 * jg + 4]);
    const float k8[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
    const float v8[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        ak[j][c] = fmaf(k8[j], q4[c], ak[j][c]);
        av[j][c] = fmaf(v8[j], o4[c], av[j][c]);
      }
  }
  // K'' = g2 o (kscale K') stored bf16; per key G = sum_c K''_jc of the stored values, B = b2 . (kscale K')
  float g4[4], b4[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    g4[c] = p.g2 ? p.g2[4 * cg + c] : 1.0f;
    b4[c] = p.b2 ? p.b2[4 * cg + c] : 0.0f;
  }
  bf16_t* kp = (bf16_t*)p.kp + (((size_t)ctx * p.H + hd) * 32 + 8 * jg) * C + 4 * cg;
  bf16_t* vp = (bf16_t*)p.vp + (((size_t)ctx * p.H + hd) * 32 + 8 * jg) * C + 4 * cg;
  float2* red = reinterpret_cast<float2*>(&xs[0][0]);        // [jg][j][cg] partial (G, B)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float k[4], gpart = 0.0f, bpart = 0.0f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float kk = ak[j][c] * p.kscale;
      k[c] = kk * g4[c];
      bpart = fmaf(b4[c], kk, bpart);
    }
    const uint2 kb = make_uint2(pack2(k[0], k[1]), pack2(k[2], k[3]));
    gpart = lo16f(kb.x) + hi16f(kb.x) + lo16f(kb.y) +
            hi16f(kb.y);
    *reinterpret_cast<uint2*>(kp + (size_t)j * C) = kb;
    *reinterpret_cast<uint2*>(vp + (size_t)j * C) = make_uint2(pack2(av[j][0], av[j][1]), pack2(av[j][2], av[j][3]));
    red[(jg * 8 + j) * ncg + cg] = make_float2(gpart, bpart);
  }
  __syncthreads();
  if (t < 32) {
    float g = 0.0f, b = 0.0f;
    for (int i = 0; i < ncg; ++i) {
      const float2 v = red[t * ncg + i];
      g += v.x;
      b += v.y;
    }
    reinterpret_cast<float2*>(p.gb)[((size_t)ctx * p.H + hd) * 32 + t] = make_float2(g, b);
  }
}

extern "C" int acth_ip_fold(const ActhIpFoldDesc* d, hipStream_t stream) {
  if (!d || !d->wo || !d->vid || !d->base || d->nctx <= 0 || d->C <= 0 || d->H <= 0) return ACTH_EINVAL;
  if (d->C % 64 || d->C > 1024 || d->H * 64 != d->C || d->ldwo % 4 || (d->vb && !d->vbw)) return ACTH_EINVAL;
  if ((size_t)d->wo & 7) return ACTH_EINVAL;
  if (d->kv && (!d->wq || !d->kp || !d->vp || !d->gb || d->ldkv < 2 * d->C || d->ldwq % 4 || ((size_t)d->wq & 7)))
    return ACTH_EINVAL;
  if (d->nctx > 65535) return ACTH_EINVAL;
  hipLaunchKernelGGL(ip_fold_kernel, dim3(d->nctx, d->H + 1), dim3(d->C), 0, stream, *d);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------ fused block
// In-kernel phase stamps (diagnostics, off unless acth_debug_xattn_stamps enabled them): s_memtime per
// workgroup at entry, heads landed, LN2 statistics, after the head loop, after epilogue phase 1, at the end.
#define XA_STAMP_WGS 8192
#define XA_NSTAMP 6
__device__ unsigned long long g_xa_stamps[XA_STAMP_WGS * XA_NSTAMP];
__device__ int g_xa_stamp_on;

// (one width, C = 320: a template instance of this kernel loses its host launch stub under hipcc 7.2)
#define XA_C 320
#define XA_TOK 64                           // tokens per workgroup: 2 wave pairs x 32
__global__ __launch_bounds__(256, 2) void xattn_kernel(const ActhXattnDesc p, unsigned k_bytes) {
  constexpr int C = XA_C;
  constexpr int T = XA_TOK;
  constexpr int KS = C / 16;               // k steps of the score product (20)
  constexpr int HF = C / 64;               // 32-channel output fragments per wave: half of C (5)
  constexpr int RB = C * 2;                // bytes of a K'' / V' / h row
  constexpr int NCK = C / 8;               // 16-byte chunks per row (40)
  constexpr int CB = 32 * RB;              // one chunk: a head's K'' or V' image (20 KB)
  constexpr int NP = CB / 1024;            // 1 KiB LDS-DMA pieces per chunk (20)
  constexpr int NW = 4;                    // waves
  constexpr int NPW = NP / NW;             // pieces per wave and chunk (5)
  constexpr int NSLOT = 3;                 // chunk ring: one being read, two landing
  constexpr int TRB = RB + 16;             // epilogue tile row stride: 656 B = 164 dwords, so the 32 rows a
                                           // wave touches in one access (lane = token) hit distinct banks
  constexpr int SLOT = 32 * TRB;           // ring slot: a chunk image (32 x RB) or 32 padded tile rows
  constexpr int TILE = T * TRB;            // epilogue row tile (41 KB): ring slots 0 / 1
  constexpr int MAXH = 16;
  static_assert(CB % 1024 == 0 && NP % NW == 0 && NCK % 8 == 0 && TILE == 2 * SLOT && T == 64, "shape");
  constexpr int H = C / 64;                // heads (compile time: the chunk ring's slots are named statically)
  // ring slots | g3 b3 base vbw (C each) | per-key (G, B) of every head | LN3 partial sums (2 x T x 2):
  // ~66 KB, two workgroups per CU, so one's loads and stores overlap the other's MFMA phases. Each slot is
  // its own LDS object and every access names its slot at compile time (the head loop is unrolled), so the
  // compiler sees that an in-flight LDS-DMA into one slot never aliases the fragment reads of another and
  // inserts no vmcnt(0) in front of them (ffn.hip)
  __shared__ __attribute__((aligned(16))) char ring0[SLOT], ring1[SLOT], ring2[SLOT];
  __shared__ __attribute__((aligned(16))) char prm[4 * C * 4 + MAXH * 32 * 8 + 2 * T * 8];
  float* const sg3 = reinterpret_cast<float*>(prm);
  float* const sb3 = sg3 + C;
  float* const sbase = sb3 + C;
  float* const svbw = sbase + C;
  float2* const sgb = reinterpret_cast<float2*>(svbw + C);
  float2* const sst = sgb + MAXH * 32;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pr = wave >> 1, half = wave & 1;
  const int l32 = lane & 31, hi = lane >> 5;
  const int row0 = blockIdx.x * T;
  const int ctx = row0 / p.rows_per_ctx;    // rows_per_ctx % T == 0: a tile lies in one context
  const int tl = pr * 32 + l32;             // this lane's token in the tile (the score product's B column)
  const int tok = row0 + tl;
  const bool use_a = p.kp != nullptr;
  const bool stamps = g_xa_stamp_on && blockIdx.x < XA_STAMP_WGS;
  auto stamp = [&](int k) {
    if (stamps && tid == 0) g_xa_stamps[blockIdx.x * XA_NSTAMP + k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);

  for (int i = tid; i < C; i += NW * 64) {
    sg3[i] = p.g3 ? p.g3[i] : 1.0f;
    sb3[i] = p.b3 ? p.b3[i] : 0.0f;
    sbase[i] = p.base[(size_t)ctx * p.ldbase + i];
    svbw[i] = p.vbw ? p.vbw[(size_t)ctx * p.ldvbw + i] : 0.0f;
  }
  if (use_a)
    for (int i = tid; i < p.H * 32; i += NW * 64)
      sgb[i] = reinterpret_cast<const float2*>(p.gb)[(size_t)ctx * p.H * 32 + i];

  // ---- LDS-DMA of chunk q of the context's stream K''_0 V'_0 K''_1 V'_1 ... into ring slot q % 3. Lane L of
  // piece pc fills LDS chunk 64 pc + L = (row, slot) with the logical 16-byte chunk of that row its image's
  // swizzle puts there: K'' XOR ((row >> 1) & 7) inside 8-chunk groups (conflict-free 32-row fragment reads,
  // ffn.hip's W1 image), V' XOR ((row >> 1) & 1) << 2 (the transpose reads of attention.hip's V tile).
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.kp ? p.kp : p.h), (short)0,
                                                                     (int)(p.kp ? k_bytes : 0u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.vp ? p.vp : p.h), (short)0,
                                                                     (int)(p.vp ? k_bytes : 0u), 0x00020000);
  unsigned koff[NPW], voff[NPW];
#pragma unroll
  for (int u = 0; u < NPW; ++u) {
    const int pc = wave + NW * u;
    const int q = 64 * pc + lane, row = q / NCK, pch = q - row * NCK;
    koff[u] = (unsigned)(row * RB + (((pch & ~7) | ((pch ^ (row >> 1)) & 7)) << 4));
    voff[u] = (unsigned)(row * RB + ((pch ^ (((row >> 1) & 1) << 2)) << 4));
  }
  const unsigned img0 = (unsigned)ctx * H * CB;
  constexpr int NCHUNK = 2 * H;
  auto slot = [&](auto q_c) -> char* {
    constexpr int q = decltype(q_c)::value;
    if constexpr (q % NSLOT == 0) return ring0;
    else if constexpr (q % NSLOT == 1) return ring1;
    else return ring2;
  };
  auto stage = [&](auto q_c) {
    constexpr int q = decltype(q_c)::value;
    char* dst = slot(q_c);
    const unsigned base = img0 + (unsigned)(q >> 1) * CB;
#pragma unroll
    for (int u = 0; u < NPW; ++u) {
      const int pc = wave + NW * u;
      if constexpr (q & 1)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_void*)(dst + pc * 1024), 16, voff[u], (int)base, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void*)(dst + pc * 1024), 16, koff[u], (int)base, 0, 0);
    }
  };
  // chunk q landed for every wave (this wave's DMAs counted, then a barrier). Called before chunk q + 2 is
  // issued: only chunk q + 1's pieces may stay in flight (vmcnt counts this wave's loads in issue order)
  // The first wait also retires this wave's LDS writes (lgkmcnt(0)): the per-key LN2 constants (sgb) and the
  // per-channel rows staged above with plain ds_writes are read by other waves after this barrier, and gfx950's
  // s_barrier does not wait for them by itself.
  auto wait_chunk = [&](auto q_c) {
    constexpr int q = decltype(q_c)::value;
    if constexpr (q == 0 && q + 1 < NCHUNK) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NPW) : "memory");
    else if constexpr (q == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else if constexpr (q + 1 < NCHUNK) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  f32x16_t acc[HF];
#pragma unroll
  for (int f = 0; f < HF; ++f)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[f][e] = 0.0f;

  // epilogue row tile: the pair's 32 token rows in ring slot 0 / 1
  bf16_t* const trow = reinterpret_cast<bf16_t*>((pr ? ring1 : ring0) + l32 * TRB);
  if (use_a) {
    // LN2 folded into the scores: with n = (h - mu) rstd g2 + b2 and K'' = g2 o K' (acth_ip_fold),
    //   n . K'_j = rstd (h . K''_j - mu G_j) + B_j,   G_j = sum_c K''_jc,  B_j = b2 . K'_j
    // so the raw bf16 row of h is the score product's B operand as loaded (channels 16 ks + 8 hi + 0..7 of
    // this lane; lane ^ 32 holds the other half), and only its mean / variance are computed here (v_dot2
    // on the packed bf16 pairs: sum h and sum h^2 without unpacking)
    bf16x8_t xf[KS];
    {
      const bf16_t* hr = (const bf16_t*)p.h + (size_t)(tok < p.M ? tok : 0) * p.ldh + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xf[ks] = *reinterpret_cast<const bf16x8_t*>(hr + 16 * ks);
    }
    using I0 = std::integral_constant<int, 0>;
    stage(I0{});
    stage(std::integral_constant<int, 1>{});
    float s1 = 0.0f, s2 = 0.0f;
    wait_chunk(I0{});
    stamp(1);
    {
      const bf16x2_t one = one2_16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16x2_t pair = {xf[ks][2 * e], xf[ks][2 * e + 1]};
          s1 = dot2acc(pair, one, s1);
          s2 = dot2acc(pair, pair, s2);
        }
    }
    {
      const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(s1), __float_as_uint(s1), false, false);
      const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s2), __float_as_uint(s2), false, false);
      s1 = __uint_as_float(a[0]) + __uint_as_float(a[1]);
      s2 = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    }
    const float mean = s1 * (1.0f / C);
    const float rstd = rsqrtf(fmaxf(s2 * (1.0f / C) - mean * mean, 0.0f) + p.eps2);
    const float nmr = -mean * rstd;
    stamp(2);

    // fragment read offsets. K'': row l32 (key), logical chunk 2 ks + hi at 8 (ks >> 2) + ((2 (ks & 3) + hi)
    // ^ key1). V' (transpose reads): lane group tg = lane / 16 covers channels 16 (tg & 1) + 4 tp of a
    // 32-channel fragment and keys 8 rd + 4 (tg >> 1) + tq of a 16-key step (the key order of the S^T
    // accumulator rows that form the B operand; attention.hip)
    const int key1 = (l32 >> 1) & 7;
    int a1[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) a1[m] = l32 * RB + (((2 * m + hi) ^ key1) << 4);
    const int tg = lane >> 4, ti = lane & 15, tq = ti >> 2, tp = ti & 3;
    const int tdcol = (tg & 1) * 16 + 4 * tp;

    static_for<0, H>([&](auto h_c) {
      constexpr int hh = decltype(h_c)::value, qk = 2 * hh, qv = qk + 1;
      using QK = std::integral_constant<int, qk>;
      using QV = std::integral_constant<int, qv>;
      if constexpr (hh > 0) wait_chunk(QK{});
      if constexpr (qk + 2 < NCHUNK) stage(std::integral_constant<int, qk + 2>{});   // slot chunk qk - 1 left
      // ---- S^T = K''_h h^T (keys x tokens), then the LN2 correction; log2 units (K' carries log2(e) / 8)
      const char* kb = slot(QK{});
      f32x16_t u;
#pragma unroll
      for (int e = 0; e < 16; ++e) u[e] = 0.0f;
      // two independent accumulation chains (even / odd k steps): a dependent 32x32x16 MFMA waits out its
      // predecessor's full latency; fragment reads run four k steps ahead of their MFMAs
      f32x16_t u1;
#pragma unroll
      for (int e = 0; e < 16; ++e) u1[e] = 0.0f;
      bf16x8_t fr[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) fr[m] = *reinterpret_cast<const bf16x8_t*>(kb + a1[m]);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8_t cur = fr[ks & 3];
        if (ks + 4 < KS) fr[ks & 3] = *reinterpret_cast<const bf16x8_t*>(kb + a1[ks & 3] + ((ks + 4) >> 2) * 128);
        if (ks & 1) u1 = mfma32x32x16(cur, xf[ks], u1);
        else u = mfma32x32x16(cur, xf[ks], u);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) u[e] += u1[e];
      const float2* gbh = sgb + hh * 32 + 4 * hi;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float2 gb = gbh[8 * jb + r];                  // key 8 jb + 4 hi + r
          u[4 * jb + r] = fmaf(rstd, u[4 * jb + r], fmaf(nmr, gb.x, gb.y));
        }
      // ---- softmax over the head's 32 keys: 16 in this lane, 16 in lane ^ 32
      float mx = u[0];
#pragma unroll
      for (int e = 1; e < 16; ++e) mx = fmaxf(mx, u[e]);
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      float ex[16], sum = 0.0f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        ex[e] = __builtin_amdgcn_exp2f(u[e] - mx);
        sum += ex[e];
      }
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(sum), __float_as_uint(sum), false, false);
        sum = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
      }
      const float inv = 1.0f / sum;
      bf16x8_t pb[2];
#pragma unroll
      for (int s2i = 0; s2i < 2; ++s2i) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = pack2(ex[8 * s2i + 2 * j] * inv, ex[8 * s2i + 2 * j + 1] * inv);
        pb[s2i] = *reinterpret_cast<bf16x8_t*>(w);
      }
      // ---- O^T += V'_h^T P^T over this wave's half of the output channels
      wait_chunk(QV{});
      if constexpr (qv + 2 < NCHUNK) stage(std::integral_constant<int, qv + 2>{});
      const char* vb = slot(QV{});
      // V' fragments read one (s2i, f) step ahead of their MFMAs
      auto vread = [&](int s2i, int f) {
        short4_t t2[2];
#pragma unroll
        for (int rd = 0; rd < 2; ++rd) {
          const int key = 16 * s2i + 8 * rd + 4 * (tg >> 1) + tq;
          const int sv = ((key >> 1) & 1) << 2;
          const int d = half * (C / 2) + 32 * f + tdcol;
          const char* a = vb + key * RB + (((d >> 3) ^ sv) << 4) + (d & 7) * 2;
          t2[rd] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)a);
        }
        return (short8_t){t2[0][0], t2[0][1], t2[0][2], t2[0][3], t2[1][0], t2[1][1], t2[1][2], t2[1][3]};
      };
      short8_t vcur = vread(0, 0), vnxt;
#pragma unroll
      for (int st = 0; st < 2 * HF; ++st) {
        const int s2i = st / HF, f = st % HF;
        if (st + 1 < 2 * HF) vnxt = vread((st + 1) / HF, (st + 1) % HF);
        acc[f] = mfma32x32x16(__builtin_bit_cast(bf16x8_t, vcur), pb[s2i], acc[f]);
        vcur = vnxt;
      }
    });
    // every wave done with the ring, then the pair's raw h rows into the tile (the epilogue's residual):
    // wave `half` writes k steps ks = half (mod 2) of its lane's channels 16 ks + 8 hi
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int ks = half; ks < KS; ks += 2) *reinterpret_cast<bf16x8_t*>(trow + 16 * ks + 8 * hi) = xf[ks];
  } else {
    // no audio term: the residual rows straight into the tile
    for (int i = tid; i < T * NCK; i += NW * 64) {
      const int r = i / NCK, c = i - r * NCK;
      const int row = row0 + r < p.M ? row0 + r : 0;
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>((r < 32 ? ring0 : ring1) + (r & 31) * TRB) + 8 * c) =
          *reinterpret_cast<const uint4*>((const bf16_t*)p.h + (size_t)row * p.ldh + 8 * c);
    }
  }
  __syncthreads();
  stamp(3);

  // ---- epilogue (no global loads, no cross-lane shuffles):
  //  (1) accumulator layout: h' = h + base + wa O + wb vbw for the wave's 80 channels of the lane's token (h
  //      from the tile, h' written back in place), rounded to bf16 (the stored residual stream); partial LN3
  //      sums over the stored values -> LDS
  //  (2) coalesced 16-byte stores of h' from the tile; LN3 statistics of each token from the partials
  //  (3) accumulator layout: n3 = (h' - mean) rstd g3 + b3 -> tile;  (4) coalesced stores of n3
  const int spos = (tok < p.M ? tok : 0) % p.S;
  {
    const float wa = use_a ? p.sa * (p.mask_a ? p.mask_a[spos] : 1.0f) : 0.0f;
    const float wb = p.vbw ? p.sb * (p.mask_b ? p.mask_b[spos] : 1.0f) : 0.0f;
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int f = 0; f < HF; ++f)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int c0 = half * (C / 2) + 32 * f + 8 * jb + 4 * hi;
        const uint2 hv = *reinterpret_cast<const uint2*>(trow + c0);
        const float4 bs = *reinterpret_cast<const float4*>(&sbase[c0]);
        const float4 vw = *reinterpret_cast<const float4*>(&svbw[c0]);
        const float x0 = lo16f(hv.x), x1 = hi16f(hv.x);
        const float x2 = lo16f(hv.y), x3 = hi16f(hv.y);
        const uint2 o = make_uint2(pack2(x0 + fmaf(wb, vw.x, fmaf(wa, acc[f][4 * jb + 0], bs.x)),
                                         x1 + fmaf(wb, vw.y, fmaf(wa, acc[f][4 * jb + 1], bs.y))),
                                   pack2(x2 + fmaf(wb, vw.z, fmaf(wa, acc[f][4 * jb + 2], bs.z)),
                                         x3 + fmaf(wb, vw.w, fmaf(wa, acc[f][4 * jb + 3], bs.w))));
        *reinterpret_cast<uint2*>(trow + c0) = o;
        acc[f][4 * jb + 0] = lo16f(o.x);
        acc[f][4 * jb + 1] = hi16f(o.x);
        acc[f][4 * jb + 2] = lo16f(o.y);
        acc[f][4 * jb + 3] = hi16f(o.y);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1 += acc[f][4 * jb + r];
          s2 = fmaf(acc[f][4 * jb + r], acc[f][4 * jb + r], s2);
        }
      }
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(s1), __float_as_uint(s1), false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s2), __float_as_uint(s2), false, false);
    if (hi == 0)
      sst[half * T + tl] = make_float2(__uint_as_float(a[0]) + __uint_as_float(a[1]),
                                       __uint_as_float(b[0]) + __uint_as_float(b[1]));
  }
  __syncthreads();
  stamp(4);
  auto store_tile = [&](void* dst, int ld) {
#pragma unroll
    for (int k = 0; k < T * NCK / (NW * 64); ++k) {
      const int i = tid + NW * 64 * k, r = i / NCK, c = i - r * NCK;
      if (row0 + r < p.M)
        *reinterpret_cast<uint4*>((bf16_t*)dst + (size_t)(row0 + r) * ld + 8 * c) = *reinterpret_cast<const uint4*>(
            reinterpret_cast<const bf16_t*>((r < 32 ? ring0 : ring1) + (r & 31) * TRB) + 8 * c);
    }
  };
  store_tile(p.out, p.ldo);
  if (!p.n3) {                                // LN3 folded into the feed-forward kernel instead
    if (stamps) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stamp(5);
    }
    return;
  }
  float mean, rstd;
  {
    const float2 x = sst[tl], y = sst[T + tl];
    mean = (x.x + y.x) * (1.0f / C);
    rstd = rsqrtf(fmaxf((x.y + y.y) * (1.0f / C) - mean * mean, 0.0f) + p.eps3);
  }
  __syncthreads();                            // every h' row read out of the tile
  {
#pragma unroll
    for (int f = 0; f < HF; ++f)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int c0 = half * (C / 2) + 32 * f + 8 * jb + 4 * hi;
        const float4 g = *reinterpret_cast<const float4*>(&sg3[c0]);
        const float4 bb = *reinterpret_cast<const float4*>(&sb3[c0]);
        const float v[4] = {acc[f][4 * jb], acc[f][4 * jb + 1], acc[f][4 * jb + 2], acc[f][4 * jb + 3]};
        *reinterpret_cast<uint2*>(trow + c0) =
            make_uint2(pack2(fmaf((v[0] - mean) * rstd, g.x, bb.x), fmaf((v[1] - mean) * rstd, g.y, bb.y)),
                       pack2(fmaf((v[2] - mean) * rstd, g.z, bb.z), fmaf((v[3] - mean) * rstd, g.w, bb.w)));
      }
  }
  __syncthreads();
  store_tile(p.n3, p.ldn3);
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(5);
  }
}

extern "C" int acth_debug_xattn_stamps(unsigned long long* host_dst, int n_wgs, int enable) {
  if (!host_dst) {
    const int on = enable ? 1 : 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_xa_stamp_on), &on, sizeof(on), 0, hipMemcpyHostToDevice) == hipSuccess
               ? ACTH_OK : ACTH_ELAUNCH;
  }
  if (n_wgs <= 0 || n_wgs > XA_STAMP_WGS) return ACTH_EINVAL;
  if (hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_xa_stamps), (size_t)n_wgs * XA_NSTAMP * sizeof(unsigned long long),
                          0, hipMemcpyDeviceToHost) != hipSuccess)
    return ACTH_ELAUNCH;
  return ACTH_OK;
}

extern "C" int acth_xattn(const ActhXattnDesc* d, hipStream_t stream) {
  if (d && d->M == 0) return ACTH_OK;   // no rows: nothing read or written
  if (!d || !d->h || !d->base || !d->out) return ACTH_EINVAL;
  if (d->C != XA_C || d->H * 64 != d->C || d->M <= 0) return ACTH_EINVAL;
  if (d->rows_per_ctx <= 0 || d->rows_per_ctx % XA_TOK || d->M % d->rows_per_ctx || d->S <= 0) return ACTH_EINVAL;
  if (d->ldh % 8 || d->ldo % 8 || d->ldh < d->C || d->ldo < d->C) return ACTH_EINVAL;
  if (d->n3 && (d->ldn3 % 8 || d->ldn3 < d->C)) return ACTH_EINVAL;
  if (((size_t)d->h | (size_t)d->out | (size_t)d->n3) & 15) return ACTH_EINVAL;
  if ((size_t)d->base & 15 || (d->vbw && ((size_t)d->vbw & 15))) return ACTH_EINVAL;
  if (d->ldbase % 4 || (d->vbw && d->ldvbw % 4)) return ACTH_EINVAL;
  if ((d->kp == nullptr) != (d->vp == nullptr) || (d->kp && !d->gb) || d->H > 16) return ACTH_EINVAL;
  const long long nctx = d->M / d->rows_per_ctx;
  const long long kb = nctx * d->H * 32LL * d->C * 2;
  if (kb >= 0x80000000LL) return ACTH_EINVAL;
  hipLaunchKernelGGL(xattn_kernel, dim3(d->M / XA_TOK), dim3(256), 0, stream, *d, (unsigned)kb);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
