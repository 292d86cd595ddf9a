// Selective scan (mamba-ssm 1.2.0 `selective_scan_fn` semantics, delta_softplus, z = None) for
// ACTalker's SS2D_Unit (mamba_layer.py:1505-1548; op call :1532-1538).
//
// Per batch b, group k (one scan direction), channel d (N = 16 states, A = -exp(A_log)):
//   delta_l = softplus( dt_w[k,d,:] . xdbl[b,l,k,0:R] + dt_b[k,d] )   (fused dt_proj, R > 0)
//           = softplus( delta_in[b,l,k*D+d] + dt_b[k,d] )            (explicit delta, R == 0)
//   h_l     = exp(delta_l * A[k,d,:]) * h_{l-1} + delta_l * B[b,l,k,:] * u[b,l,d]
//   y_l     = < h_l , C[b,l,k,:] > + D[k,d] * u[b,l,d]
// Fused SS2D mode (flip1 = 1, u_gstride = 0): both directions read the SAME u channels and
// direction 1 visits l = L-1..0, i.e. the reference's flip_L(x) copy becomes a traversal order;
// outputs kept for l < n_keep (selected image tokens; ID / condition tokens only feed the state).
//
// Two kernels. scan_pair_kernel (nchunks <= 1, the default): one pass, the 16 states of a channel
// split over a lane pair (below). scan_kernel (nchunks > 1): one thread owns one (b, k, d)
// recurrence; at ACTalker's level-0 shape that is only 56*2*640 = 71,680 sequences (~1 wave per
// SIMD) of 9,249 serial steps, so the sequence is split into nchunks chunks scanned in two passes:
//   pass 1: every chunk but the last scans from h = 0 and records its end state H_c and sum(delta)_c;
//   pass 2: chunk c folds h_in = sum_j<c ( prod_{j<i<c} exp(A*Sdelta_i) ) H_j (exact recurrence
//           composition, 16 FMAs + exps per earlier chunk) and rescans, writing y.
// Work is ~1.8x one pass, but nchunks x more waves hide the per-token latency.
//
// Layout: u / delta / y token-major (b*L + l, channels): a wave reads 64 consecutive channels of one
// token (coalesced). xdbl rows (dt | B | C, fp32) are wave-uniform per token: staged in LDS per
// tile of SC_T tokens, read back as broadcasts; the next tile is prefetched into registers while
// the current one is scanned. State and exp(A) constants stay in registers.
#include "common.h"
#include <type_traits>

#define SC_T 16
#define SC_THREADS 128
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ float softplus_fast(float x) {
  // log1p(exp(x)) = max(x, 0) + log1p(exp(-|x|)); torch's threshold (x > 20 -> x) is implied
  const float e = fast_exp2(-fabsf(x) * 1.4426950408889634f);
  return fmaxf(x, 0.0f) + __logf(1.0f + e);
}

// R: dt rank (compile-time, 0 = explicit delta input). PASS: 0 single pass, 1 chunk state, 2 chunk output.
template <int R, int PASS>
__global__ __launch_bounds__(SC_THREADS) void scan_kernel(const ActhScanDesc p) {
  constexpr int W = R + 32;                      // floats per token and group in xdbl
  constexpr int WP = (W + 3) & ~3;               // LDS row (16-byte aligned)
  constexpr int NX = (SC_T * W + SC_THREADS - 1) / SC_THREADS;
  __shared__ __attribute__((aligned(16))) float xs[SC_T * WP];
  __shared__ __attribute__((aligned(16))) bf16_t us[SC_T * SC_THREADS];
  __shared__ __attribute__((aligned(16))) float dls[R == 0 ? SC_T * SC_THREADS : 4];

  const int k = blockIdx.y;
  const int nc = p.nchunks;
  const int ncg = PASS == 1 ? nc - 1 : nc;       // pass 1 skips the last chunk (its end state is unused)
  const int c = blockIdx.z % ncg, b = blockIdx.z / ncg;
  const int t = threadIdx.x;
  const int dbase = blockIdx.x * SC_THREADS;
  const int d = dbase + t;
  const bool active = d < p.D;
  const int dd = active ? d : 0;
  const bool rev = (k == 1) && p.flip1;
  const int i_begin = c * p.chunk_len;
  const int i_end = min(p.L, i_begin + p.chunk_len);

  float w[R > 0 ? R : 1];
#pragma unroll
  for (int r = 0; r < R; ++r) w[r] = p.dt_w[((size_t)k * p.D + dd) * R + r];
  const float bias = p.dt_b ? p.dt_b[k * p.D + dd] : 0.0f;
  float a2[16], h[16];
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    a2[n] = -__expf(p.A_log[((size_t)k * p.D + dd) * 16 + n]) * 1.4426950408889634f;
    h[n] = 0.0f;
  }
  const float dsk = p.Dskip ? p.Dskip[k * p.D + dd] : 0.0f;

  // chunk workspace: [(b*G + k)*nc + c][17][D]  (H[0..15], sum delta)
  float* wsb = p.ws + (((size_t)b * p.G + k) * nc) * 17 * (size_t)p.D + dd;
  if (PASS == 2) {
    for (int j = 0; j < c; ++j) {
      const float* src = wsb + (size_t)j * 17 * p.D;
      const float sd = src[16 * (size_t)p.D];
#pragma unroll
      for (int n = 0; n < 16; ++n) h[n] = fmaf(fast_exp2(a2[n] * sd), h[n], src[(size_t)n * p.D]);
    }
  }

  const bf16_t* ub = (const bf16_t*)p.u + (size_t)b * p.L * p.ldu + (size_t)k * p.u_gstride + dbase;
  const float* xb = p.xdbl + (size_t)b * p.L * p.ldx + k * W;
  const size_t dl_off = (size_t)b * p.L * p.ld_delta + (size_t)k * p.D + dbase;
  bf16_t* yb = (p.y1 && k == 1) ? (bf16_t*)p.y1 : (bf16_t*)p.y0 + (size_t)k * p.y_gstride;
  yb += (size_t)b * p.n_keep * p.ldy + dd;

  float px[NX];
  uint4 pu[2];
  float4 pd[R == 0 ? 4 : 1];

  auto pos_of = [&](int i) { return rev ? p.L - 1 - i : i; };
  auto prefetch = [&](int i0) {
#pragma unroll
    for (int e = 0; e < NX; ++e) {
      const int idx = t + e * SC_THREADS;
      const int tt = idx / W, col = idx - tt * W;
      const int i = i0 + tt;
      px[e] = (tt < SC_T && i < i_end) ? xb[(size_t)pos_of(i) * p.ldx + col] : 0.0f;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int idx = t + e * SC_THREADS;          // 256 x 16 B = 16 tokens x 128 channels
      const int tt = idx >> 4, cc = (idx & 15) * 8;
      const int i = i0 + tt;
      pu[e] = (i < i_end && dbase + cc < p.D)
                  ? *reinterpret_cast<const uint4*>(ub + (size_t)pos_of(i) * p.ldu + cc)
                  : make_uint4(0, 0, 0, 0);
    }
    if constexpr (R == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = t + e * SC_THREADS;        // 512 x 4 floats = 16 tokens x 128 channels
        const int tt = idx >> 5, cc = (idx & 31) * 4;
        const int i = i0 + tt;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < i_end && dbase + cc < p.D) {
          const size_t o = dl_off + (size_t)pos_of(i) * p.ld_delta + cc;
          if (p.delta_f32) {
            v = *reinterpret_cast<const float4*>((const float*)p.delta + o);
          } else {
            const uint2 r2 = *reinterpret_cast<const uint2*>((const bf16_t*)p.delta + o);
            v = make_float4(lo16f(r2.x), hi16f(r2.x),
                            lo16f(r2.y), hi16f(r2.y));
          }
        }
        pd[e] = v;
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int e = 0; e < NX; ++e) {
      const int idx = t + e * SC_THREADS;
      if (idx < SC_T * W) xs[(idx / W) * WP + (idx % W)] = px[e];
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int idx = t + e * SC_THREADS;
      *reinterpret_cast<uint4*>(&us[(idx >> 4) * SC_THREADS + (idx & 15) * 8]) = pu[e];
    }
    if constexpr (R == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = t + e * SC_THREADS;
        *reinterpret_cast<float4*>(&dls[(idx >> 5) * SC_THREADS + (idx & 31) * 4]) = pd[e];
      }
    }
  };

  float dsum = 0.0f;
  if (i_begin < i_end) prefetch(i_begin);
  for (int i0 = i_begin; i0 < i_end; i0 += SC_T) {
    commit();
    __syncthreads();
    if (i0 + SC_T < i_end) prefetch(i0 + SC_T);
    const int nt = min(SC_T, i_end - i0);
    for (int tt = 0; tt < nt; ++tt) {
      const float4* xr4 = reinterpret_cast<const float4*>(xs + tt * WP);
      float dt = bias;
      if constexpr (R == 0) {
        dt += dls[tt * SC_THREADS + t];
      } else {
#pragma unroll
        for (int r4 = 0; r4 < R / 4; ++r4) {
          const float4 v = xr4[r4];
          dt = fmaf(w[4 * r4], v.x, dt);
          dt = fmaf(w[4 * r4 + 1], v.y, dt);
          dt = fmaf(w[4 * r4 + 2], v.z, dt);
          dt = fmaf(w[4 * r4 + 3], v.w, dt);
        }
#pragma unroll
        for (int r = (R / 4) * 4; r < R; ++r) dt = fmaf(w[r], xs[tt * WP + r], dt);
      }
      if (p.softplus) dt = softplus_fast(dt);
      if (PASS == 1) dsum += dt;
      const float uu = bf2f(us[tt * SC_THREADS + t]);
      const float du = dt * uu;
      const float* Bv = xs + tt * WP + R;
      float bc[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(Bv + 4 * q);
        bc[4 * q] = v.x; bc[4 * q + 1] = v.y; bc[4 * q + 2] = v.z; bc[4 * q + 3] = v.w;
      }
      float y = 0.0f;
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        h[n] = fmaf(fast_exp2(dt * a2[n]), h[n], du * bc[n]);
        if (PASS != 1) y = fmaf(h[n], bc[16 + n], y);
      }
      if (PASS != 1) {
        y = fmaf(dsk, uu, y);
        const int l = pos_of(i0 + tt);
        if (active && l < p.n_keep) yb[(size_t)l * p.ldy] = f2bf(y);
      }
    }
    __syncthreads();
  }
  if (PASS == 1 && active) {
    float* dst = wsb + (size_t)c * 17 * p.D;
#pragma unroll
    for (int n = 0; n < 16; ++n) dst[(size_t)n * p.D] = h[n];
    dst[16 * (size_t)p.D] = dsum;
  }
}

// ------------------------------------------------------------------------------------------
// Single-pass scan with the 16 states of a channel split over a lane pair: lane 2c + j owns
// states [8j, 8j+8) of channel c. Twice the parallelism of one-thread-per-channel (2240 waves at
// ACTalker's level-0 shape) without the two-pass chunk decomposition: per token a lane reads the
// token's delta (computed per tile on the matrix core, below), does 8 state updates and half of
// the C readout (summed by a DPP swap). Tiles of SC_T tokens of xdbl / u are staged in LDS (next
// tile prefetched into registers); outputs are gathered per tile in LDS and stored with 16-byte
// coalesced writes.

// softplus with the log taken by the raw v_log_f32 (log2): its argument 1 + exp(-|x|) lies in
// [1, 2], so ocml's denormal range reduction around __logf is dead weight
__device__ __forceinline__ float softplus_raw(float x) {
  const float e = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
  return fmaxf(x, 0.0f) + __builtin_amdgcn_logf(1.0f + e) * 0.6931471805599453f;
}

__device__ __forceinline__ float pair_swap(float v) {
  // value of the partner lane (lane ^ 1): DPP quad_perm [1, 0, 3, 2]
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// CH channels per block (2 CH threads).
//
// dt_proj (R > 0) runs on the matrix core: per tile, each wave computes delta for its own 32
// channels x SC_T tokens as two v_mfma_f32_16x16x4_f32 products (fp32 in, fp32 out: bitwise an fmaf
// chain, no reduced precision), adds dt_bias and applies the softplus once per (token, channel) in
// the accumulator layout, and parks the result in LDS (`dls`, the same slot the explicit-delta mode
// stages). The recurrence lanes then read delta with one ds_read: the per-token VALU dot product
// (R/2 packed FMAs per lane), its pair reduction and the softplus that both lanes of a pair used to
// repeat leave the serial loop.
// Two descriptors: blocks with blockIdx.z < nb0 scan p0's batch elements, the rest p1's (the two SS2D
// branches of one Mamba block in one launch, acth_selective_scan2); a single scan passes p1 = p0.
// XB: xdbl rows in bf16 ([dt (R4) | B | C] per direction, the reference's x_dbl dtype), staged to fp32 in LDS;
// the grid is then 1-D and dealt XCD-major (the channel blocks of one (batch, direction) share an L2), and the
// forward direction stops at n_keep.
// Occupancy: 4 waves per SIMD (128 VGPRs) for R <= 20, and for the bf16-row form at R = 40 (level 1: 6720 waves
// take two rounds of 4096 slots instead of three of 3072; 1.98 vs 2.08-2.15 ms, the paired launch 3.52-3.56 vs
// 3.74-3.76 ms, profiles/r5_scan_occupancy_ab.log); R = 80 stays at 3 (4 spills 21 VGPRs and measured slower)
template <int R, int CH, bool SOFTPLUS, bool XB = false>
__global__ __launch_bounds__(2 * CH, (R <= 20 || (XB && R <= 40)) ? 4 : 3) void scan_pair_kernel(const ActhScanDesc p0,
                                                                             const ActhScanDesc p1, int nb0) {
  int bxi = blockIdx.x, kyi = blockIdx.y, bzi = blockIdx.z;
  if constexpr (XB) {
    const unsigned P = blockIdx.x, NB = gridDim.x, gx = (p0.D + CH - 1) / CH;
    const unsigned xcd = P & 7, q8 = NB >> 3, r8 = NB & 7;
    const unsigned wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (P >> 3);
    bxi = (int)(wg % gx);
    kyi = (int)((wg / gx) & 1);
    bzi = (int)((wg / gx) >> 1);
  }
  const bool second = bzi >= nb0;
  const ActhScanDesc& p = *(second ? &p1 : &p0);  // wave-uniform: scalar loads from the kernarg segment
  constexpr int NT = 2 * CH;                     // threads
  constexpr int SP_CH = CH;
  constexpr int U16 = CH / 8;                    // 16-byte chunks per token row of the u / y tile
  constexpr int W = R + 32;                      // floats per token and group in xdbl
  constexpr int R4 = (R + 3) & ~3;               // dt columns padded to whole 16x16x4 k-steps
  constexpr int KS = R4 / 4;                     // k-steps per lane group (group g holds k = g*KS + s)
  constexpr int WP0 = R4 + 32;                   // LDS row: [dt (R4) | B | C]
  constexpr int WP = ((WP0 / 4) % 2 == 0) ? WP0 + 4 : WP0;   // odd 16-byte stride: the MFMA B reads
                                                              // of 16 token rows hit distinct banks
  constexpr int DLP = SP_CH + 4;                 // delta tile row (padded: the 16 token rows of an
                                                 // accumulator store land in different banks)
  constexpr int NX = (SC_T * W + NT - 1) / NT;
  constexpr int XQ = (R4 + 32) / 4;              // XB: 8-byte chunks of a bf16 token row
  constexpr int NXB = (SC_T * XQ + NT - 1) / NT;
  static_assert(CH % 32 == 0, "a wave owns 32 channels");
  __shared__ __attribute__((aligned(16))) float xs[SC_T * WP];
  __shared__ __attribute__((aligned(16))) bf16_t us[SC_T * SP_CH];
  __shared__ __attribute__((aligned(16))) bf16_t ys[SC_T * SP_CH];
  __shared__ __attribute__((aligned(16))) float dls[SC_T * DLP];

  const int k = kyi, b = bzi - (second ? nb0 : 0);
  const int t = threadIdx.x;
  const int half = t & 1, cl = t >> 1;           // state half, channel within the block
  const int dbase = bxi * SP_CH;
  const int d = dbase + cl;
  const bool active = d < p.D;
  const int dd = active ? d : 0;
  const bool rev = (k == 1) && p.flip1;

  // dt_proj on MFMA: lane (g = lane >> 4, i = lane & 15) of wave w supplies A = dt_w[channel
  // 32 w + 16 mb + i][g KS + s] and B = xdbl_dt[token i][g KS + s]; its accumulator rows are the
  // channels 32 w + 16 mb + 4 g + r, column token i
  const int ln = t & 63, wv = t >> 6, mg = ln >> 4, mi = ln & 15;
  float wa[2][R > 0 ? KS : 1], bo[2][4];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int ch = dbase + 32 * wv + 16 * mb + mi;
#pragma unroll
    for (int s = 0; s < (R > 0 ? KS : 1); ++s) {
      const int r = mg * KS + s;
      wa[mb][s] = (R > 0 && r < R && ch < p.D) ? p.dt_w[((size_t)k * p.D + ch) * R + r] : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = dbase + 32 * wv + 16 * mb + 4 * mg + r;
      bo[mb][r] = (p.dt_b && co < p.D) ? p.dt_b[k * p.D + co] : 0.0f;
    }
  }
  // zero the dt padding columns once (commit() never writes them; they meet zero weights)
  if (R4 > R) {
    for (int idx = t; idx < SC_T * (R4 - R); idx += NT) {
      const int tt = idx / (R4 - R), c = idx - tt * (R4 - R);
      xs[tt * WP + R + c] = 0.0f;
    }
  }
  const float bias = p.dt_b ? p.dt_b[k * p.D + dd] : 0.0f;   // explicit-delta mode only
  // this lane's 8 states as 4 pairs: A * log2(e) and h
  f32x2_t a2[4], h[4];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    a2[n / 2][n % 2] = -__expf(p.A_log[((size_t)k * p.D + dd) * 16 + 8 * half + n]) * 1.4426950408889634f;
    h[n / 2][n % 2] = 0.0f;
  }
  const float dsk = p.Dskip ? p.Dskip[k * p.D + dd] : 0.0f;

  const bf16_t* ub = (const bf16_t*)p.u + (size_t)b * p.L * p.ldu + (size_t)k * p.u_gstride + dbase;
  const float* xb = p.xdbl + (size_t)b * p.L * p.ldx + k * W;
  const bf16_t* xbh = (const bf16_t*)p.xdbl + (size_t)b * p.L * p.ldx + k * (R4 + 32);
  const size_t dl_off = (size_t)b * p.L * p.ld_delta + (size_t)k * p.D + dbase;
  bf16_t* yb = (p.y1 && k == 1) ? (bf16_t*)p.y1 : (bf16_t*)p.y0 + (size_t)k * p.y_gstride;
  yb += (size_t)b * p.n_keep * p.ldy + dbase;
  // XB: the forward direction stops at n_keep (later tokens only feed a state nobody reads)
  const int Lend = (XB && !rev) ? p.n_keep : p.L;

  auto pos_of = [&](int i) { return rev ? p.L - 1 - i : i; };
  // XB: branch-free global traffic (buffer ops; masked lanes carry an out-of-range offset: loads return 0,
  // stores are dropped) through a 2-tile register ring, so the compiler's s_waitcnt keeps the younger
  // tile's loads and the previous tile's y stores in flight instead of draining to vmcnt(0) every tile
  constexpr int NS = XB ? 2 : 1;
  const unsigned OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(xbh), (short)0, (int)((size_t)p.L * p.ldx * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t ru =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(ub), (short)0, (int)((size_t)p.L * p.ldu * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(yb, (short)0, (int)((size_t)p.n_keep * p.ldy * 2), 0x00020000);
  float px[XB ? 1 : NX];
  uint2 pxh[NS][XB ? NXB : 1];
  uint4 pu[NS];
  float4 pd[R == 0 ? 2 : 1];
  auto prefetch = [&](auto slot, int i0) {
    constexpr int S = decltype(slot)::value;
    if constexpr (XB) {
#pragma unroll
      for (int e = 0; e < NXB; ++e) {
        const int idx = t + e * NT, tt = idx / XQ, c4 = (idx - tt * XQ) * 4;
        const bool ok = tt < SC_T && i0 + tt < Lend;
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(
            rx, (int)(ok ? (unsigned)(pos_of(i0 + tt) * p.ldx + c4) * 2u : OOB), 0, 0);
        pxh[S][e] = make_uint2(v[0], v[1]);
      }
      const int tt = t / U16, cc = (t % U16) * 8;
      const bool ok = i0 + tt < Lend && dbase + cc < p.D;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(
          ru, (int)(ok ? (unsigned)(pos_of(i0 + tt) * p.ldu + cc) * 2u : OOB), 0, 0);
      pu[S] = make_uint4(v[0], v[1], v[2], v[3]);
      return;
    } else {
#pragma unroll
      for (int e = 0; e < NX; ++e) {
        const int idx = t + e * NT;
        const int tt = idx / W, col = idx - tt * W;
        const int i = i0 + tt;
        px[e] = (tt < SC_T && i < p.L) ? xb[(size_t)pos_of(i) * p.ldx + col] : 0.0f;
      }
    }
    {
      const int tt = t / U16, cc = (t % U16) * 8;   // NT x 16 B = 16 tokens x CH channels
      const int i = i0 + tt;
      pu[S] = (i < Lend && dbase + cc < p.D) ? *reinterpret_cast<const uint4*>(ub + (size_t)pos_of(i) * p.ldu + cc)
                                             : make_uint4(0, 0, 0, 0);
    }
    if constexpr (R == 0) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int idx = t + e * NT;              // 512 x 4 floats = 16 tokens x 128 channels
        const int tt = idx / (CH / 4), cc = (idx % (CH / 4)) * 4;
        const int i = i0 + tt;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < p.L && dbase + cc < p.D) {
          const size_t o = dl_off + (size_t)pos_of(i) * p.ld_delta + cc;
          if (p.delta_f32) {
            v = *reinterpret_cast<const float4*>((const float*)p.delta + o);
          } else {
            const uint2 r2 = *reinterpret_cast<const uint2*>((const bf16_t*)p.delta + o);
            v = make_float4(lo16f(r2.x), hi16f(r2.x),
                            lo16f(r2.y), hi16f(r2.y));
          }
        }
        pd[e] = v;
      }
    }
  };
  auto commit = [&](auto slot) {
    constexpr int S = decltype(slot)::value;
    if constexpr (XB) {
#pragma unroll
      for (int e = 0; e < NXB; ++e) {
        const int idx = t + e * NT, tt = idx / XQ, c4 = (idx - tt * XQ) * 4;
        if (tt < SC_T) {
          const uint2 q = pxh[S][e];
          float4 v = make_float4(lo16f(q.x), hi16f(q.x),
                                 lo16f(q.y), hi16f(q.y));
          if (R4 > R && c4 + 4 == R4) {          // dt padding columns are ignored: zero (they meet zero weights)
            if (R4 - R >= 1) v.w = 0.f;
            if (R4 - R >= 2) v.z = 0.f;
            if (R4 - R >= 3) v.y = 0.f;
          }
          *reinterpret_cast<float4*>(&xs[tt * WP + c4]) = v;
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < NX; ++e) {
        const int idx = t + e * NT;
        if (idx < SC_T * W) {
          const int tt = idx / W, col = idx - tt * W;
          xs[tt * WP + (col < R ? col : col - R + R4)] = px[e];
        }
      }
    }
    *reinterpret_cast<uint4*>(&us[(t / U16) * SP_CH + (t % U16) * 8]) = pu[S];
    if constexpr (R == 0) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int idx = t + e * NT;
        *reinterpret_cast<float4*>(&dls[(idx / (CH / 4)) * DLP + (idx % (CH / 4)) * 4]) = pd[e];
      }
    }
  };
  // delta of the committed tile for this wave's 32 channels (R > 0): dt_proj on the matrix core,
  // + dt_bias, softplus, into dls[token][channel]. Wave-local: the recurrence lanes that read a
  // channel's delta belong to the wave that wrote it (LDS ops of one wave complete in order).
  auto delta_tile = [&]() {
    if constexpr (R > 0) {
      f32x4_t acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float bv = xs[mi * WP + mg * KS + s];
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[0][s], bv, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[1][s], bv, acc[1], 0, 0, 0);
      }
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        float4 o;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = acc[mb][r] + bo[mb][r];
          v[r] = SOFTPLUS ? softplus_raw(x) : x;
        }
        o = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(&dls[mi * DLP + 32 * wv + 16 * mb + 4 * mg]) = o;
      }
    }
  };
  // delta of token tt for this lane's channel (softplus applied)
  auto dt_of = [&](int tt) {
    if constexpr (R == 0) {
      const float x = dls[tt * DLP + cl] + bias;
      return SOFTPLUS ? softplus_raw(x) : x;
    } else {
      return dls[tt * DLP + cl];
    }
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  auto tile = [&](int i0, auto slot) {
    commit(slot);
    __syncthreads();
    if constexpr (XB) prefetch(slot, i0 + 2 * SC_T);        // unconditional: past Lend every lane is masked
    else if (i0 + SC_T < Lend) prefetch(slot, i0 + SC_T);
    delta_tile();
    const int nt = max(0, min(SC_T, Lend - i0));
    // one token of the recurrence (partial last tile)
    auto token = [&](int tt) {
      const float* xr = xs + tt * WP;
      const float dt = dt_of(tt);
      const float uu = bf2f(us[tt * SP_CH + cl]);
      const float du = dt * uu;
      const float4* bv = reinterpret_cast<const float4*>(xr + R4 + 8 * half);
      const float4* cv = reinterpret_cast<const float4*>(xr + R4 + 16 + 8 * half);
      const float4 b0 = bv[0], b1 = bv[1], c0 = cv[0], c1 = cv[1];
      const f32x2_t bb[4] = {{b0.x, b0.y}, {b0.z, b0.w}, {b1.x, b1.y}, {b1.z, b1.w}};
      const f32x2_t cc[4] = {{c0.x, c0.y}, {c0.z, c0.w}, {c1.x, c1.y}, {c1.z, c1.w}};
      const f32x2_t dt2 = {dt, dt}, du2 = {du, du};
      f32x2_t y2 = {0.0f, 0.0f};
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const f32x2_t x = dt2 * a2[n];
        const f32x2_t e = {fast_exp2(x.x), fast_exp2(x.y)};
        h[n] = __builtin_elementwise_fma(e, h[n], du2 * bb[n]);
        y2 = __builtin_elementwise_fma(h[n], cc[n], y2);
      }
      float y = y2.x + y2.y;
      y += pair_swap(y);
      // both lanes of the pair hold the same y and store the same bf16: an unconditional store keeps
      // the unrolled tile one basic block, so the scheduler can overlap the h-independent work
      // (dt, softplus, exps) of later tokens with the serial state updates
      ys[tt * SP_CH + cl] = f2bf(fmaf(dsk, uu, y));
    };
    if (nt == SC_T) {
      // Full tile, software-pipelined by hand (the compiler schedules each token's dependency chain
      // on its own): token tt+1's delta / u reads, decays exp(dt A) and inputs dt u B are computed
      // before token tt's state update so their latency hides under it.
      f32x2_t ee[2][4], db[2][4];
      float uus[2];
      auto prep = [&](int tt, int slot) {
        const float* xr = xs + tt * WP;
        const float4* bv = reinterpret_cast<const float4*>(xr + R4 + 8 * half);
        const float4 b0 = bv[0], b1 = bv[1];
        const f32x2_t bb[4] = {{b0.x, b0.y}, {b0.z, b0.w}, {b1.x, b1.y}, {b1.z, b1.w}};
        const float uu = bf2f(us[tt * SP_CH + cl]);
        const float dt = dt_of(tt), du = dt * uu;
        uus[slot] = uu;
        const f32x2_t dt2 = {dt, dt}, du2 = {du, du};
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const f32x2_t x = dt2 * a2[n];
          ee[slot][n] = (f32x2_t){fast_exp2(x.x), fast_exp2(x.y)};
          db[slot][n] = du2 * bb[n];
        }
      };
      prep(0, 0);
#pragma unroll
      for (int tt = 0; tt < SC_T; ++tt) {
        if (tt + 1 < SC_T) prep(tt + 1, (tt + 1) & 1);
        const float* xr = xs + tt * WP;
        const float4* cv = reinterpret_cast<const float4*>(xr + R4 + 16 + 8 * half);
        const float4 c0 = cv[0], c1 = cv[1];
        const f32x2_t cc[4] = {{c0.x, c0.y}, {c0.z, c0.w}, {c1.x, c1.y}, {c1.z, c1.w}};
        f32x2_t y2 = {0.0f, 0.0f};
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          h[n] = __builtin_elementwise_fma(ee[tt & 1][n], h[n], db[tt & 1][n]);
          y2 = __builtin_elementwise_fma(h[n], cc[n], y2);
        }
        float y = y2.x + y2.y;
        y += pair_swap(y);
        ys[tt * SP_CH + cl] = f2bf(fmaf(dsk, uus[tt & 1], y));
      }
    } else {
      for (int tt = 0; tt < nt; ++tt) token(tt);
    }
    __syncthreads();
    // coalesced store of the tile's kept outputs: 16 tokens x CH channels, 16 B per thread
    {
      const int tt = t / U16, cc = (t % U16) * 8;
      const int i = i0 + tt;
      if constexpr (XB) {
        const int l = pos_of(i);
        const bool ok = tt < nt && dbase + cc < p.D && l < p.n_keep;
        const uint4 v = *reinterpret_cast<const uint4*>(&ys[tt * SP_CH + cc]);
        __builtin_amdgcn_raw_buffer_store_b128((u32x4_t){v.x, v.y, v.z, v.w}, ry,
                                               (int)(ok ? (unsigned)(l * p.ldy + cc) * 2u : OOB), 0, 0);
      } else if (tt < nt && dbase + cc < p.D) {
        const int l = pos_of(i);
        if (l < p.n_keep)
          *reinterpret_cast<uint4*>(yb + (size_t)l * p.ldy + cc) =
              *reinterpret_cast<const uint4*>(&ys[tt * SP_CH + cc]);
      }
    }
  };
  prefetch(S0{}, 0);
  if constexpr (XB) {
    prefetch(S1{}, SC_T);
    for (int i0 = 0; i0 < Lend; i0 += 2 * SC_T) {   // an odd tile count runs one all-masked tile
      tile(i0, S0{});
      tile(i0 + SC_T, S1{});
    }
  } else {
    for (int i0 = 0; i0 < Lend; i0 += SC_T) tile(i0, S0{});
  }
}

// ------------------------------------------------------------------------------------------
// scan_quad_kernel: the fused SS2D scan (G = 2 directions over the same u, direction 1 reversed) on
// bf16 xdbl rows -- the reference's x_dbl dtype (mamba_layer.py:1521: einsum of the half-precision xs
// and x_proj_weight; B / C go to selective_scan_fn in that dtype) -- laid out per direction as
// [dt (R rounded up to 4) | B (16) | C (16)].
//
// Lane layout. Wave w of the block owns channels dbase + 16 w + j (j = lane & 15); lane group
// g = lane >> 4 holds states 4g .. 4g+3 of channel j (h[r] = h[state 4g + r][channel j]). That is the
// accumulator layout of a 16x16 MFMA with rows = states, columns = channels, so
//  * the input term (dt u)_t[d] B_t[n] of four tokens is ONE v_mfma_f32_16x16x1_4b_f32: four 16x16
//    rank-1 outer products B_t (x) (dt u)_t, fp32 operands and products (exact, as the fmaf it
//    replaces), on the matrix core instead of 4 VALU multiplies per lane and token;
//  * delta (dt_proj + dt_bias + softplus) of a 16-token tile is a v_mfma_f32_16x16x4_f32 chain with the
//    tile's dt columns as A (rows = tokens) and dt_w as B (columns = channels): lane (g, j) receives
//    tokens 4g..4g+3 of its own channel j and parks them in LDS for the channel's four lane groups;
//  * the readout y_t[d] = sum_n C_t[n] h_t[n][d] is 4 FMAs per lane and token, then the four lane
//    groups are summed for 4 tokens at once: 2 v_permlane32_swap + 1 v_permlane16_swap + 3 adds
//    (a reduce-scatter: lane group g ends with token tau(g) = [0, 2, 1, 3][g] of the quad).
// What stays on the VALU per lane and token: 4 x (dt * A, exp2, state FMA, readout FMA) + ~1.5
// (reduction, D skip, conversions) -- the old layout's per-(state, token) dt u B multiply is gone, and
// plain f32 ops issue at ~0.55 of the cost of packed ones on gfx950 (tools/probes/valu_probe.hip).
// Forward direction stops at n_keep: tokens past the last kept output (ID / condition tokens) only feed
// a state nobody reads. Blocks are dealt XCD-major (the channel blocks of one (batch, direction) share
// their xdbl tiles through one L2).
#ifndef SQ_CH
#define SQ_CH 64              // channels per block (16 per wave)
#endif
#define SQ_NT (SQ_CH * 4)
#ifndef SQ_OCC
#define SQ_OCC 5              // waves per SIMD the register budget targets (R <= 40)
#endif
#ifndef SQ_PF
#define SQ_PF 2               // tiles of global loads in flight (register ring)
#endif
#ifndef SQ_FENCE
#define SQ_FENCE 0
#endif
// one token's exps / C reads are not hoisted above the previous token's (register budget for occupancy)
#if SQ_FENCE
#define SQ_TOKEN_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define SQ_TOKEN_FENCE() do {} while (0)
#endif

#define SQ_UP (SQ_CH + 16)    // u / y tile row in bf16: 4 token rows land on disjoint banks

template <int R, bool SOFTPLUS>
__global__ __launch_bounds__(SQ_NT, R <= 40 ? SQ_OCC : SQ_OCC - 1) void scan_quad_kernel(const ActhScanDesc p0,
                                                                           const ActhScanDesc p1, int nb0, int gx) {
  constexpr int R4 = (R + 3) & ~3;
  constexpr int KS = R4 / 4;
  constexpr int W = R4 + 32;                              // bf16 per token and direction in xdbl
  constexpr int WP = ((W / 4) % 2 == 0) ? W + 4 : W;      // LDS row in floats: odd 16-byte count
  constexpr int DLP = 20;                                 // delta row per channel: 16 tokens + pad
  constexpr int XQ = W / 4;                               // 8-byte chunks per token row
  constexpr int XN = (16 * XQ + SQ_NT - 1) / SQ_NT;       // xdbl chunks per thread
  __shared__ __attribute__((aligned(16))) float xs[16 * WP];
  __shared__ __attribute__((aligned(16))) bf16_t us[16 * SQ_UP];
  __shared__ __attribute__((aligned(16))) bf16_t ys[16 * SQ_UP];
  __shared__ __attribute__((aligned(16))) float dls[SQ_CH * DLP];
  __shared__ float wls[SQ_CH * (R4 + 1)];

  // XCD-major block order (bijective for any grid size; hardware deals block P to XCD P % 8)
  const unsigned P = blockIdx.x, NB = gridDim.x;
  const unsigned xcd = P & 7, q8 = NB >> 3, r8 = NB & 7;
  const unsigned wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (P >> 3);
  const int bx = (int)(wg % (unsigned)gx), kz = (int)(wg / (unsigned)gx);
  const int k = kz & 1, z = kz >> 1;
  const bool second = z >= nb0;
  const ActhScanDesc& p = *(second ? &p1 : &p0);
  const int b = z - (second ? nb0 : 0);

  const int t = threadIdx.x, ln = t & 63, w = t >> 6, g = ln >> 4, j = ln & 15;
  const int dbase = bx * SQ_CH;
  const int ch = dbase + 16 * w + j;
  const bool active = ch < p.D;
  const int cc = active ? ch : 0;
  const bool rev = k == 1;
  const int Lend = rev ? p.L : p.n_keep;

  // delta MFMA B operand dt_w[k][ch][4s + g], parked in LDS (wave-local rows) rather than KS registers
  float* wlw = wls + (16 * w + j) * (R4 + 1);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int r = 4 * s + g;
    wlw[4 * s + g] = (r < R && active) ? p.dt_w[((size_t)k * p.D + cc) * R + r] : 0.0f;
  }
  const float dtb = (p.dt_b && active) ? p.dt_b[k * p.D + cc] : 0.0f;
  float a2[4], h[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a2[r] = -__expf(p.A_log[((size_t)k * p.D + cc) * 16 + 4 * g + r]) * 1.4426950408889634f;
    h[r] = 0.0f;
  }
  const float dsk = (p.Dskip && active) ? p.Dskip[k * p.D + cc] : 0.0f;

  const bf16_t* ub = (const bf16_t*)p.u + (size_t)b * p.L * p.ldu + dbase;
  const bf16_t* xb = (const bf16_t*)p.xdbl + (size_t)b * p.L * p.ldx + k * W;
  bf16_t* yb = (p.y1 && k == 1) ? (bf16_t*)p.y1 : (bf16_t*)p.y0 + (size_t)k * p.y_gstride;
  yb += (size_t)b * p.n_keep * p.ldy + dbase;
  auto pos_of = [&](int i) { return rev ? p.L - 1 - i : i; };
  // Branch-free global traffic: buffer loads / stores whose masked-off lanes carry an out-of-range offset
  // (loads return 0, stores are dropped), so every tile issues the same memory ops and the compiler's
  // s_waitcnt keeps the ring's younger loads (and the previous tile's y stores) in flight.
  const unsigned OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(xb), (short)0,
                                                                      (int)((size_t)p.L * p.ldx * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(ub), (short)0,
                                                                      (int)((size_t)p.L * p.ldu * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(yb, (short)0,
                                                                      (int)((size_t)p.n_keep * p.ldy * 2), 0x00020000);

  // global -> register prefetch ring of SQ_PF tiles (slots are compile-time: the tile loop is unrolled by SQ_PF)
  uint2 px[SQ_PF][XN], pu[SQ_PF];
  const int ut = t / (SQ_CH / 4), uc = (t % (SQ_CH / 4)) * 4;   // this thread's u / y chunk: token, channel
  auto prefetch = [&](auto slot, int i0) {
    constexpr int S = decltype(slot)::value;
#pragma unroll
    for (int e = 0; e < XN; ++e) {                        // xdbl chunk idx: token idx / XQ, column 4 (idx % XQ)
      const int idx = t + e * SQ_NT, xt = idx / XQ, xc = (idx - xt * XQ) * 4;
      const bool ok = xt < 16 && i0 + xt < Lend;
      const unsigned off = ok ? (unsigned)(pos_of(i0 + xt) * p.ldx + xc) * 2u : OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rx, (int)off, 0, 0);
      px[S][e] = make_uint2(v[0], v[1]);
    }
    const bool ok = i0 + ut < Lend && dbase + uc < p.D;
    const unsigned off = ok ? (unsigned)(pos_of(i0 + ut) * p.ldu + uc) * 2u : OOB;
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(ru, (int)off, 0, 0);
    pu[S] = make_uint2(v[0], v[1]);
  };
  auto commit = [&](auto slot) {
    constexpr int S = decltype(slot)::value;
#pragma unroll
    for (int e = 0; e < XN; ++e) {
      const int idx = t + e * SQ_NT, xt = idx / XQ, xc = (idx - xt * XQ) * 4;
      if (xt < 16)
        *reinterpret_cast<float4*>(&xs[xt * WP + xc]) =
            make_float4(lo16f(px[S][e].x), hi16f(px[S][e].x),
                        lo16f(px[S][e].y), hi16f(px[S][e].y));
    }
    *reinterpret_cast<uint2*>(&us[ut * SQ_UP + uc]) = pu[S];
  };

  float* dlw = dls + (16 * w + j) * DLP;                  // this channel's delta row (wave-local)
  const int tg = ((g & 1) << 1) | (g >> 1);               // token of the quad this lane group ends with
  const f32x16_t zero16 = {};

  // quad q (tokens 4q..4q+3 of the tile): per token the input term dt u B of the lane's 4 states is one
  // v_mfma_f32_4x4x1_16b_f32 (lane l gets A(lane 4(l >> 2) + r) x B(lane l), r = 0..3: with A = B_t[4g + (j & 3)]
  // and B = (dt u)_t[j] that is B_t[4g + r] (dt u)_t[j], exactly this lane's states)
  const float dsk0 = g == 0 ? dsk : 0.0f;                 // D u added once per channel (lane group 0)
  auto quad = [&](int q) {
    const float4 dt4 = *reinterpret_cast<const float4*>(dlw + 4 * q);
    const float dts[4] = {dt4.x, dt4.y, dt4.z, dt4.w};
    float pp[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int tt = 4 * q + s;
      const float us_ = bf2f(us[tt * SQ_UP + 16 * w + j]);
      const f32x4_t db = __builtin_amdgcn_mfma_f32_4x4x1f32(xs[tt * WP + R4 + 4 * g + (j & 3)], dts[s] * us_,
                                                            (f32x4_t){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const float4 cv = *reinterpret_cast<const float4*>(&xs[tt * WP + R4 + 16 + 4 * g]);
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = fmaf(fast_exp2(dts[s] * a2[r]), h[r], db[r]);
      pp[s] = fmaf(h[3], cv.w, fmaf(h[2], cv.z, fmaf(h[1], cv.y, fmaf(h[0], cv.x, dsk0 * us_))));
      SQ_TOKEN_FENCE();
    }
    // sum the four lane groups: lane group g ends with token tau(g)
    const auto sa = __builtin_amdgcn_permlane32_swap(__float_as_uint(pp[0]), __float_as_uint(pp[1]), false, false);
    const auto sb = __builtin_amdgcn_permlane32_swap(__float_as_uint(pp[2]), __float_as_uint(pp[3]), false, false);
    const float ra = __uint_as_float(sa[0]) + __uint_as_float(sa[1]);
    const float rb = __uint_as_float(sb[0]) + __uint_as_float(sb[1]);
    const auto sc = __builtin_amdgcn_permlane16_swap(__float_as_uint(ra), __float_as_uint(rb), false, false);
    ys[(4 * q + tg) * SQ_UP + 16 * w + j] = f2bf(__uint_as_float(sc[0]) + __uint_as_float(sc[1]));
  };

  auto tile = [&](int i0, auto slot) {
    constexpr int S = decltype(slot)::value;
    commit(slot);
    __syncthreads();
    prefetch(slot, i0 + 16 * SQ_PF);
    {
      // delta of the tile: D[token][channel] = xdt[token][:] . dt_w[channel][:] (+ bias, softplus)
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[j * WP + 4 * s + g], wlw[4 * s + g], acc, 0, 0, 0);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = acc[r] + dtb;
        v[r] = SOFTPLUS ? softplus_raw(x) : x;
      }
      *reinterpret_cast<float4*>(dlw + 4 * g) = make_float4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll 1
    for (int q = 0; q < 4; ++q) quad(q);
    __syncthreads();
    {
      const int i = i0 + ut, l = pos_of(i);
      const bool ok = i < Lend && dbase + uc < p.D && l < p.n_keep;
      const uint2 v = *reinterpret_cast<const uint2*>(&ys[ut * SQ_UP + uc]);
      __builtin_amdgcn_raw_buffer_store_b64((u32x2_t){v.x, v.y}, ry, (int)(ok ? (unsigned)(l * p.ldy + uc) * 2u : OOB),
                                            0, 0);
    }
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  prefetch(S0{}, 0);
  if constexpr (SQ_PF == 2) {
    prefetch(S1{}, 16);
    for (int i0 = 0; i0 < Lend; i0 += 32) {   // an odd tile count runs one all-masked tile (loads 0, no stores)
      tile(i0, S0{});
      tile(i0 + 16, S1{});
    }
  } else {
    for (int i0 = 0; i0 < Lend; i0 += 16) tile(i0, S0{});
  }
}

template <int R>
static int launch_scan_quad(const ActhScanDesc& a, const ActhScanDesc& b, int nb_total, hipStream_t stream) {
  const int gx = (a.D + SQ_CH - 1) / SQ_CH;
  const dim3 grid((unsigned)(gx * 2 * nb_total));
  if (a.softplus) hipLaunchKernelGGL((scan_quad_kernel<R, true>), grid, dim3(SQ_NT), 0, stream, a, b, a.nb, gx);
  else hipLaunchKernelGGL((scan_quad_kernel<R, false>), grid, dim3(SQ_NT), 0, stream, a, b, a.nb, gx);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

static int dispatch_scan_quad(const ActhScanDesc& a, const ActhScanDesc& b, int nb_total, hipStream_t stream) {
  switch (a.R) {
    case 1: return launch_scan_quad<1>(a, b, nb_total, stream);
    case 2: return launch_scan_quad<2>(a, b, nb_total, stream);
    case 3: return launch_scan_quad<3>(a, b, nb_total, stream);
    case 4: return launch_scan_quad<4>(a, b, nb_total, stream);
    case 5: return launch_scan_quad<5>(a, b, nb_total, stream);
    case 6: return launch_scan_quad<6>(a, b, nb_total, stream);
    case 8: return launch_scan_quad<8>(a, b, nb_total, stream);
    case 16: return launch_scan_quad<16>(a, b, nb_total, stream);
    case 20: return launch_scan_quad<20>(a, b, nb_total, stream);
    case 40: return launch_scan_quad<40>(a, b, nb_total, stream);
    case 80: return launch_scan_quad<80>(a, b, nb_total, stream);
    default: return ACTH_EINVAL;
  }
}

// the paired-lane kernel on bf16 xdbl rows: 1-D grid dealt XCD-major inside the kernel
template <int R>
static int launch_pair_bf16(const ActhScanDesc& a, const ActhScanDesc& b, int nb_total, hipStream_t stream) {
  const dim3 grid((unsigned)(((a.D + 127) / 128) * 2 * nb_total));
  if (a.softplus) hipLaunchKernelGGL((scan_pair_kernel<R, 128, true, true>), grid, dim3(256), 0, stream, a, b, a.nb);
  else hipLaunchKernelGGL((scan_pair_kernel<R, 128, false, true>), grid, dim3(256), 0, stream, a, b, a.nb);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

static int dispatch_pair_bf16(const ActhScanDesc& a, const ActhScanDesc& b, int nb_total, hipStream_t stream) {
  switch (a.R) {
    case 1: return launch_pair_bf16<1>(a, b, nb_total, stream);
    case 2: return launch_pair_bf16<2>(a, b, nb_total, stream);
    case 3: return launch_pair_bf16<3>(a, b, nb_total, stream);
    case 4: return launch_pair_bf16<4>(a, b, nb_total, stream);
    case 5: return launch_pair_bf16<5>(a, b, nb_total, stream);
    case 6: return launch_pair_bf16<6>(a, b, nb_total, stream);
    case 8: return launch_pair_bf16<8>(a, b, nb_total, stream);
    case 16: return launch_pair_bf16<16>(a, b, nb_total, stream);
    case 20: return launch_pair_bf16<20>(a, b, nb_total, stream);
    case 40: return launch_pair_bf16<40>(a, b, nb_total, stream);
    case 80: return launch_pair_bf16<80>(a, b, nb_total, stream);
    default: return ACTH_EINVAL;
  }
}

template <int R>
static int launch_scan(const ActhScanDesc& d, hipStream_t stream) {
  const unsigned gx = (d.D + SC_THREADS - 1) / SC_THREADS;
  if (d.nchunks <= 1) {
    // paired-lane single pass, 128 channels per block. (Measured alternatives, tools/bench_scan.py:
    // 32-channel one-wave blocks +2 % / +22 % / +22 % at levels 0 / 1 / 2; the 16 states split over
    // two waves with the xdbl row in SGPRs via scalar loads 1.9-3.2x slower, each token waiting
    // on its scalar loads.)
    // (320-channel blocks, which stage each token tile's fp32 xdbl row 2.5x less often, were measured
    // and rejected: 3.84 vs 3.98 ms at nb 56, L 9249, but 7.31 vs 4.96 ms per level-0 call in the
    // bench step (nb 84: 336 ten-wave blocks on 256 CUs run as two rounds; 840 four-wave blocks
    // balance), profiles/r2_step6_bench_scan_ch*.log, r2_step7_kernel_stats.csv.)
    const dim3 grid((d.D + 127) / 128, d.G, d.nb);
    if (d.softplus) hipLaunchKernelGGL((scan_pair_kernel<R, 128, true>), grid, dim3(256), 0, stream, d, d, d.nb);
    else hipLaunchKernelGGL((scan_pair_kernel<R, 128, false>), grid, dim3(256), 0, stream, d, d, d.nb);
  } else {
    // pass 1: every chunk but the last records its end state
    hipLaunchKernelGGL((scan_kernel<R, 1>), dim3(gx, d.G, d.nb * (d.nchunks - 1)), dim3(SC_THREADS), 0, stream, d);
    ACTH_CHECK_LAUNCH();
    hipLaunchKernelGGL((scan_kernel<R, 2>), dim3(gx, d.G, d.nb * d.nchunks), dim3(SC_THREADS), 0, stream, d);
  }
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

extern "C" size_t acth_selective_scan_workspace_size(int nb, int G, int D, int nchunks) {
  return nchunks <= 1 ? 0 : (size_t)nb * G * nchunks * 17 * (size_t)D * sizeof(float);
}

// argument checks and derived fields (nchunks / chunk_len); 1 = valid with nothing to do (n_keep 0)
static int scan_prepare(ActhScanDesc& d) {
  if (d.nb == 0) return 1;                                          // empty batch: nothing read or written
  if (!d.u || !d.xdbl || !d.A_log || !d.y0) return ACTH_EINVAL;
  if (d.R > 0 && (!d.dt_w || d.delta)) return ACTH_EINVAL;          // exactly one delta source
  if (d.R == 0 && !d.delta) return ACTH_EINVAL;
  if (d.N != 16 || d.R < 0 || d.L <= 0 || d.D <= 0 || d.nb <= 0) return ACTH_EINVAL;
  if (d.G < 1 || d.G > 65535 || (d.flip1 && d.G != 2) || (d.y1 && d.G != 2)) return ACTH_EINVAL;
  if (d.n_keep < 0 || d.n_keep > d.L) return ACTH_EINVAL;
  if (d.xdbl_bf16) {
    // bf16 xdbl: the fused SS2D form only (scan_quad_kernel), rows of [dt (R4) | B | C] per direction
    if (d.R <= 0 || d.G != 2 || !d.flip1 || d.u_gstride != 0 || d.nchunks > 1) return ACTH_EINVAL;
    if (d.ldx < 2 * (((d.R + 3) & ~3) + 32) || d.ldx % 4 || d.ldy % 4) return ACTH_EINVAL;
    // one batch element's u / xdbl / y rows must be addressable by a 32-bit buffer offset
    if ((long long)d.L * d.ldu * 2 >= (1ll << 31) || (long long)d.L * d.ldx * 2 >= (1ll << 31) ||
        (long long)d.n_keep * d.ldy * 2 >= (1ll << 31))
      return ACTH_EINVAL;
  } else if (d.ldx < d.G * (d.R + 32)) {
    return ACTH_EINVAL;
  }
  if (d.D % 8 || d.ldu % 8 || (d.delta && (d.D % 4 || d.ld_delta % 4))) return ACTH_EINVAL;
  if (d.n_keep == 0) return 1;
  if (d.nchunks < 1) d.nchunks = 1;
  if (d.nchunks > d.L) d.nchunks = d.L;
  d.chunk_len = (d.L + d.nchunks - 1) / d.nchunks;
  d.chunk_len = (d.chunk_len + SC_T - 1) / SC_T * SC_T;
  d.nchunks = (d.L + d.chunk_len - 1) / d.chunk_len;
  if (d.nchunks > 1 && !d.ws) return ACTH_EINVAL;
  if ((long long)d.nb * d.nchunks > 65535) return ACTH_EINVAL;
  if (d.R != 0 && d.R != 1 && d.R != 2 && d.R != 3 && d.R != 4 && d.R != 5 && d.R != 6 && d.R != 8 &&
      d.R != 16 && d.R != 20 && d.R != 40 && d.R != 80)
    return ACTH_EINVAL;   // dt_rank = ceil(d_model / 16): 20/40/80 in the SVD UNet; 1,2,4 toy widths
  return ACTH_OK;
}

extern "C" int acth_selective_scan(const ActhScanDesc* dp, hipStream_t stream) {
  if (!dp) return ACTH_EINVAL;
  ActhScanDesc d = *dp;
  const int rc = scan_prepare(d);
  if (rc != ACTH_OK) return rc == 1 ? ACTH_OK : rc;
  if (d.xdbl_bf16) return d.scan_algo == 1 ? dispatch_scan_quad(d, d, d.nb, stream) : dispatch_pair_bf16(d, d, d.nb, stream);
  switch (d.R) {
    case 0: return launch_scan<0>(d, stream);
    case 1: return launch_scan<1>(d, stream);
    case 2: return launch_scan<2>(d, stream);
    case 3: return launch_scan<3>(d, stream);
    case 4: return launch_scan<4>(d, stream);
    case 5: return launch_scan<5>(d, stream);
    case 6: return launch_scan<6>(d, stream);
    case 8: return launch_scan<8>(d, stream);
    case 16: return launch_scan<16>(d, stream);
    case 20: return launch_scan<20>(d, stream);
    case 40: return launch_scan<40>(d, stream);
    case 80: return launch_scan<80>(d, stream);
    default: return ACTH_EINVAL;
  }
}

template <int R>
static int launch_scan2(const ActhScanDesc& a, const ActhScanDesc& b, hipStream_t stream) {
  const dim3 grid((a.D + 127) / 128, a.G, a.nb + b.nb);
  if (a.softplus) hipLaunchKernelGGL((scan_pair_kernel<R, 128, true>), grid, dim3(256), 0, stream, a, b, a.nb);
  else hipLaunchKernelGGL((scan_pair_kernel<R, 128, false>), grid, dim3(256), 0, stream, a, b, a.nb);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// Two independent scans of the same kernel configuration (R, D, G, softplus, single pass) in one
// launch: SS2D_cond_v10's audio and expression branches (mamba_layer.py:1955-1986, each an SS2D_Unit
// scan, :1532-1538). One launch of both holds twice the waves, so the level-0 grid's last partial
// round of waves (3360 waves on 1024 SIMDs per branch) is shared instead of paid twice.
extern "C" int acth_selective_scan2(const ActhScanDesc* d0p, const ActhScanDesc* d1p, hipStream_t stream) {
  if (!d0p || !d1p) return ACTH_EINVAL;
  ActhScanDesc a = *d0p, b = *d1p;
  const int ra = scan_prepare(a), rb = scan_prepare(b);
  if ((ra != ACTH_OK && ra != 1) || (rb != ACTH_OK && rb != 1)) return ACTH_EINVAL;
  if (ra == 1 || rb == 1 || a.nchunks > 1 || b.nchunks > 1 || a.R != b.R || a.D != b.D || a.G != b.G ||
      a.softplus != b.softplus || a.xdbl_bf16 != b.xdbl_bf16 || a.scan_algo != b.scan_algo ||
      (long long)a.nb + b.nb > 65535) {
    // nothing to pair: the separate launches
    int rc = ACTH_OK;
    if (ra != 1) rc = acth_selective_scan(d0p, stream);
    if (rc == ACTH_OK && rb != 1) rc = acth_selective_scan(d1p, stream);
    return rc;
  }
  if (a.xdbl_bf16)
    return a.scan_algo == 1 ? dispatch_scan_quad(a, b, a.nb + b.nb, stream) : dispatch_pair_bf16(a, b, a.nb + b.nb, stream);
  switch (a.R) {
    case 0: return launch_scan2<0>(a, b, stream);
    case 1: return launch_scan2<1>(a, b, stream);
    case 2: return launch_scan2<2>(a, b, stream);
    case 3: return launch_scan2<3>(a, b, stream);
    case 4: return launch_scan2<4>(a, b, stream);
    case 5: return launch_scan2<5>(a, b, stream);
    case 6: return launch_scan2<6>(a, b, stream);
    case 8: return launch_scan2<8>(a, b, stream);
    case 16: return launch_scan2<16>(a, b, stream);
    case 20: return launch_scan2<20>(a, b, stream);
    case 40: return launch_scan2<40>(a, b, stream);
    case 80: return launch_scan2<80>(a, b, stream);
    default: return ACTH_EINVAL;
  }
}
