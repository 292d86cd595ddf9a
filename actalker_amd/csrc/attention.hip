// Attention kernels for the SVD spatio-temporal UNet (head_dim = 64 everywhere).
//
//  * acth_flash_attn   : spatial self-attention softmax(Q K^T * scale) V over S <= 9216 tokens
//                        (AttnProcessor2_0, reference attention_processor.py:1528-1605).
//                        Default: flash16_kernel (v_mfma_f32_16x16x32_bf16, below); FA_M16=0
//                        builds the original flash_attn_kernel.
//                        Flash-style online softmax on v_mfma_f32_32x32x16_bf16. The QK^T
//                        product is computed transposed (S^T = K Q^T) so each lane owns one
//                        query column: row max / row sum stay lane-local (+1 lane^32 exchange),
//                        and S^T's accumulator registers feed the P.V product directly as the
//                        B operand (O^T = V^T P^T), so no LDS round trip for P.
//  * acth_temporal_attn: self-attention over the F (<=32) frames of a window at every spatial
//                        position (TemporalBasicTransformerBlock.attn1, attention.py:446-448).
//  * acth_ip_attn      : IP-adapter cross attention (IPAdapterAttnProcessor2_0,
//                        attention_processor.py:2747-2934). 1-key attentions (ID, VASA) are
//                        exactly their V row (softmax over one key == 1), so only the 32-key
//                        audio attention is evaluated; region masks weight it per token.
#include "common.h"

typedef __attribute__((address_space(3))) void lds_void;

// ------------------------------------------------------------------------------------------

// Flash attention v2 structure (per block: 4 or 8 waves x 32 queries, KV tiles of 64 keys):
//  * K and V tiles move HBM/L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB = 8 rows per
//    wave-instruction), double-buffered: tile j+1 is in flight while tile j is consumed; one
//    vmcnt(0) + barrier per tile. Rows past Skv read zeros (buffer range check).
//  * Both tiles stay row-major [key][d] (128-B rows). K feeds S^T = K Q^T as the A operand
//    (ds_read_b128, 16-B chunks XOR-swizzled by (key >> 1) & 7: conflict-free for the 32x32x16
//    row pattern); V feeds O^T = V^T P^T through ds_read_b64_tr_b16, the hardware transpose read
//    (chunks swizzled by ((key >> 1) & 1) << 2: conflict-free for its 4-row x 16-column blocks).
//  * P never leaves registers: S^T's accumulator rows are the B operand of the P.V product.

#define FA_TILE 8192            // 64 keys x 128 B
// long-sequence configuration (Sq >= 2048): waves per block and 32-query groups per wave
#ifndef FA_BIG_NW
#define FA_BIG_NW 8
#endif
#ifndef FA_BIG_QG
#define FA_BIG_QG 1
#endif
// 1: no per-tile max search; the tile's bf16 P sum bounds every p (FA_LSUM_MAX), the max is taken only
// when that bound is exceeded. 0: max search on every tile (p <= 2^FA_DEFER)
#ifndef FA_SUM_CHECK
#define FA_SUM_CHECK 1
#endif
// fp16 build: P is packed to fp16 (max 65504), so the lane sum that bounds every p stays at 2^15
#if ACTH_F16
#define FA_LSUM_MAX 32768.0f
#else
#define FA_LSUM_MAX 65536.0f
#endif
// 1: flash16_kernel (v_mfma_f32_16x16x32_bf16) for every flash launch; 0: flash_attn_kernel (32x32x16)
#ifndef FA_M16
#define FA_M16 1
#endif
#ifndef FA16_PRIO
#define FA16_PRIO 0
#endif
#ifndef FA16_BIG_NW
#define FA16_BIG_NW 8
#endif
#ifndef FA_PRIO
#define FA_PRIO 0
#endif
#ifndef FA_LATE_DMA
#define FA_LATE_DMA 0
#endif
#if FA_PRIO
#define FA_PRIO_ON() __builtin_amdgcn_s_setprio(1)
#define FA_PRIO_OFF() __builtin_amdgcn_s_setprio(0)
#else
#define FA_PRIO_ON() do {} while (0)
#define FA_PRIO_OFF() do {} while (0)
#endif

typedef short short4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4_t lds_short4;

// 16x16x16 MFMA on raw 16-bit activation fragments (4 per lane)
__device__ __forceinline__ f32x4_t mfma16x16x16_s4(short4_t a, short4_t b, f32x4_t c) {
#if ACTH_F16
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4, a), __builtin_bit_cast(h4, b), c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
#endif
}

__device__ __forceinline__ int fa_swk(int key) { return (key >> 1) & 7; }
__device__ __forceinline__ int fa_swv(int key) { return ((key >> 1) & 1) << 2; }

// IP-adapter epilogue (acth_ip_attn): out = vbase[ctx] + sa * ma[s] * attn + sb * mb[s] * vb[ctx]
struct FaIpEpi {
  const bf16_t* vbase; int ldvbase;
  const bf16_t* vb; int ldvb;
  const float* ma; const float* mb;
  float sa, sb;
  int S;
};

// NW waves per block share every K/V tile; each wave owns QG groups of 32 queries. QG = 2 halves the LDS
// fragment reads per MFMA (every K / V fragment a wave reads feeds both query groups) at twice the
// accumulator registers per wave (2 waves per SIMD instead of 4).
template <int NW, bool IP, int QG = 1>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(4 / QG, 4 / QG))) void flash_attn_kernel(const ActhAttnDesc p,
                                                                                 unsigned k_bytes, unsigned v_bytes,
                                                                                 const FaIpEpi ip) {
  __shared__ __attribute__((aligned(16))) char smem[4 * FA_TILE];   // [buf][K | V]
  constexpr int PPW = 8 / NW;                    // DMA pieces (8 rows) per wave per tile and operand

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  // XCD-aware block order: hardware block ids are dealt round-robin over the 8 XCDs (b, b + 8, ...
  // share one L2), so consecutive ids would put the query blocks of one (batch, head) -- which all
  // stream that head's K / V -- on every XCD, and each XCD would fetch K / V from beyond its L2
  // (measured: 6.2 GB read per level-0 dispatch for 0.99 GB of Q / K / V). Each XCD instead takes
  // a contiguous range of (q-block fastest, head, batch) blocks, so a head's K / V is fetched into
  // one L2 and re-read from it.
  int qblk, h, bat;
  {
    const int nq = gridDim.x, nh = gridDim.y;
    const int nwg = nq * nh * (int)gridDim.z;
    const int bid = blockIdx.x + nq * (blockIdx.y + nh * blockIdx.z);
    const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    qblk = lin % nq;
    h = (lin / nq) % nh;
    bat = lin / (nq * nh);
  }
  const int q0 = qblk * (32 * NW * QG) + wave * (32 * QG) + r32;   // query of group g: q0 + 32 g
  const bf16_t* qb = (const bf16_t*)p.q + bat * p.bsq + h * 64;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((const bf16_t*)p.k + bat * p.bsk + h * 64), (short)0, (int)k_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((const bf16_t*)p.v + bat * p.bsv + h * 64), (short)0, (int)v_bytes, 0x00020000);

  // Q^T fragments as the B operand: lane holds Q[q][16s + 8hh + j], prescaled by c = scale * log2(e)
  // (rounded to bf16) so the S^T accumulators are scores in log2 units
  const float c = p.scale * 1.4426950408889634f;
  bf16x8_t qf[QG][4];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int q = q0 + 32 * g;
      uint4 t = make_uint4(0, 0, 0, 0);
      if (q < p.Sq) t = *reinterpret_cast<const uint4*>(qb + (size_t)q * p.ldq + 16 * s + 8 * hh);
      const uint32_t tw[4] = {t.x, t.y, t.z, t.w};
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = pack2(lo16f(tw[j]) * c, hi16f(tw[j]) * c);
      qf[g][s] = *reinterpret_cast<bf16x8_t*>(w);
    }

  // DMA: wave w fills rows [8(w + NW u), +8) of each tile; lane -> (row, physical 16-B slot
  // lane & 7) holding logical chunk slot ^ swizzle(row)
  const int lrow = lane >> 3, slot = lane & 7;
  int krow[PPW], kch[PPW], vch[PPW];
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    krow[u] = (wave + NW * u) * 8 + lrow;
    kch[u] = slot ^ fa_swk(krow[u]);
    vch[u] = slot ^ fa_swv(krow[u]);
  }
  auto stage = [&](int kv0, int buf) {
    char* kt = smem + buf * 2 * FA_TILE;
    char* vt = kt + FA_TILE;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int key = kv0 + krow[u];
      const unsigned ko = key < p.Skv ? ((unsigned)key * p.ldk + kch[u] * 8) * 2u : 0x80000000u;
      const unsigned vo = key < p.Skv ? ((unsigned)key * p.ldv + vch[u] * 8) * 2u : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void*)(kt + (wave + NW * u) * 1024), 16, ko, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_void*)(vt + (wave + NW * u) * 1024), 16, vo, 0, 0, 0);
    }
  };

  // Running max m (log2 units) per query, held NEGATED in all 16 entries of an accumulator-shaped
  // vector: the first S^T MFMA of a tile accumulates onto it, so S^T comes out as s c - m, ready for
  // v_exp with no per-score FMA. The max is deferred: m is raised (O and l rescaled, the tile
  // exponentiated against the new m) only when some score of the tile exceeds it by more than
  // FA_DEFER; otherwise p = exp2(s c - m) <= 2^FA_DEFER, well inside bf16 P / fp32 O and l range.
  // The first tile always sets m. Per score the common path costs half a v_max3, one v_exp, one add
  // and half a v_cvt_pk (the textbook loop adds an FMA per score and a rescale per max increase).
  constexpr float FA_DEFER = 8.0f;
  f32x16_t negm[QG], o[QG][2];
  float l_run[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    l_run[g] = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) { negm[g][r] = 0.0f; o[g][0][r] = 0.0f; o[g][1][r] = 0.0f; }
  }

  // V transpose-read addressing: lane group tg = lane / 16 covers d block (tg & 1) * 16 (+32 for o[.][1])
  // and keys 8 * rd + 4 * (tg >> 1) + tq of the 16-key step (the k order of S^T's accumulator rows,
  // which are the B operand: element j of lane half h is key 8 * (j >> 2) + 4h + (j & 3)); lane
  // 4tq + tp of the group supplies row tq, columns 4tp..4tp+3
  const int tg = lane >> 4, ti = lane & 15, tq = ti >> 2, tp = ti & 3;
  const int tdcol = (tg & 1) * 16 + 4 * tp;          // d of this lane's 8-byte piece (o[.][0])

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int buf = 0;
  for (int kv0 = 0; kv0 < p.Skv; kv0 += 64) {
    if (!FA_LATE_DMA && kv0 + 64 < p.Skv) stage(kv0 + 64, buf ^ 1);
    const char* kt = smem + buf * 2 * FA_TILE;
    const char* vt = kt + FA_TILE;

    // ---- S^T = K Q^T - m for two 32-key subtiles (all 8 K fragments read before the first MFMA) ----
    bf16x8_t kf[2][4];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int key = sub * 32 + r32;
      const char* kr = kt + key * 128;
      const int sk = fa_swk(key);
#pragma unroll
      for (int s = 0; s < 4; ++s) kf[sub][s] = *reinterpret_cast<const bf16x8_t*>(kr + (((2 * s + hh) ^ sk) << 4));
    }
    f32x16_t st[QG][2];
    FA_PRIO_ON();
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < QG; ++g)
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
          st[g][sub] = mfma32x32x16(kf[sub][s], qf[g][s], s == 0 ? negm[g] : st[g][sub]);
    FA_PRIO_OFF();
    if (FA_LATE_DMA && kv0 + 64 < p.Skv) stage(kv0 + 64, buf ^ 1);
    if (kv0 + 64 > p.Skv) {
#pragma unroll
      for (int g = 0; g < QG; ++g)
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kv0 + sub * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh >= p.Skv) st[g][sub][r] = -INFINITY;
    }
    // ---- softmax numerators (lane = query column) ----
    bf16x8_t pf[QG][2][2];
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      float ls;
#if FA_SUM_CHECK
      // common path: no max search. p = exp2(s c - m) packed to bf16 and summed (v_dot2 on the packed
      // pairs: l accumulates exactly the bf16 weights the P.V product uses); every p <= the lane's tile sum,
      // so a sum <= FA_LSUM_MAX bounds them all and m needs no update. Otherwise (and always on the first
      // tile, which sets m) the exact max is taken and the tile is exponentiated again.
      auto expack = [&]() {
        const bf16x2_t one = one2_16();
        float l0 = 0.0f, l1 = 0.0f;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              w[j] = pack2(__builtin_amdgcn_exp2f(st[g][sub][8 * s2 + 2 * j]),
                           __builtin_amdgcn_exp2f(st[g][sub][8 * s2 + 2 * j + 1]));
              const bf16x2_t pr = __builtin_bit_cast(bf16x2_t, w[j]);
              if (j & 1) l1 = dot2acc(pr, one, l1);
              else l0 = dot2acc(pr, one, l0);
            }
            pf[g][sub][s2] = *reinterpret_cast<bf16x8_t*>(w);
          }
        return l0 + l1;
      };
      ls = expack();
      if (kv0 == 0 || __any(!(ls <= FA_LSUM_MAX))) {    // rare: raise m (NaN-safe test)
        // S^T again from the K tile still in LDS (st need not stay live through the common path)
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          const int key = sub * 32 + r32;
          const char* kr = kt + key * 128;
          const int sk = fa_swk(key);
#pragma unroll
          for (int s = 0; s < 4; ++s)
            st[g][sub] = mfma32x32x16(
                *reinterpret_cast<const bf16x8_t*>(kr + (((2 * s + hh) ^ sk) << 4)), qf[g][s],
                s == 0 ? negm[g] : st[g][sub]);
        }
        if (kv0 + 64 > p.Skv) {
#pragma unroll
          for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (kv0 + sub * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh >= p.Skv) st[g][sub][r] = -INFINITY;
        }
        float mx = st[g][0][0];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = (sub == 0 ? 1 : 0); r < 16; ++r) mx = fmaxf(mx, st[g][sub][r]);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        const float dm = kv0 == 0 ? mx : fmaxf(mx, 0.0f);
        if (kv0 > 0) {
          const float alpha = __builtin_amdgcn_exp2f(-dm);
          l_run[g] *= alpha;
#pragma unroll
          for (int r = 0; r < 16; ++r) { o[g][0][r] *= alpha; o[g][1][r] *= alpha; }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) { negm[g][r] -= dm; st[g][0][r] -= dm; st[g][1][r] -= dm; }
        ls = expack();
      }
#else
      float mx = st[g][0][0];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = (sub == 0 ? 1 : 0); r < 16; ++r) mx = fmaxf(mx, st[g][sub][r]);
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      if (kv0 == 0 || __any(!(mx <= FA_DEFER))) {    // rare: raise m (NaN-safe test)
        const float dm = kv0 == 0 ? mx : fmaxf(mx, 0.0f);
        if (kv0 > 0) {
          const float alpha = __builtin_amdgcn_exp2f(-dm);
          l_run[g] *= alpha;
#pragma unroll
          for (int r = 0; r < 16; ++r) { o[g][0][r] *= alpha; o[g][1][r] *= alpha; }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) { negm[g][r] -= dm; st[g][0][r] -= dm; st[g][1][r] -= dm; }
      }
      ls = 0.0f;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          uint32_t w[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float p0 = __builtin_amdgcn_exp2f(st[g][sub][8 * s2 + 2 * j]);
            const float p1 = __builtin_amdgcn_exp2f(st[g][sub][8 * s2 + 2 * j + 1]);
            ls += p0 + p1;
            w[j] = pack2(p0, p1);
          }
          pf[g][sub][s2] = *reinterpret_cast<bf16x8_t*>(w);
        }
#endif
      l_run[g] += ls;
    }
    // ---- O^T += V^T P^T: A operand (d rows x 16 keys) by transpose reads of row-major V ----
    FA_PRIO_ON();
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        short4_t t[2][2];
#pragma unroll
        for (int rd = 0; rd < 2; ++rd) {
          const int key = sub * 32 + 16 * s2 + 8 * rd + 4 * (tg >> 1) + tq;
          const int sv = fa_swv(key);
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) {
            const int d = tdcol + 32 * dh;
            const char* a = vt + key * 128 + ((((d >> 3) ^ sv)) << 4) + (d & 7) * 2;
            t[dh][rd] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)a);
          }
        }
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          short4_t lo = t[dh][0], hi = t[dh][1];
          typedef short short8_t __attribute__((ext_vector_type(8)));
          short8_t v8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const bf16x8_t af = *reinterpret_cast<bf16x8_t*>(&v8);
#pragma unroll
          for (int g = 0; g < QG; ++g)
            o[g][dh] = mfma32x32x16(af, pf[g][sub][s2], o[g][dh]);
        }
      }
    FA_PRIO_OFF();
    // next tile landed (this wave's DMAs) and every wave is done reading `buf`
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    buf ^= 1;
  }

#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const float lr = l_run[g] + __shfl_xor(l_run[g], 32, 64);
    const int q = q0 + 32 * g;
    if (q >= p.Sq) continue;
    float inv = 1.0f / lr;
    bf16_t* ob = (bf16_t*)p.o + bat * p.bso + (size_t)q * p.ldo + h * 64;
    float wb = 0.0f;
    const bf16_t* vbr = nullptr;
    const bf16_t* vbb = nullptr;
    if (IP) {
      const int s = q % ip.S;
      inv *= ip.sa * (ip.ma ? ip.ma[s] : 1.0f);
      vbr = ip.vbase + (size_t)bat * ip.ldvbase + h * 64;
      if (ip.vb) {
        wb = ip.sb * (ip.mb ? ip.mb[s] : 1.0f);
        vbb = ip.vb + (size_t)bat * ip.ldvb + h * 64;
      }
    }
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int d0 = 8 * gg + 4 * hh;
      float a[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) { a[e] = o[g][0][4 * gg + e] * inv; a[4 + e] = o[g][1][4 * gg + e] * inv; }
      if (IP) {
        // + vbase (+ wb * vb): 4 columns at d0 and 4 at 32 + d0
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const uint2 bw = *reinterpret_cast<const uint2*>(vbr + 32 * half + d0);
          a[4 * half + 0] += lo16f(bw.x); a[4 * half + 1] += hi16f(bw.x);
          a[4 * half + 2] += lo16f(bw.y); a[4 * half + 3] += hi16f(bw.y);
          if (vbb) {
            const uint2 cw = *reinterpret_cast<const uint2*>(vbb + 32 * half + d0);
            a[4 * half + 0] = fmaf(wb, lo16f(cw.x), a[4 * half + 0]);
            a[4 * half + 1] = fmaf(wb, hi16f(cw.x), a[4 * half + 1]);
            a[4 * half + 2] = fmaf(wb, lo16f(cw.y), a[4 * half + 2]);
            a[4 * half + 3] = fmaf(wb, hi16f(cw.y), a[4 * half + 3]);
          }
        }
      }
      uint2 w0, w1;
      w0.x = pack2(a[0], a[1]); w0.y = pack2(a[2], a[3]);
      w1.x = pack2(a[4], a[5]); w1.y = pack2(a[6], a[7]);
      *reinterpret_cast<uint2*>(ob + d0) = w0;
      *reinterpret_cast<uint2*>(ob + 32 + d0) = w1;
    }
  }
}

// ------------------------------------------------------------------------------------------
// The same flash attention on v_mfma_f32_16x16x32_bf16 (per wave 32 queries = 2 query blocks of 16;
// per 64-key tile 4 key blocks): the MI355X holds a higher clock on the 16x16 shape under sustained
// load at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS item 7). Layouts:
//  * S^T[key block kb][query block qb] (4 accumulators per lane: keys 16 kb + 4 g + r, query 16 qb +
//    (lane & 15), g = lane >> 4) = K Q^T - m, A = K rows (16 keys x 32 d, ds_read_b128 of chunk 4 ks + g),
//    B = Q^T (lane: query lane & 15, d 32 ks + 8 g .. + 7).
//  * P^T as the PV product's B operand needs no data movement: for the 32-key step t the lane's 8 k values
//    are keys 32 t + 4 g + 0..3 (S^T[2t]) and 32 t + 16 + 4 g + 0..3 (S^T[2t + 1]); the V^T A operand is
//    read in that same key order by two ds_read_b64_tr_b16 (4 keys x 16 d each; the 16 lanes of group g
//    supply keys 32 t (+16) + 4 g + (lane & 15) / 4, d 16 db + 4 (lane & 3)).
//  * V chunks are swizzled by ((key >> 1) & 3) << 1 (even, so a 32-byte d slice stays whole): the 16 keys
//    x 32 bytes of one transpose read land on distinct banks.
//  * Softmax without a per-tile max search (FA_SUM_CHECK scheme, above); row sums are lane-partial
//    (4 lanes per query) until the end.
__device__ __forceinline__ int fa_swv16(int key) { return ((key >> 1) & 3) << 1; }

template <int NW, bool IP>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(4, 4))) void flash16_kernel(
    const ActhAttnDesc p, unsigned k_bytes, unsigned v_bytes, const FaIpEpi ip) {
  __shared__ __attribute__((aligned(16))) char smem[4 * FA_TILE];   // [buf][K | V]
  constexpr int PPW = 8 / NW;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  int qblk, h, bat;
  {
    const int nq = gridDim.x, nh = gridDim.y;
    const int nwg = nq * nh * (int)gridDim.z;
    const int bid = blockIdx.x + nq * (blockIdx.y + nh * blockIdx.z);
    const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    qblk = lin % nq;
    h = (lin / nq) % nh;
    bat = lin / (nq * nh);
  }
  const int q0 = qblk * (32 * NW) + wave * 32 + l16;     // query of block qb: q0 + 16 qb
  const bf16_t* qb_ = (const bf16_t*)p.q + bat * p.bsq + h * 64;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((const bf16_t*)p.k + bat * p.bsk + h * 64), (short)0, (int)k_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((const bf16_t*)p.v + bat * p.bsv + h * 64), (short)0, (int)v_bytes, 0x00020000);

  const float c = p.scale * 1.4426950408889634f;
  bf16x8_t qf[2][2];                                    // [qb][ks]
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int q = q0 + 16 * qb;
      uint4 t = make_uint4(0, 0, 0, 0);
      if (q < p.Sq) t = *reinterpret_cast<const uint4*>(qb_ + (size_t)q * p.ldq + 32 * ks + 8 * g);
      const uint32_t tw[4] = {t.x, t.y, t.z, t.w};
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = pack2(lo16f(tw[j]) * c, hi16f(tw[j]) * c);
      qf[qb][ks] = *reinterpret_cast<bf16x8_t*>(w);
    }

  const int lrow = lane >> 3, slot = lane & 7;
  int krow[PPW], kch[PPW], vch[PPW];
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    krow[u] = (wave + NW * u) * 8 + lrow;
    kch[u] = slot ^ fa_swk(krow[u]);
    vch[u] = slot ^ fa_swv16(krow[u]);
  }
  auto stage = [&](int kv0, int buf) {
    char* kt = smem + buf * 2 * FA_TILE;
    char* vt = kt + FA_TILE;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int key = kv0 + krow[u];
      const unsigned ko = key < p.Skv ? ((unsigned)key * p.ldk + kch[u] * 8) * 2u : 0x80000000u;
      const unsigned vo = key < p.Skv ? ((unsigned)key * p.ldv + vch[u] * 8) * 2u : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void*)(kt + (wave + NW * u) * 1024), 16, ko, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_void*)(vt + (wave + NW * u) * 1024), 16, vo, 0, 0, 0);
    }
  };

  f32x4_t negm[2], o[4][2];                            // o[db][qb]: d 16 db + 4 g + r, query 16 qb + l16
  float l_run[2] = {0.0f, 0.0f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    negm[0][r] = 0.0f; negm[1][r] = 0.0f;
#pragma unroll
    for (int db = 0; db < 4; ++db) { o[db][0][r] = 0.0f; o[db][1][r] = 0.0f; }
  }
  // K fragment offsets (k step ks; key block kb adds 2048 kb: the swizzle of key 16 kb + l16 is that of l16)
  // and V transpose-read offsets (d block db; key step t / half add 4096 t + 2048 half), buffer-relative
  int koff[2], voff[4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) koff[ks] = l16 * 128 + (((4 * ks + g) ^ fa_swk(l16)) << 4);
  {
    const int tq = l16 >> 2, tp = l16 & 3, vkey = 4 * g + tq;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int d = 16 * db + 4 * tp;
      voff[db] = vkey * 128 + (((d >> 3) ^ fa_swv16(vkey)) << 4) + (d & 7) * 2;
    }
  }

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (FA16_PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);   // static priority for the younger half
  int buf = 0;
  for (int kv0 = 0; kv0 < p.Skv; kv0 += 64) {
    if (kv0 + 64 < p.Skv) stage(kv0 + 64, buf ^ 1);
    const char* kt = smem + buf * 2 * FA_TILE;
    const char* vt = kt + FA_TILE;

    // ---- S^T = K Q^T - m ----
    f32x4_t st[2][4];                                   // [qb][kb]
    {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(kt + koff[ks] + 2048 * kb);
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            st[qb][kb] = mfma16x16x32(kf, qf[qb][ks], ks == 0 ? negm[qb] : st[qb][kb]);
        }
      if (kv0 + 64 > p.Skv) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
          for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (kv0 + 16 * kb + 4 * g + r >= p.Skv) st[qb][kb][r] = -INFINITY;
      }
    }
    // ---- softmax numerators: P^T B operands pf[t][qb] (keys 32 t + 4 g + 0..3, 32 t + 16 + 4 g + 0..3) ----
    bf16x8_t pf[2][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      auto expack = [&]() {
        const bf16x2_t one = one2_16();
        float l0 = 0.0f, l1 = 0.0f;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          uint32_t w[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4_t& sv = st[qb][2 * t + (j >> 1)];
            w[j] = pack2(__builtin_amdgcn_exp2f(sv[2 * (j & 1)]), __builtin_amdgcn_exp2f(sv[2 * (j & 1) + 1]));
            const bf16x2_t pr = __builtin_bit_cast(bf16x2_t, w[j]);
            if (j & 1) l1 = dot2acc(pr, one, l1);
            else l0 = dot2acc(pr, one, l0);
          }
          pf[t][qb] = *reinterpret_cast<bf16x8_t*>(w);
        }
        return l0 + l1;
      };
      float ls = expack();
      if (kv0 == 0 || __any(!(ls <= FA_LSUM_MAX))) {    // rare: raise m (NaN-safe test)
        float mx = st[qb][0][0];
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, st[qb][kb][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float dm = kv0 == 0 ? mx : fmaxf(mx, 0.0f);
        if (kv0 > 0) {
          const float alpha = __builtin_amdgcn_exp2f(-dm);
          l_run[qb] *= alpha;
#pragma unroll
          for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[db][qb][r] *= alpha;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          negm[qb][r] -= dm;
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) st[qb][kb][r] -= dm;
        }
        ls = expack();
      }
      l_run[qb] += ls;
    }
    // ---- O^T += V^T P^T ----
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        short4_t rd2[2];
#pragma unroll
        for (int half = 0; half < 2; ++half)
          rd2[half] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(vt + voff[db] + 4096 * t + 2048 * half));
        typedef short short8_t __attribute__((ext_vector_type(8)));
        const short8_t v8 = {rd2[0][0], rd2[0][1], rd2[0][2], rd2[0][3], rd2[1][0], rd2[1][1], rd2[1][2], rd2[1][3]};
        const bf16x8_t af = __builtin_bit_cast(bf16x8_t, v8);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          o[db][qb] = mfma16x16x32(af, pf[t][qb], o[db][qb]);
      }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    buf ^= 1;
  }

#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float lr = l_run[qb] + __shfl_xor(l_run[qb], 16, 64);
    lr += __shfl_xor(lr, 32, 64);
    const int q = q0 + 16 * qb;
    if (q >= p.Sq) continue;
    float inv = 1.0f / lr;
    bf16_t* ob = (bf16_t*)p.o + bat * p.bso + (size_t)q * p.ldo + h * 64;
    float wb = 0.0f;
    const bf16_t* vbr = nullptr;
    const bf16_t* vbb = nullptr;
    if (IP) {
      const int s = q % ip.S;
      inv *= ip.sa * (ip.ma ? ip.ma[s] : 1.0f);
      vbr = ip.vbase + (size_t)bat * ip.ldvbase + h * 64;
      if (ip.vb) {
        wb = ip.sb * (ip.mb ? ip.mb[s] : 1.0f);
        vbb = ip.vb + (size_t)bat * ip.ldvb + h * 64;
      }
    }
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int d0 = 16 * db + 4 * g;
      float a[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = o[db][qb][r] * inv;
      if (IP) {
        const uint2 bw = *reinterpret_cast<const uint2*>(vbr + d0);
        a[0] += lo16f(bw.x); a[1] += hi16f(bw.x);
        a[2] += lo16f(bw.y); a[3] += hi16f(bw.y);
        if (vbb) {
          const uint2 cw = *reinterpret_cast<const uint2*>(vbb + d0);
          a[0] = fmaf(wb, lo16f(cw.x), a[0]);
          a[1] = fmaf(wb, hi16f(cw.x), a[1]);
          a[2] = fmaf(wb, lo16f(cw.y), a[2]);
          a[3] = fmaf(wb, hi16f(cw.y), a[3]);
        }
      }
      *reinterpret_cast<uint2*>(ob + d0) = make_uint2(pack2(a[0], a[1]), pack2(a[2], a[3]));
    }
  }
}

extern "C" int acth_flash_attn(const ActhAttnDesc* d, hipStream_t stream) {
  // no work (the other sizes in range): nothing read
  if (d && d->nbatch >= 0 && d->nheads >= 0 && d->Sq >= 0 && d->Skv >= 0 &&
      (d->nbatch == 0 || d->nheads == 0 || d->Sq == 0))
    return ACTH_OK;
  if (!d || !d->q || !d->k || !d->v || !d->o) return ACTH_EINVAL;
  if (d->Sq <= 0 || d->Skv <= 0 || d->nheads <= 0 || d->nbatch <= 0) return ACTH_EINVAL;
  if (d->ldq % 8 || d->ldk % 8 || d->ldv % 8 || d->ldo % 4) return ACTH_EINVAL;
  if (d->nheads > 65535 || d->nbatch > 65535) return ACTH_EINVAL;
  // K / V buffer extents seen from one (batch, head) base: rows x ld, minus the head offset
  const long long kb = ((long long)(d->Skv - 1) * d->ldk + 64) * 2, vb = ((long long)(d->Skv - 1) * d->ldv + 64) * 2;
  if (kb >= 0x80000000LL || vb >= 0x80000000LL) return ACTH_EINVAL;
  const FaIpEpi none = {};
  if (FA_M16) {
    if (d->Sq >= 2048) {
      constexpr int nq = FA16_BIG_NW * 32;
      dim3 grid((d->Sq + nq - 1) / nq, d->nheads, d->nbatch);
      hipLaunchKernelGGL((flash16_kernel<FA16_BIG_NW, false>), grid, dim3(FA16_BIG_NW * 64), 0, stream, *d,
                         (unsigned)kb, (unsigned)vb, none);
    } else {
      dim3 grid((d->Sq + 127) / 128, d->nheads, d->nbatch);
      hipLaunchKernelGGL((flash16_kernel<4, false>), grid, dim3(256), 0, stream, *d, (unsigned)kb, (unsigned)vb, none);
    }
  } else if (d->Sq >= 2048) {
    constexpr int nq = FA_BIG_NW * 32 * FA_BIG_QG;
    dim3 grid((d->Sq + nq - 1) / nq, d->nheads, d->nbatch);
    hipLaunchKernelGGL((flash_attn_kernel<FA_BIG_NW, false, FA_BIG_QG>), grid, dim3(FA_BIG_NW * 64), 0, stream, *d,
                       (unsigned)kb, (unsigned)vb, none);
  } else {
    dim3 grid((d->Sq + 127) / 128, d->nheads, d->nbatch);
    hipLaunchKernelGGL((flash_attn_kernel<4, false>), grid, dim3(256), 0, stream, *d, (unsigned)kb, (unsigned)vb,
                       none);
  }
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// Temporal self-attention over frames. qkv rows are tokens (b, f, s) = (b*F + f)*S + s with
// [q | k | v] column blocks of width C = H*64. Output o rows use the same token order.

// One wave per (b, s, head) tuple at a time, the F <= 16 NB frames padded to NB 16-frame blocks (NB = 1:
// F <= 16, the 14-frame windows of the benched workload; NB = 2: F <= 32, the reference's shipped
// n_sample_frames = 25 window, config/inference.yaml:4 -> Inference.py:573). Per tuple a lane issues 6 NB
// 16-byte loads (frames fr + 16 blk) and the wave 2 NB^2 + 4 NB^2 MFMAs:
//   S^T = K Q^T  v_mfma_f32_16x16x32_bf16 x 2 per (key block kb, query block qb): A = K, B = Q^T, both
//                loaded as 16-B row chunks (lane l -> frame 16 blk + l % 16, dims 32 ks + 8 (l / 16)); lane l
//                then holds the scores of keys 16 kb + 4 (l / 16) + i for query 16 qb + l % 16, so the softmax
//                is in-lane (over kb, i) + xor 16 / 32.
//   O^T = V^T P^T  v_mfma_f32_16x16x16bf16_1k x 4 (d tiles) x NB (query blocks) x NB (key blocks, accumulated):
//                B = P^T is the score accumulator itself (as bf16), A = V^T from a per-wave LDS transpose.
// (A thread-per-query VALU kernel spent ~1000 VALU wave-instructions per tuple against ~60 here; both
// are bound by the frame-strided row reads: 4.1-4.5 TB/s at the level-0..2 shapes, tools/bench_attn.py.)
// Tuples per wave (consecutive: heads of one row segment), all loads issued before the first use. Measured
// at NB = 1 (profiles/r4_step8_temporal_attn_tpw.log, B = 4 CFG branches): 2 -> 4.50 / 4.29 / 4.13 TB/s at
// S = 9216 / 2304 / 576, 4 -> 4.45 / 4.11 / 3.94, 8 -> 3.59 / 3.41 / 3.36 (VGPRs for 8 tuples of loads cut the
// waves per SIMD). NB = 2 keeps the same bytes in flight per wave with one tuple.
#ifndef TM_TPW
#define TM_TPW 2
#endif

template <int NB, int TPW>
__global__ __launch_bounds__(256) void temporal_attn_mfma_kernel(const ActhTemporalAttnDesc p) {
  constexpr int VLD = 16 * NB + 4;        // V^T LDS row: 16 NB keys + pad (8-B aligned reads)
  __shared__ __attribute__((aligned(16))) bf16_t vts[4][64 * VLD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const long long ntup = (long long)p.B * p.S * p.H;
  const int C = p.H * 64;
  const float c = p.scale * 1.4426950408889634f;
  bf16_t* vt = vts[wave];
  bool fok[NB];
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) fok[blk] = 16 * blk + fr < p.F;
  // every load of the wave's TPW tuples is issued before the first is used (one latency per
  // wave instead of one per tuple: the rows of a tuple are S rows apart, 64 B per lane group)
  const uint4 z = make_uint4(0, 0, 0, 0);
  uint4 qa[TPW][NB][2], ka[TPW][NB][2], va[TPW][NB][2];
  size_t rows[TPW][NB];
  int heads[TPW];
  const long long tp0 = ((long long)blockIdx.x * 4 + wave) * TPW;
#pragma unroll
  for (int it = 0; it < TPW; ++it) {
    const long long tp = tp0 + it < ntup ? tp0 + it : ntup - 1;
    const int h = (int)(tp % p.H);
    const long long bs = tp / p.H;
    const int s = (int)(bs % p.S), b = (int)(bs / p.S);
    heads[it] = h;
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      rows[it][blk] = ((size_t)b * p.F + (fok[blk] ? 16 * blk + fr : 0)) * p.S + s;   // frame 16 blk + fr
      const bf16_t* base = (const bf16_t*)p.qkv + rows[it][blk] * p.ldqkv + h * 64 + 8 * g;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        qa[it][blk][ks] = z; ka[it][blk][ks] = z; va[it][blk][ks] = z;   // guarded loads, not `fok ? *p : z`
        if (fok[blk]) {                                                  // (that form went through a stack slot)
          qa[it][blk][ks] = *reinterpret_cast<const uint4*>(base + 32 * ks);
          ka[it][blk][ks] = *reinterpret_cast<const uint4*>(base + C + 32 * ks);
          va[it][blk][ks] = *reinterpret_cast<const uint4*>(base + 2 * C + 32 * ks);
        }
      }
    }
  }
#pragma unroll
  for (int it = 0; it < TPW; ++it) {
    if (tp0 + it >= ntup) break;
    const int h = heads[it];
    // V^T[d][key] (lane holds V[key 16 blk + fr][d = 32 ks + 8 g + e]); the previous tuple's reads of vt
    // were issued earlier by this wave, and a wave's LDS operations complete in order
#pragma unroll
    for (int blk = 0; blk < NB; ++blk)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint4 vv = va[it][blk][ks];
        const uint32_t w4[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          vt[(32 * ks + 8 * g + e) * VLD + 16 * blk + fr] =
              (bf16_t)(e & 1 ? w4[e >> 1] >> 16 : w4[e >> 1] & 0xffffu);
      }
#pragma unroll
    for (int qb = 0; qb < NB; ++qb) {
      f32x4_t st[NB];
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
        st[kb] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          st[kb] = mfma16x16x32(*reinterpret_cast<const bf16x8_t*>(&ka[it][kb][ks]),
                                *reinterpret_cast<const bf16x8_t*>(&qa[it][qb][ks]), st[kb]);
      }
      // softmax over the keys of query 16 qb + fr: keys 16 kb + 4 g + i here, the rest in lanes fr + 16 k
      float sc[NB][4], mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sc[kb][i] = (16 * kb + 4 * g + i < p.F) ? st[kb][i] * c : -INFINITY;
          mx = fmaxf(mx, sc[kb][i]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float sum = 0.0f;
      short4_t pb[NB];
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
        float pr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pr[i] = __builtin_amdgcn_exp2f(sc[kb][i] - mx);
          sum += pr[i];
        }
        // P^T as the B operand: element j = key 16 kb + 4 g + j of query 16 qb + fr
        pb[kb] = __builtin_bit_cast(short4_t, make_uint2(pack2(pr[0], pr[1]), pack2(pr[2], pr[3])));
      }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      const float inv = 1.0f / sum;
      bf16_t* orow = (bf16_t*)p.o + rows[it][qb] * p.ldo + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        f32x4_t o = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int kb = 0; kb < NB; ++kb) {
          const short4_t a = *reinterpret_cast<const short4_t*>(&vt[(16 * dt + fr) * VLD + 16 * kb + 4 * g]);
          o = mfma16x16x16_s4(a, pb[kb], o);
        }
        // o[i] = O[query 16 qb + fr][d = 16 dt + 4 g + i]
        if (fok[qb])
          *reinterpret_cast<uint2*>(orow + 16 * dt) =
              make_uint2(pack2(o[0] * inv, o[1] * inv), pack2(o[2] * inv, o[3] * inv));
      }
    }
  }
}

extern "C" int acth_temporal_attn(const ActhTemporalAttnDesc* d, hipStream_t stream) {
  // no work (the other sizes in range): nothing read
  if (d && d->B >= 0 && d->S >= 0 && d->H >= 0 && d->F > 0 && d->F <= 32 && (d->B == 0 || d->S == 0 || d->H == 0))
    return ACTH_OK;
  if (!d || !d->qkv || !d->o) return ACTH_EINVAL;
  if (d->F <= 0 || d->F > 32 || d->B <= 0 || d->S <= 0 || d->H <= 0) return ACTH_EINVAL;
  if (d->ldqkv % 8 || d->ldo % 8) return ACTH_EINVAL;
  const long long ntup = (long long)d->B * d->S * d->H;
  if (d->F <= 16) {
    const long long nblk = (ntup + 4 * TM_TPW - 1) / (4 * TM_TPW);
    if (nblk > 0x7fffffffLL) return ACTH_EINVAL;
    hipLaunchKernelGGL((temporal_attn_mfma_kernel<1, TM_TPW>), dim3((unsigned)nblk), dim3(256), 0, stream, *d);
  } else {
    const long long nblk = (ntup + 3) / 4;
    if (nblk > 0x7fffffffLL) return ACTH_EINVAL;
    hipLaunchKernelGGL((temporal_attn_mfma_kernel<2, 1>), dim3((unsigned)nblk), dim3(256), 0, stream, *d);
  }
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

// ------------------------------------------------------------------------------------------
// IP-adapter cross attention, combined pre-projection output:
//   out[m, :] = vbase[ctx, :] + sa * ma[s] * softmax(q_h K_h^T * scale) V_h  (32-key audio tokens)
//             + sb * mb[s] * vb[ctx, :]                                     (1-key VASA token)
// ctx = m / rows_per_ctx (frame for spatial blocks, batch for temporal blocks), s = m % S.
// kv rows: ctx*nkeys + key, K in columns [0, C), V in [C, 2C).

__global__ __launch_bounds__(256) void ip_attn_kernel(const ActhIpAttnDesc p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = blockIdx.y * 4 + wave;
  const long long m = (long long)blockIdx.x * 64 + lane;
  if (h >= p.H || m >= p.M) return;
  const int C = p.H * 64;
  const long long ctx = m / p.rows_per_ctx;
  const int s = (int)(m % p.S);

  float acc[64];
  {
    const bf16_t* vrow = (const bf16_t*)p.vbase + ctx * p.ldvbase + h * 64;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) unpack8(*reinterpret_cast<const uint4*>(vrow + cc * 8), acc + cc * 8);
  }
  if (p.vb) {
    const float w = p.sb * (p.mask_b ? p.mask_b[s] : 1.0f);
    const bf16_t* vrow = (const bf16_t*)p.vb + ctx * p.ldvb + h * 64;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      float t[8];
      unpack8(*reinterpret_cast<const uint4*>(vrow + cc * 8), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[cc * 8 + e] = fmaf(w, t[e], acc[cc * 8 + e]);
    }
  }
  if (p.kv) {
    float qv[64];
    const bf16_t* qrow = (const bf16_t*)p.q + m * p.ldq + h * 64;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) unpack8(*reinterpret_cast<const uint4*>(qrow + cc * 8), qv + cc * 8);
    const bf16_t* kbase = (const bf16_t*)p.kv + ctx * p.nkeys * (long long)p.ldkv + h * 64;
    float sc[32];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      float a = -INFINITY;
      if (j < p.nkeys) {
        a = 0.0f;
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
          float kf[8];
          unpack8(*reinterpret_cast<const uint4*>(kbase + (size_t)j * p.ldkv + cc * 8), kf);
#pragma unroll
          for (int e = 0; e < 8; ++e) a = fmaf(qv[cc * 8 + e], kf[e], a);
        }
        a *= p.scale;
      }
      sc[j] = a;
      mx = fmaxf(mx, a);
    }
    float den = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) { const float e = j < p.nkeys ? __expf(sc[j] - mx) : 0.0f; sc[j] = e; den += e; }
    const float w0 = p.sa * (p.mask_a ? p.mask_a[s] : 1.0f) / den;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (j < p.nkeys) {
        const float w = w0 * sc[j];
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
          float vf[8];
          unpack8(*reinterpret_cast<const uint4*>(kbase + (size_t)j * p.ldkv + C + cc * 8), vf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[cc * 8 + e] = fmaf(w, vf[e], acc[cc * 8 + e]);
        }
      }
    }
  }
  bf16_t* orow = (bf16_t*)p.out + m * p.ldo + h * 64;
#pragma unroll
  for (int cc = 0; cc < 8; ++cc) *reinterpret_cast<uint4*>(orow + cc * 8) = pack8(acc + cc * 8);
}

extern "C" int acth_ip_attn(const ActhIpAttnDesc* d, hipStream_t stream) {
  // no work (the other sizes in range): nothing read
  if (d && d->M == 0 && d->H >= 0 && d->S >= 0 && d->rows_per_ctx >= 0) return ACTH_OK;
  if (!d || !d->vbase || !d->out) return ACTH_EINVAL;
  if (d->kv && (!d->q || d->nkeys <= 0 || d->nkeys > 32 || d->ldkv % 8 || d->ldq % 8)) return ACTH_EINVAL;
  if (d->M <= 0 || d->H <= 0 || d->rows_per_ctx <= 0 || d->S <= 0) return ACTH_EINVAL;
  if (d->ldvbase % 8 || d->ldo % 8 || (d->vb && d->ldvb % 8)) return ACTH_EINVAL;
  if (d->kv) {
    // the 32-key audio attention is a batched flash attention (one batch per context, one 64-key
    // tile with keys >= nkeys masked) whose epilogue adds the ID value, the masked/scaled audio
    // term and the VASA value
    if (d->M % d->rows_per_ctx || d->rows_per_ctx % d->S) return ACTH_EINVAL;
    const int C = d->H * 64;
    ActhAttnDesc a = {};
    a.q = d->q; a.k = d->kv; a.v = (const bf16_t*)d->kv + C; a.o = d->out;
    a.ldq = d->ldq; a.ldk = a.ldv = d->ldkv; a.ldo = d->ldo;
    a.bsq = (long long)d->rows_per_ctx * d->ldq;
    a.bsk = a.bsv = (long long)d->nkeys * d->ldkv;
    a.bso = (long long)d->rows_per_ctx * d->ldo;
    a.nbatch = d->M / d->rows_per_ctx; a.nheads = d->H; a.Sq = d->rows_per_ctx; a.Skv = d->nkeys;
    a.scale = d->scale;
    if (a.nbatch > 65535 || d->H > 65535 || d->ldo % 4) return ACTH_EINVAL;
    FaIpEpi ep;
    ep.vbase = (const bf16_t*)d->vbase; ep.ldvbase = d->ldvbase;
    ep.vb = (const bf16_t*)d->vb; ep.ldvb = d->ldvb;
    ep.ma = d->mask_a; ep.mb = d->mask_b; ep.sa = d->sa; ep.sb = d->sb; ep.S = d->S;
    const long long kb = ((long long)(d->nkeys - 1) * d->ldkv + 64) * 2;
    if (FA_M16 && a.Sq >= 2048) {
      dim3 grid((a.Sq + 255) / 256, a.nheads, a.nbatch);
      hipLaunchKernelGGL((flash16_kernel<8, true>), grid, dim3(512), 0, stream, a, (unsigned)kb, (unsigned)kb, ep);
    } else if (FA_M16) {
      dim3 grid((a.Sq + 127) / 128, a.nheads, a.nbatch);
      hipLaunchKernelGGL((flash16_kernel<4, true>), grid, dim3(256), 0, stream, a, (unsigned)kb, (unsigned)kb, ep);
    } else if (a.Sq >= 2048) {
      dim3 grid((a.Sq + 255) / 256, a.nheads, a.nbatch);
      hipLaunchKernelGGL((flash_attn_kernel<8, true>), grid, dim3(512), 0, stream, a, (unsigned)kb, (unsigned)kb, ep);
    } else {
      dim3 grid((a.Sq + 127) / 128, a.nheads, a.nbatch);
      hipLaunchKernelGGL((flash_attn_kernel<4, true>), grid, dim3(256), 0, stream, a, (unsigned)kb, (unsigned)kb, ep);
    }
    ACTH_CHECK_LAUNCH();
    return ACTH_OK;
  }
  const long long nblk = ((long long)d->M + 63) / 64;
  if (nblk > 0x7fffffffLL) return ACTH_EINVAL;
  dim3 grid((unsigned)nblk, (d->H + 3) / 4);
  hipLaunchKernelGGL(ip_attn_kernel, grid, dim3(256), 0, stream, *d);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
