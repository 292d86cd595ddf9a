// bf16 MFMA GEMM, 256x256 tile, 8 waves, 4-phase-per-K-tile interleaved schedule (gfx950).
//
// Same operands, loaders and fused epilogues as gemm.hip / gemm256.hip (gemm_common.h); this is
// the main-loop schedule of the CDNA4 "8-phase" GEMM template (cdna_hip_programming.md §5,
// T2+T3+T4+T5): each 64-deep K tile is split into 4 phases, one per quadrant of the 256x256 block
// tile; in a phase every wave computes its 64x32 share of that quadrant (4x2 fragments x 2 k-steps
// = 16 v_mfma_f32_16x16x32_bf16), so a phase needs only one A half-tile (128 rows) and one B
// half-tile (128 columns). Quadrant order (0,0) (0,1) (1,1) (1,0) means fragments are re-read only
// when their half changes (12, 4, 8, 4 ds_read_b128 per phase).
//
// Staging: the next K tile's four 16 KB half-tiles are LDS-DMA'd one per phase (2 wave-instructions
// per wave), in the order they are first needed (A0 B0 B1 A1), into the other of two 64 KB buffers,
// and waited for with a counted `s_waitcnt vmcnt(2)` one phase before their first reader, so loads
// stay in flight across barriers (never vmcnt(0) in the loop).
//
// Wave stagger: waves 4-7 run one barrier behind waves 0-3, so on every SIMD (which hosts one wave
// of each half) one wave's ds_read + DMA issue segment overlaps the other's MFMA segment. Hazards
// under the stagger (one barrier = half a phase): a half-tile is read >= one phase after the last
// wait that retires it; a buffer is re-staged >= two phases after its last read.
#include <type_traits>

#include "gemm_common.h"

using namespace gemm;

// 3x3-conv K order: tap-major (K index tap * Cin + c). Two L2-reuse orders were measured and dropped: the
// 64-channel slice outer / tap inner (level-0 conv 951 -> 881 TFLOP/s, profiles/r3_step31_conv_order_rejected.log)
// and (ky, slice, kx) (11-20 % slower on every conv shape, profiles/r5_conv_korder_rejected.log): re-deriving
// the rows' tap offsets every K tile costs more than the L2 reuse returns.
// 1: 3x3-conv rows (no upsample) carry their tap-(0, 0) pixel and a 9-bit in-image tap mask
#ifndef G8_RING_STAMPS
#define G8_RING_STAMPS 0      // 1: diagnostic build, per-wave segment cycle sums of the ring loop (tile bit 0x400)
#endif
#ifndef G8_TAP_MASK
#define G8_TAP_MASK 1
#endif

namespace {

// A row's source coordinates packed into two registers (four rows per wave stay live across the whole
// K loop; the unpacked RowInfo + row index form made the conv instantiation spill 12 VGPRs, and the
// scratch reloads at every tap change waited out the in-flight LDS-DMA with them):
//   amode 0: a = row (-1 past M);  amode 1: a = (y << 16) | x, b = image (-1 past M);
//   amode 2: a = row (-1 past M), b = frame.
struct RowPk { int a, b; };

template <int AMODE>
__device__ __forceinline__ RowPk pack_row(const ActhGemmDesc& p, int m) {
  const RowInfo ri = row_info(p, m);
  RowPk r;
  if (AMODE == 1 && G8_TAP_MASK && !p.upsample) {
    // a = input pixel index of tap (0, 0) (may be negative), b = 9-bit mask of the taps inside the image
    // (-1 past M): a tap's pixel is then a + (tap / 3) W + tap % 3, one add and a bit test per row
    const int iy0 = ri.y * p.conv_stride - 1, ix0 = ri.x * p.conv_stride - 1;
    int mask = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = iy0 + t / 3, ix = ix0 + t % 3;
      if (iy >= 0 && ix >= 0 && iy < p.H && ix < p.W) mask |= 1 << t;
    }
    r.a = (ri.b * p.H + iy0) * p.W + ix0;
    r.b = ri.ok ? mask : -1;
  } else if (AMODE == 1) {
    r.a = (ri.y << 16) | ri.x;
    r.b = ri.ok ? ri.b : -1;
  } else {
    r.a = ri.ok ? m : -1;
    r.b = ri.y;
  }
  return r;
}

template <int AMODE>
__device__ __forceinline__ int tap_pixel8(const ActhGemmDesc& p, const RowPk& rin, int tap) {
  // opaque copies: without them LICM hoists y*stride / b*H products of all four rows out of the K
  // loop, which is what pushed the conv instantiation past 256 VGPRs
  RowPk r = rin;
  asm volatile("" : "+v"(r.a), "+v"(r.b));
  if (AMODE == 0) return r.a;
  if (AMODE == 1 && G8_TAP_MASK && !p.upsample) {
    if (r.b < 0 || !((r.b >> tap) & 1)) return -1;
    const int ky = tap / 3;
    return r.a + ky * p.W + (tap - 3 * ky);
  }
  if (AMODE == 1) {
    if (r.b < 0) return -1;
    const int y = r.a >> 16, x = r.a & 0xffff;
    const int ky = tap / 3, kx = tap - ky * 3;
    int iy, ix;
    if (p.upsample) {
      iy = y + ky - 1; ix = x + kx - 1;
      if (iy < 0 || ix < 0 || iy >= 2 * p.H || ix >= 2 * p.W) return -1;
      iy >>= 1; ix >>= 1;
    } else {
      iy = y * p.conv_stride + ky - 1; ix = x * p.conv_stride + kx - 1;
      if (iy < 0 || ix < 0 || iy >= p.H || ix >= p.W) return -1;
    }
    return (r.b * p.H + iy) * p.W + ix;
  }
  if (r.a < 0) return -1;
  const int f = r.b + tap - 1;
  if (f < 0 || f >= p.F) return -1;
  return r.a + (tap - 1) * p.S;
}

// In-kernel phase stamps (tile bit 0x400, diagnostics only): s_memtime at kernel entry, after the
// prologue wait, after the main loop and at the end of the epilogue, per workgroup
// (tools/gemm_stamps.py reads them back through acth_debug_gemm_stamps).
#define STAMP_WGS 16384
__device__ unsigned long long g_gemm_stamps[STAMP_WGS * 4];

#ifndef G8_TR_ALL
#define G8_TR_ALL 0           // 0: transposed product for the GEGLU launches only; 1: every launch, with the TR fast
                              // epilogue; 2: the launches without a residual / mix operand. Measured (same box,
                              // profiles/r3_step26_*): 1 loses 7-10 % on residual GEMMs (8-byte fragment loads of the
                              // residual) and +1 % per step; 2 gains 3-8 % on residual-free K = 320 shapes in
                              // isolation but is within noise per step (360.3-361.0 vs 360.3-360.6 ms)
#endif

#define BAR() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); \
                   __builtin_amdgcn_sched_barrier(0); } while (0)

}  // namespace

// BN_ = 256: waves 2 (rows) x 4 (cols), a wave's quadrant share is 64 x 32 (4 x 2 fragments);
// BN_ = 320 (the C = 320 projections and convs, one tile spans N): waves 4 x 2, share 32 x 80
// (2 x 5 fragments), B half-tiles of 160 rows (20 DMA pieces: waves 0-3 issue 3, waves 4-7 two).
// TR: the MFMAs compute the transposed product (B fragment as the A operand), so a lane's accumulator holds
// four consecutive columns of one row (used by the GEGLU launches, whose gated outputs then leave straight from
// registers); TR = false keeps four consecutive rows of one column, which the slab-based epilogues write out
// marginally faster (the convs measured 2-5 % slower transposed, profiles/r3_step24_*).
// RING: the main loop as a 4-slot ring of 32-deep sub-tiles (see the ring branch below) instead of the
// 4-phase-per-64-deep-K-tile schedule; same LDS bytes, same epilogue.
template <int BN_, int AMODE, bool TR = false, bool RING = true>
__global__ __launch_bounds__(512, 2) void gemm8p_kernel(const ActhGemmDesc p, unsigned a_bytes, unsigned a2_bytes,
                                                        unsigned b_bytes, int vec_ok) {
  constexpr int WR = BN_ == 256 ? 2 : 4, WC = 8 / WR;
  constexpr int TMQ = 128 / WR / 16, TNQ = BN_ / 2 / WC / 16;   // fragments per wave and quadrant
  constexpr int AH = 128 * 128;                 // A half-tile: 128 rows x 64 k
  constexpr int BH = BN_ / 2 * 128;             // B half-tile: BN/2 rows x 64 k
  constexpr int BUF = 2 * AH + 2 * BH;          // A0 A1 B0 B1
  constexpr int NBP = BN_ / 16;                 // DMA pieces per B half-tile
  constexpr int NBJ = (NBP + 7) / 8;
  static_assert(TMQ * WR * 16 == 128 && TNQ * WC * 16 == BN_ / 2, "quadrant split");
  static_assert(2 * BUF + 5 * BN_ * 4 <= 160 * 1024, "LDS");
  // epilogue bias / row-bias (temb) rows of this tile, staged once at kernel start so the epilogue
  // issues no global load after its first store (vmcnt counts stores too: a load waited for after
  // a store waits for that store's round trip). They live in the SAME __shared__ array as the
  // staging buffers, past them: a second __shared__ object makes hipcc emit vmcnt(0) before every
  // phase's ds_reads (it cannot rule out the in-flight LDS-DMA writing it), which drains the
  // counted-vmcnt pipeline (cdna_hip_programming.md §5, "Projection GEMM" item 4(a)).
  constexpr int RB_IMG = 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + (1 + RB_IMG) * BN_ * 4];
  float* const sbias = reinterpret_cast<float*>(smem + 2 * BUF);
  float* const srb = sbias + BN_;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave % WR, wc = wave / WR;     // wave's row / column slot inside a quadrant
  const bool stamps = (p.tile & 0x400) != 0;
  const int stamp_wg = blockIdx.x + gridDim.x * blockIdx.y;
  const bool rt = (p.tile & 0x800) != 0;          // stamps from the 100 MHz real-time counter (chip-wide timeline)
  auto stamp = [&](int k) {
    if (!G8_RING_STAMPS && stamps && tid == 0 && stamp_wg < STAMP_WGS)
      g_gemm_stamps[stamp_wg * 4 + k] = rt ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const bool late = wave >= 4;                  // staggered half
  // B-half DMA pieces this wave issues (wave + 8u < NBP): the count differs by wave when NBP % 8
  const int nbw = (NBP - wave + 7) / 8;

  // XCD-aware bijective tile order (n fastest), as gemm.hip
  const int ntn = gridDim.x;
  const int nwg = gridDim.x * gridDim.y;
  const int bid = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  // Optional M-grouped raster (tile bits 16-23 = gm > 1): inside a run, gm row blocks x all N tiles
  // with m fastest, so the ~32 tiles an XCD holds at once share gm A panels and a few B tiles
  // instead of streaming the whole B (> 4 MB L2 for the wide GEGLU weights) per row block.
  const int gm = (p.tile >> 16) & 0xff;
  int tn_idx, tm_idx;
  if (gm > 1) {
    const int g = lin / (gm * ntn);
    const int m0 = g * gm;
    const int gcur = min(gm, (int)gridDim.y - m0);
    const int r = lin - g * gm * ntn;
    tn_idx = r / gcur;
    tm_idx = m0 + (r - tn_idx * gcur);
  } else {
    tn_idx = lin % ntn;
    tm_idx = lin / ntn;
  }
  const int tile_n = tn_idx * BN_;
  const int tile_m = tm_idx * 256;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t ra2 = make_rsrc(p.A2 ? p.A2 : p.A, p.A2 ? a2_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);
  const bool two_src = p.A2 != nullptr;
  const int cin = AMODE == 0 ? 0x7fffffff : p.Cin;
  const int fr = lane & 15, fq = lane >> 4;        // fragment row / K chunk of this lane (MFMA layout)

  f32x4_t acc[2][2][TMQ][TNQ];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < TMQ; ++i)
#pragma unroll
        for (int j = 0; j < TNQ; ++j) acc[a][b][i][j] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};

  // the epilogue's bias and row-bias (temb) rows, loaded in the prologue beside the first DMA
  int rb_img0 = 0, rb_nimg = 0;
  if (p.rowbias) {
    rb_img0 = udiv22(tile_m, p.rb_div);
    rb_nimg = udiv22(min(p.M, tile_m + 256) - 1, p.rb_div) - rb_img0 + 1;
  }
  const bool rb_lds = rb_nimg <= RB_IMG;
  auto stage_bias = [&]() {
    for (int i = tid; i < BN_; i += 512) {
      const int col = tile_n + i;
      sbias[i] = (p.bias && col < p.N) ? p.bias[col] : 0.0f;
    }
    if (p.rowbias && rb_lds) {
      for (int i = tid; i < rb_nimg * BN_; i += 512) {
        const int im = i / BN_, c = i - im * BN_, col = tile_n + c;
        srb[i] = col < p.N ? p.rowbias[(size_t)(rb_img0 + im) * p.ldrb + col] : 0.0f;
      }
    }
  };

  if constexpr (RING) {
    // ---- Ring main loop. K is walked in 32-deep sub-tiles (256 A rows + BN_ B rows, 64 B each: SLOT bytes)
    // through four LDS slots: in the segment that reads sub-tile s from slot s % 4, sub-tile s + 2 is
    // LDS-DMA'd into slot (s + 2) % 4. One MFMA segment per sub-tile -- a wave's whole 4 TMQ TNQ fragment
    // block (32 MFMAs at 256x256, 40 at 256x320) from 2 TMQ + 2 TNQ ds_read_b128 -- so two barriers per 32
    // deep where the 4-phase loop below has four; that loop's MFMA pipe sat idle ~35 % of its main loop
    // (SQ_VALU_MFMA_BUSY_CYCLES 62 % at 8192^3, in-kernel stamps 3170 cycles per 64-deep K tile against
    // 2048 of MFMA issue), i.e. ~140 cycles per barrier.
    // Stagger as in the 4-phase loop: waves 4-7 run one barrier behind, so each SIMD alternates one wave's
    // read + DMA segment with the other's MFMA segment. Hazards (physical barrier k = k-th s_barrier; the
    // early waves read sub-tile s in segment 2s + 1 and multiply it in 2s + 2, the late waves one segment
    // later): slot (s + 2) % 4 last held sub-tile s - 2, whose late reads retired inside their MFMA segment
    // 2s - 1, i.e. by barrier 2s, before any wave stages s + 2 (segment >= 2s + 1); sub-tile s + 1 is
    // retired by every issuer before barrier 2s + 3 (early waves: after MFMA(s); late waves: after
    // staging s + 2), the barrier its first reader (early, segment 2s + 3) passes.
    constexpr int SLOT = (256 + BN_) * 64;
    constexpr int NBP16 = BN_ / 16, NBJ16 = (NBP16 + 7) / 8;
    static_assert(4 * SLOT == 2 * BUF, "the ring takes the 4-phase loop's LDS bytes");
    // DMA wave-instructions a wave issues per sub-tile: 2 A pieces + its share of the B pieces (waves 0-3 take
    // the odd ones: uniform per wave half, so each half's wait count is a constant)
    constexpr int PW_E = 2 + (NBP16 + 7) / 8, PW_L = 2 + (NBP16 + 3) / 8;
    // DMA piece = 16 rows x 64 B; lane -> row lane / 4 of the piece, physical 16-B chunk lane % 4 holding
    // logical K chunk (lane % 4) ^ S[lane / 16], S = {0, 2, 3, 1} (= S[(row / 4) & 3]): a fragment read
    // (row lane % 16, chunk lane / 16) then covers 16 distinct 16-B bank slots in every ds_read_b128 lane group
    const int lrow = lane >> 2;
    const int cch = (lane & 3) ^ ((0x78 >> (2 * (lane >> 4))) & 3);
    RowPk rp[2];
    unsigned aoff[2], aoff2[2], boff[NBJ16];
#pragma unroll
    for (int u = 0; u < 2; ++u) rp[u] = pack_row<AMODE>(p, tile_m + (wave + 8 * u) * 16 + lrow);
#pragma unroll
    for (int u = 0; u < NBJ16; ++u) {
      const int brow = tile_n + (wave + 8 * u) * 16 + lrow;
      boff[u] = brow < p.N ? ((unsigned)brow * p.ldb + cch * 8) * 2u : OOB;
    }
    auto set_tap = [&](int tap) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int pix = tap_pixel8<AMODE>(p, rp[u], tap);
        aoff[u] = pix < 0 ? OOB : ((unsigned)pix * p.lda + cch * 8) * 2u;
        aoff2[u] = pix < 0 ? OOB : ((unsigned)pix * p.lda2 + cch * 8) * 2u;
      }
    };
    set_tap(0);
    const int ns = (p.K + 31) / 32, nfull = p.K / 32;
    // staging state of the next sub-tile to stage, advanced by prep() in K order (tap-major conv K order:
    // K index tap * Cin + c, the tap's pixel offsets re-derived when c wraps)
    // (tap-major conv K order; the 32-channel-slice-outer order, whose nine taps of a slice read one ~4-row window in
    // consecutive sub-tiles, measured 6-16 % slower on every conv shape on the ring too: profiles/r6_cslice_ab.log)
    int s_tap = 0, s_c0 = 0, k_c0 = 0, k_k0 = 0, k_kb = 0;
    bool k_second = false, k_tail = false;
    auto prep = [&](int st) {
      k_k0 = st * 32;
      k_kb = k_k0;
      if (AMODE == 0) {
        k_c0 = k_k0;
      } else {
        if (s_c0 == 0 && s_tap > 0) set_tap(s_tap);
        k_c0 = s_c0;
        s_c0 += 32;
        if (s_c0 == cin) { s_c0 = 0; ++s_tap; }
      }
      k_second = two_src && k_c0 >= p.K1;
      k_tail = st >= nfull;
    };
    // The K advance rides in the DMA's scalar offset (not range-checked; the per-lane voffset is, and carries
    // OOB for rows outside the operand), so a piece costs no VALU: only the last sub-tile of a K that is not a
    // multiple of 32 takes the per-lane tail test.
    auto stage = [&](int slot) {
      char* dst0 = smem + slot * SLOT;
      const bool dead = k_tail && k_k0 + cch * 8 >= p.K;   // this lane's chunk lies past K (last sub-tile only)
      const int soa = k_second ? (k_c0 - p.K1) * 2 : k_c0 * 2, sob = k_kb * 2;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        unsigned off = k_second ? aoff2[u] : aoff[u];
        if (dead) off = OOB;
        lds_void* dst = (lds_void*)(dst0 + (wave + 8 * u) * 1024);
        if (k_second) __builtin_amdgcn_raw_ptr_buffer_load_lds(ra2, dst, 16, off, soa, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, dst, 16, off, soa, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < NBJ16; ++u) {
        if (NBP16 % 8 == 0 || wave + 8 * u < NBP16) {
          unsigned off = boff[u];
          if (dead) off = OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst0 + 256 * 64 + (wave + 8 * u) * 1024), 16, off,
                                                   sob, 0, 0);
        }
      }
    };
    // fragment t of a 16-row block: row 16 t + lane % 16, logical chunk lane / 16 at its swizzled slot
    const int frag = fr * 64 + ((fq ^ ((0x78 >> (2 * (fr >> 2))) & 3)) << 4);
    const int a_base = (wr * TMQ * 16) * 64 + frag;
    const int b_base = 256 * 64 + (wc * TNQ * 16) * 64 + frag;
    bf16x8_t af[2][TMQ], bfr[2][TNQ];
    auto read = [&](int slot) {
      const char* s = smem + slot * SLOT;
      auto ra_ = [&](int qm) {
#pragma unroll
        for (int i = 0; i < TMQ; ++i)
          af[qm][i] = *reinterpret_cast<const bf16x8_t*>(s + a_base + qm * 128 * 64 + i * 1024);
      };
      auto rb_ = [&](int qn) {
#pragma unroll
        for (int j = 0; j < TNQ; ++j)
          bfr[qn][j] = *reinterpret_cast<const bf16x8_t*>(s + b_base + qn * (BN_ / 2) * 64 + j * 1024);
      };
      ra_(0); rb_(0); rb_(1); ra_(1);                  // in the order the quadrants below consume them
    };
    auto mma = [&]() {
      constexpr int QM[4] = {0, 0, 1, 1}, QN[4] = {0, 1, 1, 0};
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < TMQ; ++i)
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            f32x4_t& c = acc[QM[q]][QN[q]][i][j];
            c = TR ? mfma16x16x32(bfr[QN[q]][j], af[QM[q]][i], c) : mfma16x16x32(af[QM[q]][i], bfr[QN[q]][j], c);
          }
      __builtin_amdgcn_s_setprio(0);
    };
    // retire sub-tile s + 1: everything but this wave's s + 2 pieces (when staged)
    auto wait_next = [&](bool more, auto pw_c) {
      if (!more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(pw_c)::value) : "memory");
    };

    // prologue: sub-tiles 0 and 1 staged and landed
    prep(0);
    stage(0);
    if (ns > 1) {
      prep(1);
      stage(1);
    }
    stage_bias();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    BAR();
    stamp(1);
    if (late) BAR();
#if G8_RING_STAMPS
    // diagnostic build only: per-wave cycle sums of the four segments of a ring iteration (read + DMA issue,
    // first barrier, MFMA, second barrier), s_memtime with lgkmcnt(0) (so ds_read latency counts as read time)
    unsigned long long sg[4] = {0, 0, 0, 0}, tprev = 0;
    auto tick = [&]() {
      unsigned long long t;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
      __builtin_amdgcn_sched_barrier(0);
      return t;
    };
    tprev = tick();
#endif
    for (int st = 0; st < ns; ++st) {
      const bool more = st + 2 < ns;
#if G8_RING_STAMPS
      const unsigned long long t0 = tick();
      if (st) sg[3] += t0 - tprev;
#endif
      if (!(p.tile & 0x8000)) read(st & 3);          // diagnostic 0x8000: no fragment reads (wrong output)
      if (more && !(p.tile & 0x4000)) {                 // diagnostic 0x4000: no DMA in the loop (wrong output)
        prep(st + 2);
        stage((st + 2) & 3);
      }
      if (late) wait_next(more, std::integral_constant<int, PW_L>{});
#if G8_RING_STAMPS
      const unsigned long long t1 = tick();
      sg[0] += t1 - t0;
#endif
      BAR();
#if G8_RING_STAMPS
      const unsigned long long t2 = tick();
      sg[1] += t2 - t1;
#endif
      mma();
      if (!late) wait_next(more, std::integral_constant<int, PW_E>{});
#if G8_RING_STAMPS
      tprev = tick();
      sg[2] += tprev - t2;
#endif
      BAR();
    }
#if G8_RING_STAMPS
    if (stamps && lane == 0 && stamp_wg < 512)
      for (int k = 0; k < 4; ++k) g_gemm_stamps[(stamp_wg * 8 + wave) * 4 + k] = sg[k];
#endif
    if (!late) BAR();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    BAR();
  } else {
    // DMA: half-tile piece i (0..15) = rows [8i, 8i+8); wave w issues pieces w and w + 8.
    // Lane -> (row 8i + lane/8, physical 16-B slot lane%8) holding logical K chunk slot ^ (row & 7).
    const int lrow = lane >> 3;
    const int cch = (lane & 7) ^ lrow;
    // rows [h][u]: half h, piece w + 8u
    RowPk rp[2][2];
    unsigned aoff[2][2], aoff2[2][2], boff[2][NBJ];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        rp[h][u] = pack_row<AMODE>(p, tile_m + h * 128 + (wave + 8 * u) * 8 + lrow);
      }
#pragma unroll
      for (int u = 0; u < NBJ; ++u) {
        const int brow = tile_n + h * (BN_ / 2) + (wave + 8 * u) * 8 + lrow;
        boff[h][u] = brow < p.N ? ((unsigned)brow * p.ldb + cch * 8) * 2u : OOB;
      }
    }
    auto set_tap = [&](int tap) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int pix = tap_pixel8<AMODE>(p, rp[h][u], tap);
          aoff[h][u] = pix < 0 ? OOB : ((unsigned)pix * p.lda + cch * 8) * 2u;
          aoff2[h][u] = pix < 0 ? OOB : ((unsigned)pix * p.lda2 + cch * 8) * 2u;
        }
    };
    set_tap(0);
    const int nk = (p.K + 63) / 64;
    const int kfull = p.K / 64;

    // per-K-tile staging parameters, advanced by prep_k() in K order
    int s_tap = 0, s_c0 = 0;
    int k_c0 = 0, k_k0 = 0, k_kb = 0;
    bool k_second = false, k_tail = false;
    auto prep_k = [&](int kt) {
      k_k0 = kt * 64;
      k_kb = k_k0;
      if (AMODE == 0) {
        k_c0 = k_k0;
      } else {
        if (s_c0 == 0 && s_tap > 0) set_tap(s_tap);
        k_c0 = s_c0;
        s_c0 += 64;
        if (s_c0 == cin) { s_c0 = 0; ++s_tap; }
      }
      k_second = two_src && k_c0 >= p.K1;
      k_tail = kt >= kfull;
    };
    auto stage_a = [&](int h, int buf) {
      char* dst0 = smem + buf * BUF + h * AH;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        unsigned off = k_second ? aoff2[h][u] + (unsigned)(k_c0 - p.K1) * 2u : aoff[h][u] + (unsigned)k_c0 * 2u;
        if (k_tail && k_k0 + cch * 8 >= p.K) off = OOB;
        lds_void* dst = (lds_void*)(dst0 + (wave + 8 * u) * 1024);
        if (k_second) __builtin_amdgcn_raw_ptr_buffer_load_lds(ra2, dst, 16, off, 0, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, dst, 16, off, 0, 0, 0);
      }
    };
    auto stage_b = [&](int h, int buf) {
      char* dst0 = smem + buf * BUF + 2 * AH + h * BH;
#pragma unroll
      for (int u = 0; u < NBJ; ++u) {
        if (NBP % 8 == 0 || wave + 8 * u < NBP) {
          unsigned off = boff[h][u] + (unsigned)k_kb * 2u;
          if (k_tail && k_k0 + cch * 8 >= p.K) off = OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst0 + (wave + 8 * u) * 1024), 16, off, 0, 0, 0);
        }
      }
    };

    // fragment reads: row base + 16 t + lane%16, swizzle key row & 7 == lane & 7
    const int fkey = lane & 7;
    const int sw0 = ((0 + fq) ^ fkey) << 4, sw1 = ((4 + fq) ^ fkey) << 4;
    const int a_row = (wr * TMQ * 16 + fr) * 128;   // inside an A half
    const int b_row = (wc * TNQ * 16 + fr) * 128;   // inside a B half

    bf16x8_t af[TMQ][2], bfr[TNQ][2];

    auto read_a = [&](int buf, int h) {
      const char* s = smem + buf * BUF + h * AH + a_row;
#pragma unroll
      for (int i = 0; i < TMQ; ++i) {
        af[i][0] = *reinterpret_cast<const bf16x8_t*>(s + i * 2048 + sw0);
        af[i][1] = *reinterpret_cast<const bf16x8_t*>(s + i * 2048 + sw1);
      }
    };
    auto read_b = [&](int buf, int h) {
      const char* s = smem + buf * BUF + 2 * AH + h * BH + b_row;
#pragma unroll
      for (int j = 0; j < TNQ; ++j) {
        bfr[j][0] = *reinterpret_cast<const bf16x8_t*>(s + j * 2048 + sw0);
        bfr[j][1] = *reinterpret_cast<const bf16x8_t*>(s + j * 2048 + sw1);
      }
    };
    auto mma = [&](f32x4_t (&c)[TMQ][TNQ]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < TMQ; ++i)
#pragma unroll
          for (int j = 0; j < TNQ; ++j)
            c[i][j] = TR ? mfma16x16x32(bfr[j][s], af[i][s], c[i][j])
                         : mfma16x16x32(af[i][s], bfr[j][s], c[i][j]);
      __builtin_amdgcn_s_setprio(0);
    };

    // prologue: K tile 0 fully staged and landed
    prep_k(0);
    stage_a(0, 0); stage_b(0, 0); stage_b(1, 0); stage_a(1, 0);
    stage_bias();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    BAR();
    stamp(1);
    if (late) BAR();

    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1, nxt = cur ^ 1;
      const bool more = kt + 1 < nk;
      if (more) prep_k(kt + 1);
      // phase 0: quadrant (0,0); stage A0(k+1)
      read_a(cur, 0); read_b(cur, 0);
      if (more) stage_a(0, nxt);
      BAR();
      mma(acc[0][0]);
      // A1(k) is read in phase 2: retire it now (DMA'd in the previous tile's phase 3)
      if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      BAR();
      // phase 1: quadrant (0,1); stage B0(k+1)
      read_b(cur, 1);
      if (more) stage_b(0, nxt);
      BAR();
      mma(acc[0][1]);
      BAR();
      // phase 2: quadrant (1,1); stage B1(k+1)
      read_a(cur, 1);
      if (more) stage_b(1, nxt);
      BAR();
      mma(acc[1][1]);
      // A0(k+1), B0(k+1) are read in the next tile's phase 0: retire everything but this wave's B1(k+1)
      // pieces (nbw: 3 / 2 for the 256x320 tile's two wave halves, 2 at 256x256, 1 at 256x128)
      if (nbw >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (nbw == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (nbw == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      BAR();
      // phase 3: quadrant (1,0); stage A1(k+1)
      read_b(cur, 0);
      if (more) stage_a(1, nxt);
      BAR();
      mma(acc[1][0]);
      // B1(k+1) is read in the next tile's phase 1
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      BAR();
    }
    if (!late) BAR();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    BAR();

  }
  stamp(2);

  if (p.tile & 0x100) {                          // diagnostic: main loop only (keeps acc live)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < TMQ; ++i)
#pragma unroll
          for (int j = 0; j < TNQ; ++j) asm volatile("" ::"v"(acc[a][b][i][j]));
    return;
  }
  // ---- epilogue: per quadrant, the wave's (16 TMQ) x (16 TNQ) accumulators -> private LDS slab ->
  // 8-column row chunks (16-byte coalesced epilogue loads / stores). (Storing straight from the
  // fragments, 8 bytes per lane across 16 rows, measured up to 1.7x slower on the small-K shapes.)
  // Bias / row bias come from LDS (staged at kernel start): a global load waited for after a store
  // waits for that store too (vmcnt counts both, in order), which made every chunk pay a store
  // round trip. Measured split of the 256x320 tile at K = 320 (tools/bench_gemm.py diagnostics):
  // main loop 53 %, slab 2 %, chunk math 16 %, stores 29 % of the kernel.
  constexpr int SR = TMQ * 16, SC = TNQ * 16, EPI_LD = SC + 4, CPR = SC / 8;
  static_assert(8 * SR * EPI_LD * 4 <= 2 * BUF, "epilogue slabs");
  float* et = reinterpret_cast<float*>(smem) + wave * (SR * EPI_LD);
  const bool geglu = p.act == 2;
  // c[i][j][r] = C[row 16 i + 4 fq + r][col 16 j + fr] (TR: C[row 16 i + fr][col 16 j + 4 fq + r], four
  // consecutive columns: one ds_write_b128)
  auto slab = [&](const f32x4_t (&c)[TMQ][TNQ]) {
#pragma unroll
    for (int i = 0; i < TMQ; ++i)
#pragma unroll
      for (int j = 0; j < TNQ; ++j) {
        if constexpr (TR) {
          *reinterpret_cast<f32x4_t*>(&et[(i * 16 + fr) * EPI_LD + j * 16 + 4 * fq]) = c[i][j];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) et[(i * 16 + fq * 4 + r) * EPI_LD + j * 16 + fr] = c[i][j][r];
        }
      }
  };
  // GEGLU straight from the accumulators (BN_ = 256: a wave's 32 columns are one (hidden 16 | gate 16) granule
  // pair, so c[i][0][r] and c[i][1][r] are the hidden and gate values of the same output column 4 fq + r): the
  // gated outputs of fragment rows 2p and 2p + 1 are widened to 8 columns per lane by v_permlane16_swap (as the
  // fast epilogue) and stored 16 bytes at a time; no LDS slab.
  const bool geglu_direct = TR && geglu && BN_ == 256 && !p.out_f32 && p.orow_div >= p.M && vec_ok && !p.rmap &&
                            (p.N & 31) == 0;
  if (geglu_direct) {
    if constexpr (TR && BN_ == 256) {
      const int gl = fq & 1, gh = fq >> 1;
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        const int qm = qi >> 1, qn = qi & 1;
        const f32x4_t (&c)[TMQ][TNQ] = acc[qm][qn];
        const int lc0 = qn * (BN_ / 2) + wc * SC;
        const float4 bh = *reinterpret_cast<const float4*>(&sbias[lc0 + 4 * fq]);
        const float4 bg = *reinterpret_cast<const float4*>(&sbias[lc0 + 16 + 4 * fq]);
        const float bhv[4] = {bh.x, bh.y, bh.z, bh.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
        const int ocol = (tile_n + lc0) / 2 + 8 * gh;
#pragma unroll
        for (int pp = 0; pp < TMQ / 2; ++pp) {
          float o[2][4];
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
              const float2_pk gg = GEGLU_GELU((float2_pk){fmaf(c[2 * pp + h2][1][r], p.alpha, bgv[r]),
                                                          fmaf(c[2 * pp + h2][1][r + 1], p.alpha, bgv[r + 1])});
              o[h2][r] = fmaf(c[2 * pp + h2][0][r], p.alpha, bhv[r]) * gg.x;
              o[h2][r + 1] = fmaf(c[2 * pp + h2][0][r + 1], p.alpha, bhv[r + 1]) * gg.y;
            }
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(o[0][r]), __float_as_uint(o[1][r]), false, false);
            v[r] = __uint_as_float(sw[0]);
            v[4 + r] = __uint_as_float(sw[1]);
          }
          const int row = tile_m + qm * 128 + wr * SR + 16 * (2 * pp + gl) + fr;
          if (row < p.M && ocol < p.N / 2)
            *reinterpret_cast<uint4*>((bf16_t*)p.C + (size_t)(row + p.orow_off) * p.ldc + ocol) = pack8(v);
        }
      }
    }
  } else if (geglu) {
    // BN_ = 256: one (hidden 16 | gate 16) granule pair -> 16 outputs: SR rows x 2 chunks per quadrant
    constexpr int NCH = SR * 2 / 64;
    static_assert(SR * 2 % 64 == 0, "GEGLU chunks per lane");
    auto flush_g = [&](int qm, int qn, const f32x4_t (&c)[TMQ][TNQ]) {
      const int row0 = tile_m + qm * 128 + wr * SR;
      const int lc0 = qn * (BN_ / 2) + wc * SC;            // tile-local first column
      const int col0 = tile_n + lc0;
      slab(c);
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int ch = lane + 64 * u;
        const int r = ch >> 1, oc = (ch & 1) * 8;
        if (row0 + r < p.M && col0 < p.N) {
          float h[8], gt[8], v[8];
          const float* hs = &et[r * EPI_LD + oc];
          const float* gs = &et[r * EPI_LD + 16 + oc];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            h[e] = hs[e] * p.alpha + sbias[lc0 + oc + e];
            gt[e] = gs[e] * p.alpha + sbias[lc0 + 16 + oc + e];
          }
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const float2_pk gg = GEGLU_GELU((float2_pk){gt[e], gt[e + 1]});
            v[e] = h[e] * gg.x;
            v[e + 1] = h[e + 1] * gg.y;
          }
          store8(p, out_row(p, row0 + r), col0 / 2 + oc, v, true, vec_ok);
        }
      }
    };
    flush_g(0, 0, acc[0][0]);
    flush_g(0, 1, acc[0][1]);
    flush_g(1, 0, acc[1][0]);
    flush_g(1, 1, acc[1][1]);
  } else {
    auto flush = [&](int qm, int qn) {
      const int row0 = tile_m + qm * 128 + wr * SR;
      const int lc0 = qn * (BN_ / 2) + wc * SC;
      const int col0 = tile_n + lc0;
      // the residual chunk is loaded one chunk ahead (software pipelined across iterations), so its
      // HBM latency overlaps the previous chunk's math and store instead of stalling it
      uint4 rnext = make_uint4(0, 0, 0, 0);
      auto pre = [&](int chx) {
        const int rx = chx / CPR, cx = (chx - rx * CPR) * 8;
        rnext = epi_load_r(p, row0 + rx, col0 + cx, vec_ok && row0 + rx < p.M);
      };
      if (p.R) pre(lane);
#pragma unroll 1
      for (int ch = lane; ch < SR * CPR; ch += 64) {
        const int r = ch / CPR, c8 = (ch - r * CPR) * 8;
        const int row = row0 + r, ocol = col0 + c8;
        EpiPre e;
        e.r = rnext;
        if (p.R && ch + 64 < SR * CPR) pre(ch + 64);
        if (p.MIX) e.mix = epi_load_mix(p, row, ocol, vec_ok && row < p.M);
        if (row < p.M && ocol < p.N) {
          float v[8];
          const float4 x0 = *reinterpret_cast<const float4*>(&et[r * EPI_LD + c8]);
          const float4 x1 = *reinterpret_cast<const float4*>(&et[r * EPI_LD + c8 + 4]);
          const float4 b0 = *reinterpret_cast<const float4*>(&sbias[lc0 + c8]);
          const float4 b1 = *reinterpret_cast<const float4*>(&sbias[lc0 + c8 + 4]);
          v[0] = fmaf(x0.x, p.alpha, b0.x); v[1] = fmaf(x0.y, p.alpha, b0.y);
          v[2] = fmaf(x0.z, p.alpha, b0.z); v[3] = fmaf(x0.w, p.alpha, b0.w);
          v[4] = fmaf(x1.x, p.alpha, b1.x); v[5] = fmaf(x1.y, p.alpha, b1.y);
          v[6] = fmaf(x1.z, p.alpha, b1.z); v[7] = fmaf(x1.w, p.alpha, b1.w);
          if (p.rowbias) {
            if (rb_lds) {
              const float* rs = &srb[(udiv22(row, p.rb_div) - rb_img0) * BN_ + lc0 + c8];
#pragma unroll
              for (int k = 0; k < 8; ++k) v[k] += rs[k];
            } else {
              const float* rb2 = p.rowbias + (size_t)udiv22(row, p.rb_div) * p.ldrb + ocol;
              add8(v, rb2, ocol + 8 <= p.N && !((size_t)rb2 & 15), p.N - ocol);
            }
          }
          epilogue8_tail(p, row, ocol, v, vec_ok, e);
        }
      }
    };
    // Fast path for the UNet's residual-stream / conv epilogues (no activation, bf16 out, identity row
    // map, 16-byte aligned rows, whole 8-column chunks, residual without a row map, row bias staged in
    // LDS; the slab transposes the accumulators so one store instruction writes whole 128-byte row
    // segments: a register-direct variant, widened to 16 B per lane by v_permlane16_swap like the GEGLU path
    // above, wrote 32-byte row pieces per instruction and measured 9-12 % slower on the K = 320 shapes,
    // profiles/r3_step24_bench_gemm_epilogue_variants.log): the combination of bias / row bias / residual / mix is a compile-time choice, so the chunk
    // loop is branch-free, and each lane keeps one 8-column chunk across the quadrant's rows (its bias
    // chunk in registers, row-strided pointers) instead of re-deriving 64-bit addresses per chunk.
    // Measured with tools/gemm_stamps.py: the generic loop spent ~29k cycles per 256x320 tile.
    const bool fast = p.act == 0 && !p.out_f32 && (p.orow_div >= p.M || p.orow_div % SR == 0) && vec_ok &&
                      (p.N & 7) == 0 && !p.rmap && (!p.rowbias || rb_lds);
    auto fast_epilogue = [&](auto res_c, auto mix_c, auto rb_c) {
      constexpr bool RES = decltype(res_c)::value, MIXB = decltype(mix_c)::value, RB = decltype(rb_c)::value;
      constexpr int RPI = 64 / CPR, LPI = RPI * CPR, NIT = (SR + RPI - 1) / RPI;
      // residual double-buffered across quadrants; with a mix operand too the registers allow one buffer
      constexpr int NRB = (RES && !MIXB) ? 2 : 1, NMB = MIXB ? 1 : 0;
      const int r0 = lane / CPR, c8 = (lane - r0 * CPR) * 8;
      const bool lane_ok = lane < LPI;
      const size_t step_c = (size_t)RPI * p.ldc, step_r = (size_t)RPI * p.ldr, step_m = (size_t)RPI * p.ldmix;
      auto q_col = [&](int qn) { return tile_n + qn * (BN_ / 2) + wc * SC + c8; };
      auto q_row = [&](int qm) { return tile_m + qm * 128 + wr * SR + r0; };
      auto ld_ok = [&](int rowf, int col, int it) {
        return lane_ok && col < p.N && r0 + it * RPI < SR && rowf + it * RPI < p.M;
      };
      // a quadrant's residual (mix) chunks for every iteration, issued together: the residual of the
      // next quadrant is in flight while this one is processed (the chunk loop was HBM-latency bound
      // with one chunk of look-ahead: ~49k cycles per tile). Invalid (row, column) slots read the
      // tensor's first chunk instead (never used), so the loads are unconditional.
      uint4 rbuf[NRB][NIT], mbuf[NMB > 0 ? NMB : 1][NIT];
      auto load_res = [&](int qm, int qn, uint4 (&dst)[NIT]) {
        const int rowf = q_row(qm), col = q_col(qn);
        const bf16_t* rp = (const bf16_t*)p.R + (size_t)rowf * p.ldr + col;
#pragma unroll
        for (int it = 0; it < NIT; ++it)
          dst[it] = *reinterpret_cast<const uint4*>(ld_ok(rowf, col, it) ? rp + it * step_r : (const bf16_t*)p.R);
      };
      auto load_mix = [&](int qm, int qn, uint4 (&dst)[NIT]) {
        const int rowf = q_row(qm), col = q_col(qn);
        const bf16_t* mp = (const bf16_t*)p.MIX + (size_t)rowf * p.ldmix + col;
#pragma unroll
        for (int it = 0; it < NIT; ++it)
          dst[it] = *reinterpret_cast<const uint4*>(ld_ok(rowf, col, it) ? mp + it * step_m : (const bf16_t*)p.MIX);
      };
      auto one = [&](int qm, int qn, const uint4 (&rq)[NIT], const uint4 (&mq)[NIT]) {
        const int lc0 = qn * (BN_ / 2) + wc * SC;
        const int col = q_col(qn), rowf = q_row(qm);
        const float4 b0 = *reinterpret_cast<const float4*>(&sbias[lc0 + c8]);
        const float4 b1 = *reinterpret_cast<const float4*>(&sbias[lc0 + c8 + 4]);
        // output rows through the remap (in_proj's xz rows into the scan sequence): a wave's SR rows lie in one
        // remap group (fast requires orow_div % SR == 0), so one division per quadrant
        bf16_t* cp = (bf16_t*)p.C + (out_row(p, rowf - r0) + r0) * p.ldc + col;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
          const int r = r0 + it * RPI;
          const int rr = r < SR ? r : 0;
          const float4 x0 = *reinterpret_cast<const float4*>(&et[rr * EPI_LD + c8]);
          const float4 x1 = *reinterpret_cast<const float4*>(&et[rr * EPI_LD + c8 + 4]);
          float v[8];
          v[0] = fmaf(x0.x, p.alpha, b0.x); v[1] = fmaf(x0.y, p.alpha, b0.y);
          v[2] = fmaf(x0.z, p.alpha, b0.z); v[3] = fmaf(x0.w, p.alpha, b0.w);
          v[4] = fmaf(x1.x, p.alpha, b1.x); v[5] = fmaf(x1.y, p.alpha, b1.y);
          v[6] = fmaf(x1.z, p.alpha, b1.z); v[7] = fmaf(x1.w, p.alpha, b1.w);
          if (RB) {
            const int row = rowf + it * RPI;
            const int img = min(max(udiv22(row < p.M ? row : p.M - 1, p.rb_div) - rb_img0, 0), RB_IMG - 1);
            const float4 q0 = *reinterpret_cast<const float4*>(&srb[img * BN_ + lc0 + c8]);
            const float4 q1 = *reinterpret_cast<const float4*>(&srb[img * BN_ + lc0 + c8 + 4]);
            v[0] += q0.x; v[1] += q0.y; v[2] += q0.z; v[3] += q0.w;
            v[4] += q1.x; v[5] += q1.y; v[6] += q1.z; v[7] += q1.w;
          }
          if (RES) {
            float t[8];
            unpack8(rq[it], t);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += t[e];
          }
          if (MIXB) {
            float t[8];
            unpack8(mq[it], t);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = p.mix_alpha * t[e] + (1.0f - p.mix_alpha) * v[e];
          }
          if (ld_ok(rowf, col, it)) *reinterpret_cast<uint4*>(cp + it * step_c) = pack8(v);
        }
      };
      constexpr int QM[4] = {0, 0, 1, 1}, QN[4] = {0, 1, 0, 1};
      if (RES && NRB == 2) load_res(0, 0, rbuf[0]);
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        if (RES && NRB == 2 && qi + 1 < 4) load_res(QM[qi + 1], QN[qi + 1], rbuf[(qi + 1) % NRB]);
        if (RES && NRB == 1) load_res(QM[qi], QN[qi], rbuf[0]);
        if (MIXB) load_mix(QM[qi], QN[qi], mbuf[0]);
        slab(acc[QM[qi]][QN[qi]]);
        one(QM[qi], QN[qi], rbuf[qi % NRB], mbuf[0]);
      }
    };
    // TR form of the fast path: the whole epilogue (alpha, bias, row bias, residual, mix) runs in fp32 on the
    // accumulators themselves (residual / mix fetched in the accumulator layout, 8 bytes per lane and
    // fragment), rounds once to bf16 and goes through a bf16 slab: half the LDS bytes of the fp32 slab,
    // ds_write_b64 instead of four ds_write_b32, and the store phase is a plain 16-byte copy.
    auto fast_epilogue_tr = [&](auto res_c, auto mix_c, auto rb_c) {
      constexpr bool RES = decltype(res_c)::value, MIXB = decltype(mix_c)::value, RB = decltype(rb_c)::value;
      constexpr int NF = TMQ * TNQ, EHL = SC + 8;               // bf16 slab row: SC + 16 B pad
      constexpr int RPI = 64 / CPR, LPI = RPI * CPR, NIT = (SR + RPI - 1) / RPI;
      constexpr int NRB = (RES && !MIXB) ? 2 : 1;
      bf16_t* const eh = reinterpret_cast<bf16_t*>(et);
      auto f_row = [&](int qm, int i) { return tile_m + qm * 128 + wr * SR + 16 * i + fr; };
      auto f_col = [&](int qn, int j) { return tile_n + qn * (BN_ / 2) + wc * SC + 16 * j + 4 * fq; };
      uint2 rbuf[NRB][NF], mbuf[NF];   // mbuf unused (and dropped) without a mix operand
      // invalid (row, column) slots read the tensor's first element pair instead: loads stay unconditional
      auto load_f = [&](const void* base, int ld, int qm, int qn, uint2 (&dst)[NF]) {
#pragma unroll
        for (int i = 0; i < TMQ; ++i)
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            const int row = f_row(qm, i), col = f_col(qn, j);
            const bool ok = row < p.M && col < p.N;
            dst[i * TNQ + j] = *reinterpret_cast<const uint2*>((const bf16_t*)base + (ok ? (size_t)row * ld + col : 0));
          }
      };
      auto to_slab = [&](int qm, int qn, const f32x4_t (&c)[TMQ][TNQ], const uint2 (&rq)[NF], const uint2 (&mq)[NF]) {
        const int lc0 = qn * (BN_ / 2) + wc * SC;
#pragma unroll
        for (int i = 0; i < TMQ; ++i) {
          int img = 0;
          if (RB) {
            const int row = f_row(qm, i);
            img = min(max(udiv22(row < p.M ? row : p.M - 1, p.rb_div) - rb_img0, 0), RB_IMG - 1);
          }
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            const int lc = lc0 + 16 * j + 4 * fq;
            const float4 b = *reinterpret_cast<const float4*>(&sbias[lc]);
            float v[4] = {fmaf(c[i][j][0], p.alpha, b.x), fmaf(c[i][j][1], p.alpha, b.y),
                          fmaf(c[i][j][2], p.alpha, b.z), fmaf(c[i][j][3], p.alpha, b.w)};
            if (RB) {
              const float4 q = *reinterpret_cast<const float4*>(&srb[img * BN_ + lc]);
              v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
            }
            if (RES) {
              const uint2 t = rq[i * TNQ + j];
              v[0] += lo16f(t.x); v[1] += hi16f(t.x);
              v[2] += lo16f(t.y); v[3] += hi16f(t.y);
            }
            if (MIXB) {
              const uint2 t = mq[i * TNQ + j];
              const float m4[4] = {lo16f(t.x), hi16f(t.x),
                                   lo16f(t.y), hi16f(t.y)};
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = p.mix_alpha * m4[e] + (1.0f - p.mix_alpha) * v[e];
            }
            *reinterpret_cast<uint2*>(&eh[(16 * i + fr) * EHL + 16 * j + 4 * fq]) =
                make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          }
        }
      };
      const int r0 = lane / CPR, c8 = (lane - r0 * CPR) * 8;
      auto from_slab = [&](int qm, int qn) {
        const int rowf = tile_m + qm * 128 + wr * SR + r0, col = tile_n + qn * (BN_ / 2) + wc * SC + c8;
        bf16_t* cp = (bf16_t*)p.C + (out_row(p, rowf - r0) + r0) * p.ldc + col;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
          const int r = r0 + it * RPI;
          if (lane < LPI && r < SR && rowf + it * RPI < p.M && col < p.N)
            *reinterpret_cast<uint4*>(cp + (size_t)it * RPI * p.ldc) = *reinterpret_cast<const uint4*>(&eh[r * EHL + c8]);
        }
      };
      constexpr int QM[4] = {0, 0, 1, 1}, QN[4] = {0, 1, 0, 1};
      if (RES && NRB == 2) load_f(p.R, p.ldr, 0, 0, rbuf[0]);
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        if (RES && NRB == 2 && qi + 1 < 4) load_f(p.R, p.ldr, QM[qi + 1], QN[qi + 1], rbuf[(qi + 1) % NRB]);
        if (RES && NRB == 1) load_f(p.R, p.ldr, QM[qi], QN[qi], rbuf[0]);
        if (MIXB) load_f(p.MIX, p.ldmix, QM[qi], QN[qi], mbuf);
        to_slab(QM[qi], QN[qi], acc[QM[qi]][QN[qi]], rbuf[qi % NRB], mbuf);
        from_slab(QM[qi], QN[qi]);     // wave-private slab: LDS ops of one wave complete in order
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (fast && TR) {
      const int sel = (p.R ? 1 : 0) | (p.MIX ? 2 : 0) | (p.rowbias ? 4 : 0);
      switch (sel) {
        case 0: fast_epilogue_tr(F_{}, F_{}, F_{}); break;
        case 1: fast_epilogue_tr(T_{}, F_{}, F_{}); break;
        case 3: fast_epilogue_tr(T_{}, T_{}, F_{}); break;
        case 4: fast_epilogue_tr(F_{}, F_{}, T_{}); break;
        case 5: fast_epilogue_tr(T_{}, F_{}, T_{}); break;
        default:
          slab(acc[0][0]); flush(0, 0);
          slab(acc[0][1]); flush(0, 1);
          slab(acc[1][0]); flush(1, 0);
          slab(acc[1][1]); flush(1, 1);
      }
    } else if (fast) {
      const int sel = (p.R ? 1 : 0) | (p.MIX ? 2 : 0) | (p.rowbias ? 4 : 0);
      switch (sel) {
        case 0: fast_epilogue(F_{}, F_{}, F_{}); break;
        case 1: fast_epilogue(T_{}, F_{}, F_{}); break;
        case 3: fast_epilogue(T_{}, T_{}, F_{}); break;
        case 4: fast_epilogue(F_{}, F_{}, T_{}); break;
        default:
          slab(acc[0][0]); flush(0, 0);
          slab(acc[0][1]); flush(0, 1);
          slab(acc[1][0]); flush(1, 0);
          slab(acc[1][1]); flush(1, 1);
      }
    } else {
      slab(acc[0][0]); flush(0, 0);
      slab(acc[0][1]); flush(0, 1);
      slab(acc[1][0]); flush(1, 0);
      slab(acc[1][1]); flush(1, 1);
    }
  }
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(3);
  }
}

extern "C" int acth_debug_gemm_stamps(unsigned long long* host_dst, int n_wgs) {
  if (!host_dst || n_wgs <= 0 || n_wgs > STAMP_WGS) return ACTH_EINVAL;
  if (hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_gemm_stamps), (size_t)n_wgs * 4 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return ACTH_ELAUNCH;
  return ACTH_OK;
}

template <int BN_, bool RING>
static void launch8p_(const ActhGemmDesc* d, dim3 grid, unsigned a_bytes, unsigned a2_bytes, unsigned b_bytes,
                      int vec_ok, hipStream_t stream) {
  if constexpr (BN_ == 256) {
    if (d->act == 2 && d->amode == 0) {     // GEGLU: gated outputs straight from the transposed accumulators
      hipLaunchKernelGGL((gemm8p_kernel<256, 0, true, RING>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes,
                         b_bytes, vec_ok);
      return;
    }
  }
  if constexpr (G8_TR_ALL != 0) {
    if (G8_TR_ALL == 1 || (!d->R && !d->MIX)) {
      if (d->amode == 1)
        hipLaunchKernelGGL((gemm8p_kernel<BN_, 1, true, RING>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes,
                           b_bytes, vec_ok);
      else if (d->amode == 2)
        hipLaunchKernelGGL((gemm8p_kernel<BN_, 2, true, RING>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes,
                           b_bytes, vec_ok);
      else
        hipLaunchKernelGGL((gemm8p_kernel<BN_, 0, true, RING>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes,
                           b_bytes, vec_ok);
      return;
    }
  }
  if (d->amode == 1)
    hipLaunchKernelGGL((gemm8p_kernel<BN_, 1, false, RING>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes,
                       b_bytes, vec_ok);
  else if (d->amode == 2)
    hipLaunchKernelGGL((gemm8p_kernel<BN_, 2, false, RING>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes,
                       b_bytes, vec_ok);
  else
    hipLaunchKernelGGL((gemm8p_kernel<BN_, 0, false, RING>), grid, dim3(512), 0, stream, *d, a_bytes, a2_bytes,
                       b_bytes, vec_ok);
}

// Main-loop choice: the ring for the 3x3 convs (+6-11 % on the UNet conv shapes, tools/ab_gemm.py,
// profiles/r6_ring_ab.log), the 4-phase loop elsewhere (dense shapes within -6..+8 %, the small-K projections
// slower on the ring). Tile bit 0x1000 forces the ring, 0x2000 the 4-phase loop (A/B in one process).
template <int BN_>
static void launch8p(const ActhGemmDesc* d, dim3 grid, unsigned a_bytes, unsigned a2_bytes, unsigned b_bytes,
                     int vec_ok, hipStream_t stream) {
  const bool ring = (d->tile & 0x1000) || (!(d->tile & 0x2000) && d->amode == 1);
  if (ring) launch8p_<BN_, true>(d, grid, a_bytes, a2_bytes, b_bytes, vec_ok, stream);
  else launch8p_<BN_, false>(d, grid, a_bytes, a2_bytes, b_bytes, vec_ok, stream);
}

// Row-block group of the M-grouped raster: explicit in tile bits 16-23 (bench / tests), else
// 8 for B operands larger than an XCD's 4 MB L2 and 0 (plain n-fastest runs) otherwise.
static int gemm8p_group_m(const ActhGemmDesc* d) {
  const int g = (d->tile >> 16) & 0xff;
  if (g) return g;
  // measured (tools/bench_gemm.py --flags): gm = 8 lifts the level-1 / level-2 GEGLU shapes
  // (B = 6.5 / 26 MB) 3.8 / 4.6 % and the level-1 conv (7.4 MB) 1.6 %; L2-resident B: +-1 % noise
  return (long long)d->N * d->K * 2 > (4ll << 20) ? 8 : 0;
}

// tile 4: 256 x 256; tile 5: 256 x 320; tile 6: 256 x 128 (the tall-skinny Mamba x_proj: N = 104 on
// 776916 rows, HBM-bound on A); tile 7: 256 x 64 (the UNet conv_out, N = 4: a quarter of tile 6's
// padded MFMA work). Tiles 5-7: no GEGLU (wave column shares are not granule pairs).
int gemm8p_launch(const ActhGemmDesc* d, int tile, unsigned a_bytes, unsigned a2_bytes, unsigned b_bytes,
                  int vec_ok, hipStream_t stream) {
  const int mt = (d->M + 255) / 256;
  if (mt > 65535) return ACTH_EINVAL;
  ActhGemmDesc dd = *d;
  dd.tile = (d->tile & 0xffff) | (gemm8p_group_m(d) << 16);
  if (tile == 4) {
    launch8p<256>(&dd, dim3((d->N + 255) / 256, mt), a_bytes, a2_bytes, b_bytes, vec_ok, stream);
  } else if (tile == 5 && d->act != 2) {
    launch8p<320>(&dd, dim3((d->N + 319) / 320, mt), a_bytes, a2_bytes, b_bytes, vec_ok, stream);
  } else if (tile == 6 && d->act != 2) {
    launch8p<128>(&dd, dim3((d->N + 127) / 128, mt), a_bytes, a2_bytes, b_bytes, vec_ok, stream);
  } else if (tile == 7 && d->act != 2) {
    launch8p<64>(&dd, dim3((d->N + 63) / 64, mt), a_bytes, a2_bytes, b_bytes, vec_ok, stream);
  } else {
    return ACTH_EINVAL;
  }
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
