// bf16 MFMA GEMM with implicit-conv A loaders and fused epilogues (gfx950).
//
// C[M,N] = epilogue( A[M,K] . B[N,K]^T )
//   * B is a weight matrix stored like nn.Linear.weight: (N, K) row-major, bf16.
//   * A is produced by one of three loaders (all NHWC / token-major activations):
//       dense     : A[m, k] = src[m*lda + k]                      (nn.Linear, 1x1 conv)
//       conv3x3   : A[m, (ky*3+kx)*Cin + c] = img[b, y*s+ky-1, x*s+kx-1, c]   (ResBlock convs,
//                   Downsample2D with s=2, Upsample2D with a nearest-x2 source remap)
//       temporal3 : A[m, kf*Cin + c] = x[(b,f+kf-1,s), c]          (Conv3d kernel (3,1,1))
//     each loader can read its K range from two tensors (channel concat of UNet skips).
//   * epilogue: alpha*acc + bias[n] + rowbias[row/rb_div, n] + R[rmap(row), n],
//     optional SiLU / GELU / GEGLU (h * gelu(g) on interleaved 16-column granules),
//     optional AlphaBlender mix with a second tensor, fp32 or bf16 output, row remap.
//
// Structure: 128x128x64 workgroup tile, 4 waves (2x2), each wave 64x64 = 2x2 tiles of
// v_mfma_f32_32x32x16_bf16. Operands move HBM/L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds):
// each wave-instruction fills 1 KiB = 8 tile rows x 128 B; the per-lane SOURCE address carries the
// im2col / concat / upsample remapping and an XOR swizzle (chunk ^ (row & 7)) so the MFMA fragment
// reads (ds_read_b128, 16 rows per lane group) spread over the bank row; lanes whose element is
// outside the tensor (conv zero padding, M/N/K tails) get an offset past the buffer's num_records
// and the hardware range check returns zeros. Two LDS stages: the next K tile's DMA is in flight
// while the current one feeds the MFMAs. The epilogue transposes the accumulators through LDS so
// every thread owns 8 consecutive columns of a row: bias / residual / mix loads and the output
// store are 16-byte and fully coalesced.
#include "gemm_common.h"

#define BM 128
#define BN 128
#define BKT 64
#define STAGE_BYTES (2 * BM * BKT * 2)        // A + B tile, bf16
#define EPI_LD 132                            // fp32 row stride of the epilogue tile
#define SMEM_BYTES (BM * EPI_LD * 4)          // >= 2 * STAGE_BYTES


using namespace gemm;

__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(const ActhGemmDesc p, unsigned a_bytes,
                                                           unsigned a2_bytes, unsigned b_bytes, int vec_ok) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  // readfirstlane: the wave id is uniform, and proving it keeps the LDS-DMA destination (M0)
  // scalar; otherwise hipcc wraps every DMA in a waterfall loop
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: dispatch deals block ids round-robin over the 8 XCDs, so block b and
  // b + 8 share an L2. Give each XCD a contiguous run of (m, n) tiles (n fastest) so the N tiles that
  // share an A panel are read from one L2 (bijective for any grid size).
  const int ntn = gridDim.x;
  const int nwg = gridDim.x * gridDim.y;
  const int bid = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int tile_n = (lin % ntn) * BN;
  const int tile_m = (lin / ntn) * BM;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t ra2 = make_rsrc(p.A2 ? p.A2 : p.A, p.A2 ? a2_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);

  // this lane's DMA slots: instruction j of wave w fills tile rows [32w + 8j, +8), lane -> (row, slot)
  const int lrow = lane >> 3;                // 0..7
  const int pchunk = lane & 7;               // physical 16-B slot in the 128-B LDS row
  RowInfo ri[4];
  int arow[4], brow[4], cchunk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = wave * 32 + j * 8 + lrow;  // tile row 0..127
    cchunk[j] = pchunk ^ (r & 7);            // logical K chunk this lane fetches
    arow[j] = tile_m + r;
    brow[j] = tile_n + r;
    ri[j] = row_info(p, arow[j]);
  }

  const int nk = (p.K + BKT - 1) / BKT;

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BKT;
    char* sA = smem + buf * STAGE_BYTES;
    char* sB = sA + BM * BKT * 2;
    // A2 (skip-connection half of a channel concat) holds K columns [K1, K): one source per K tile
    const bool second = second_source(p, k0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + cchunk[j] * 8;
      const unsigned off = a_offset(p, arow[j], ri[j], k0, k, second);
      lds_void* dst = (lds_void*)(sA + (wave * 32 + j * 8) * 128);
      if (second) __builtin_amdgcn_raw_ptr_buffer_load_lds(ra2, dst, 16, off, 0, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, dst, 16, off, 0, 0, 0);
      const unsigned boff = (brow[j] < p.N && k < p.K) ? ((unsigned)brow[j] * p.ldb + k) * 2u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(sB + (wave * 32 + j * 8) * 128), 16, boff, 0, 0, 0);
    }
  };

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int r32 = lane & 31, hh = lane >> 5;
  // fragment rows read by this lane and their swizzle keys
  const int ar0 = wm * 64 + r32, ar1 = ar0 + 32;
  const int br0 = wn * 64 + r32, br1 = br0 + 32;

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* sA = smem + cur * STAGE_BYTES;
    const char* sB = sA + BM * BKT * 2;
#pragma unroll
    for (int kk = 0; kk < BKT / 16; ++kk) {
      const int c = kk * 2 + hh;
      const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(sA + ar0 * 128 + ((c ^ (ar0 & 7)) << 4));
      const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(sA + ar1 * 128 + ((c ^ (ar1 & 7)) << 4));
      const bf16x8_t b0 = *reinterpret_cast<const bf16x8_t*>(sB + br0 * 128 + ((c ^ (br0 & 7)) << 4));
      const bf16x8_t b1 = *reinterpret_cast<const bf16x8_t*>(sB + br1 * 128 + ((c ^ (br1 & 7)) << 4));
      acc[0][0] = mfma32x32x16(a0, b0, acc[0][0]);
      acc[0][1] = mfma32x32x16(a0, b1, acc[0][1]);
      acc[1][0] = mfma32x32x16(a1, b0, acc[1][0]);
      acc[1][1] = mfma32x32x16(a1, b1, acc[1][1]);
    }
    // next tile landed (this wave's DMAs) and every wave is done reading `cur`
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur ^= 1;
  }

  // ---------------- epilogue: accumulators -> LDS (fp32 [128][EPI_LD]) -> row-contiguous ----------
  float* et = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const int col = wn * 64 + j * 32 + r32;
        et[row * EPI_LD + col] = acc[i][j][r];
      }
  __syncthreads();

  const bool geglu = p.act == 2;
  // each thread: 8 consecutive output columns of a row; 16 (or 8 for GEGLU) threads per row
  const int tpr = geglu ? 8 : 16;
  const int rows_per_pass = 256 / tpr;
  const int cg = tid % tpr;
  for (int r0 = tid / tpr; r0 < BM; r0 += rows_per_pass) {
    const int row = tile_m + r0;
    if (row >= p.M) break;
    if (geglu) {
      // output columns [tile_n/2 + 8cg, +8): hidden at tile col 32g + j, gate at 32g + 16 + j
      const int oc = cg * 8;
      const int hc = 32 * (oc >> 4) + (oc & 15);
      if (tile_n + hc + 16 >= p.N) continue;
      epilogue_geglu8(p, row, tile_n + hc, tile_n + hc + 16, tile_n / 2 + oc, &et[r0 * EPI_LD + hc],
                      &et[r0 * EPI_LD + hc + 16], vec_ok);
    } else {
      const int c0 = cg * 8;
      const int ocol = tile_n + c0;
      if (ocol >= p.N) continue;
      float v[8];
      const float4 x0 = *reinterpret_cast<const float4*>(&et[r0 * EPI_LD + c0]);
      const float4 x1 = *reinterpret_cast<const float4*>(&et[r0 * EPI_LD + c0 + 4]);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      epilogue8(p, row, ocol, v, vec_ok);
    }
  }
}

int gemm256_launch(const ActhGemmDesc* d, int tile, unsigned a_bytes, unsigned a2_bytes, unsigned b_bytes,
                   int vec_ok, hipStream_t stream);
int gemm8p_launch(const ActhGemmDesc* d, int tile, unsigned a_bytes, unsigned a2_bytes, unsigned b_bytes,
                  int vec_ok, hipStream_t stream);

// Tile choice (measured on MI355X, tools/bench_gemm.py, profiles/r2_step3_bench_gemm_tiles.log): the
// phased 256x256 kernel for GEGLU (its wave tiles hold whole hidden|gate granule pairs); otherwise
// whichever phased tile (256x320 or 256x256) wastes less of the machine -- the fraction of its
// columns that are real (N / padded N) times the fraction of its last round of tiles over the CUs
// that is occupied -- provided that is >= 0.7 (e.g. 774144x320: 256x320; 12096x1280 and 4096^2:
// 256x256, +18-60 % over the alternatives); the persistent 256x160 kernel for grids too small for
// either, the 128x128 kernel for small M or N.
static double tile_eff(long long mt, int N, int bn) {
  const long long nt = (N + bn - 1) / bn, t = mt * nt;
  const long long rounds = (t + 255) / 256;
  return (double)N / (double)(nt * bn) * (double)t / (double)(rounds * 256);
}

static int choose_tile(const ActhGemmDesc* d) {
  if (d->tile & 0xff) return d->tile & 0xff;
  // Tall-skinny, HBM-bound on A (>= 128 row tiles; the Mamba x_proj, N = 2 (R + 32) = 104 / 144 / 224,
  // and the UNet conv_out, N = 4): the phased kernels stream A through LDS-DMA whatever the column
  // padding costs. Measured (tools/bench_gemm.py, profiles/r2_step19_bench_gemm_tall_skinny.log):
  // 776916x104x640 311 -> 374 TF/s (256x128), 196308x144x1280 451 -> 516 and 51156x224x2560
  // 382 -> 773 (256x256 instead of 256x160), conv 774144x4x2880 17.7 -> 21.4.
  const bool tall = d->act != 2 && d->M >= 256 * 128;
  if (tall && d->N <= 32) return 7;
  if (tall && d->N < 128) return 6;
  if (d->N < 128 || d->M < 256) return 1;
  const long long mt = (d->M + 255) / 256;
  if (d->act == 2) return (d->N % 256 == 0 && mt * (d->N / 256) >= 192) ? 4 : 1;
  const double e5 = tile_eff(mt, d->N, 320), e4 = tile_eff(mt, d->N, 256);
  if (e5 >= 0.7 && e5 >= e4) return 5;
  if (e4 >= 0.7) return 4;
  if (tall && d->N > 128 && d->N <= 256) return 4;
  return 3;
}

// An A operand past the kernels' 2 GiB buffer extent (32-bit buffer offsets / num_records) runs as
// consecutive launches over row chunks whose A extents fit, the descriptor rebased per chunk: rows
// of C / R / MIX and row-bias images shifted, A (and A2) advanced by the chunk's first source row.
// A chunk is whole units of the A mode -- any rows (dense), whole images (conv: the 3x3 taps stay
// inside an image), whole batch elements (temporal: the frame taps stay inside one) -- whole
// row-bias images and whole output-row-remap groups (orow_div source rows land orow_stride output
// rows apart: a chunk starting at source row m0 = j * orow_div starts its C at output row
// j * orow_stride, orow_off kept). Residual row maps (rmap) are not rebased: such calls keep the
// 2 GiB limit. (The 112-frame mode-2 UNet call at 576x1024 reads 2.7 GB Mamba xz rows through x_proj;
// with every token selected, the in_proj GEMM writes its level-0 xz rows through an orow remap.)
extern "C" int acth_gemm(const ActhGemmDesc* d, hipStream_t stream);

static long long lcm_ll(long long a, long long b) {
  long long g = a, r = b;
  while (r) { const long long t = g % r; g = r; r = t; }
  return a / g * b;
}

static int gemm_split_rows(const ActhGemmDesc* d, hipStream_t stream) {
  if (d->rmap) return ACTH_EINVAL;
  const bool remap = d->orow_div < d->M;
  long long unit_rows = 1, unit_arows = 1;                 // output rows / A rows per indivisible unit
  if (d->amode == 1) { unit_rows = (long long)d->Ho * d->Wo; unit_arows = (long long)d->H * d->W; }
  if (d->amode == 2) { unit_rows = unit_arows = (long long)d->F * d->S; }
  long long need = 1;                                      // output-row multiples a chunk must keep
  if (d->rowbias) need = lcm_ll(need, d->rb_div);
  if (remap) need = lcm_ll(need, d->orow_div);
  {
    const long long lu = lcm_ll(unit_rows, need), mult = lu / unit_rows;
    unit_rows = lu; unit_arows *= mult;
  }
  if (d->M % unit_rows && d->amode != 0) return ACTH_EINVAL;
  const long long lda_max = d->A2 ? (d->lda > d->lda2 ? d->lda : d->lda2) : d->lda;
  const long long units_per_chunk = ((0x7fffffffLL / 2) - 65536) / (unit_arows * lda_max);
  if (units_per_chunk < 1) return ACTH_EINVAL;
  const long long chunk_rows = units_per_chunk * unit_rows, chunk_arows = units_per_chunk * unit_arows;
  const int esz = d->out_f32 ? 4 : 2;
  for (long long m0 = 0, a0 = 0; m0 < d->M; m0 += chunk_rows, a0 += chunk_arows) {
    ActhGemmDesc c = *d;
    const long long mc = (d->M - m0 < chunk_rows) ? d->M - m0 : chunk_rows;
    c.M = (int)mc;
    c.A = (const char*)d->A + a0 * d->lda * 2;
    if (d->A2) c.A2 = (const char*)d->A2 + a0 * d->lda2 * 2;
    const long long crow = remap ? (m0 / d->orow_div) * d->orow_stride : m0;
    c.C = (char*)d->C + crow * d->ldc * esz;
    if (d->R) c.R = (const char*)d->R + m0 * d->ldr * 2;
    if (d->MIX) c.MIX = (const char*)d->MIX + m0 * d->ldmix * 2;
    if (d->rowbias) c.rowbias = d->rowbias + (m0 / d->rb_div) * d->ldrb;
    if (!remap) c.orow_div = c.orow_stride = (int)mc;
    const int rc = acth_gemm(&c, stream);
    if (rc != ACTH_OK) return rc;
  }
  return ACTH_OK;
}

extern "C" int acth_gemm(const ActhGemmDesc* d, hipStream_t stream) {
  if (d && d->M == 0) return ACTH_OK;   // no rows: nothing read or written
  if (!d || !d->A || !d->B || !d->C) return ACTH_EINVAL;
  // rows < 2^22: the epilogues divide row indices with a float-reciprocal estimate (udiv22)
  if (d->M < 0 || d->M >= (1 << 22) || d->N <= 0 || d->K <= 0) return ACTH_EINVAL;
  if (d->M == 0) return ACTH_OK;
  if (d->K % 8 || d->lda % 8 || (d->A2 && (d->lda2 % 8 || d->K1 % 64)) || d->ldb % 8) return ACTH_EINVAL;
  // 16-byte epilogue vectors need 16-byte aligned rows in C / R / MIX; otherwise scalar path
  const int esz = d->out_f32 ? 4 : 2;
  const int vec_ok = ((size_t)d->C % 16 == 0) && ((d->ldc * esz) % 16 == 0) &&
                     (!d->R || ((size_t)d->R % 16 == 0 && d->ldr % 8 == 0)) &&
                     (!d->MIX || ((size_t)d->MIX % 16 == 0 && d->ldmix % 8 == 0));
  if (d->amode != 0 && (d->Cin % BKT || d->K % d->Cin)) return ACTH_EINVAL;
  if (d->amode == 1 && d->K != 9 * d->Cin) return ACTH_EINVAL;
  if (d->amode == 2 && (d->K != 3 * d->Cin || d->F <= 0 || d->S <= 0)) return ACTH_EINVAL;
  if (d->act == 2 && d->N % 32) return ACTH_EINVAL;
  if (d->orow_div <= 0 || (d->rowbias && d->rb_div <= 0) || (d->rmap && (d->r_div <= 0 || d->r_mod <= 0)))
    return ACTH_EINVAL;
  // operand extents (buffer num_records): rows of each A source and of B
  long long a_rows, a2_rows;
  if (d->amode == 1) a_rows = a2_rows = (long long)(d->M / (d->Ho * d->Wo)) * d->H * d->W;
  else a_rows = a2_rows = d->M;
  const int c1 = d->A2 ? d->K1 : (d->amode == 0 ? d->K : d->Cin);
  const long long a_bytes = ((a_rows - 1) * (long long)d->lda + (d->A2 ? c1 : (d->amode == 0 ? d->K : d->Cin))) * 2;
  const long long a2_bytes = d->A2 ? ((a2_rows - 1) * (long long)d->lda2 +
                                      ((d->amode == 0 ? d->K : d->Cin) - c1)) * 2 : 0;
  const long long b_bytes = ((long long)(d->N - 1) * d->ldb + d->K) * 2;
  if (b_bytes >= 0x80000000LL) return ACTH_EINVAL;
  if (a_bytes >= 0x80000000LL || a2_bytes >= 0x80000000LL) return gemm_split_rows(d, stream);
  const int tile = choose_tile(d) & 0xff;
  if (tile >= 4 && tile <= 7)
    return gemm8p_launch(d, tile, (unsigned)a_bytes, (unsigned)a2_bytes, (unsigned)b_bytes, vec_ok, stream);
  if (tile == 2 || tile == 3)
    return gemm256_launch(d, tile, (unsigned)a_bytes, (unsigned)a2_bytes, (unsigned)b_bytes, vec_ok, stream);
  if (tile != 1) return ACTH_EINVAL;
  dim3 grid((d->N + BN - 1) / BN, (d->M + BM - 1) / BM);
  if (grid.y > 65535) return ACTH_EINVAL;
  hipLaunchKernelGGL(gemm_bf16_kernel, grid, dim3(256), 0, stream, *d, (unsigned)a_bytes,
                     (unsigned)a2_bytes, (unsigned)b_bytes, vec_ok);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}

extern "C" int acth_gemm_desc_size(void) { return (int)sizeof(ActhGemmDesc); }
