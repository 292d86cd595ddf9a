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
// Layout: u / delta / y token-major (b*L + l, channels): a wave reads 64 consecutive channels of one
// token (coalesced 128 B). xdbl rows (dt | B | C, fp32) are wave-uniform per token: staged in LDS
// per chunk of T tokens and read back as broadcasts. The next chunk's tiles are prefetched into
// registers while the current chunk is scanned. State and exp(A) constants live in registers.
#include "common.h"

#define SC_T 16
#define SC_THREADS 128
#define SC_WMAX 128   // max R + 2N floats per token and group

template <int RMAX>
__global__ __launch_bounds__(SC_THREADS) void scan_kernel(const ActhScanDesc p) {
  __shared__ __attribute__((aligned(16))) float xs[SC_T * SC_WMAX];
  __shared__ __attribute__((aligned(16))) bf16_t us[SC_T * SC_THREADS];
  __shared__ __attribute__((aligned(16))) float dls[SC_T * SC_THREADS];
  const int k = blockIdx.y, b = blockIdx.z;
  const int t = threadIdx.x;
  const int dbase = blockIdx.x * SC_THREADS;
  const int d = dbase + t;
  const bool active = d < p.D;
  const int dd = active ? d : 0;
  const int W = p.R + 32;
  const bool has_delta = p.delta != nullptr;
  const bool rev = (k == 1) && p.flip1;

  float w[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) w[r] = r < p.R ? p.dt_w[((size_t)k * p.D + dd) * p.R + r] : 0.0f;
  const float bias = p.dt_b ? p.dt_b[k * p.D + dd] : 0.0f;
  float a2[16], h[16];
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    a2[n] = -__expf(p.A_log[((size_t)k * p.D + dd) * 16 + n]) * 1.4426950408889634f;
    h[n] = 0.0f;
  }
  const float dsk = p.Dskip ? p.Dskip[k * p.D + dd] : 0.0f;

  const bf16_t* ub = (const bf16_t*)p.u + (size_t)b * p.L * p.ldu + (size_t)k * p.u_gstride + dbase;
  const float* xb = p.xdbl + (size_t)b * p.L * p.ldx + k * W;
  const size_t dl_off = (size_t)b * p.L * p.ld_delta + (size_t)k * p.D + dbase;
  bf16_t* yb = (p.y1 && k == 1) ? (bf16_t*)p.y1 : (bf16_t*)p.y0 + (size_t)k * p.y_gstride;
  yb += (size_t)b * p.n_keep * p.ldy + dd;

  const int nchunks = (p.L + SC_T - 1) / SC_T;
  const int per_thread = (SC_T * W + SC_THREADS - 1) / SC_THREADS;

  float px[(SC_T * SC_WMAX) / SC_THREADS];
  uint4 pu[2];
  float4 pd[4];

  auto pos_of = [&](int i) { return rev ? p.L - 1 - i : i; };
  auto prefetch = [&](int c) {
#pragma unroll
    for (int e = 0; e < (SC_T * SC_WMAX) / SC_THREADS; ++e) {
      if (e < per_thread) {
        const int idx = t + e * SC_THREADS;
        const int tt = idx / W, col = idx - tt * W;
        const int i = c * SC_T + tt;
        px[e] = (tt < SC_T && i < p.L) ? xb[(size_t)pos_of(i) * p.ldx + col] : 0.0f;
      }
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int idx = t + e * SC_THREADS;          // 256 x 16 B = 16 tokens x 128 channels
      const int tt = idx >> 4, cc = (idx & 15) * 8;
      const int i = c * SC_T + tt;
      pu[e] = (i < p.L && dbase + cc < p.D)
                  ? *reinterpret_cast<const uint4*>(ub + (size_t)pos_of(i) * p.ldu + cc)
                  : make_uint4(0, 0, 0, 0);
    }
    if (has_delta) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = t + e * SC_THREADS;        // 512 x 4 floats = 16 tokens x 128 channels
        const int tt = idx >> 5, cc = (idx & 31) * 4;
        const int i = c * SC_T + tt;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < p.L && dbase + cc < p.D) {
          const size_t o = dl_off + (size_t)pos_of(i) * p.ld_delta + cc;
          if (p.delta_f32) {
            v = *reinterpret_cast<const float4*>((const float*)p.delta + o);
          } else {
            const uint2 r = *reinterpret_cast<const uint2*>((const bf16_t*)p.delta + o);
            v = make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                            __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u));
          }
        }
        pd[e] = v;
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int e = 0; e < (SC_T * SC_WMAX) / SC_THREADS; ++e) {
      if (e < per_thread) {
        const int idx = t + e * SC_THREADS;
        if (idx < SC_T * W) xs[(idx / W) * SC_WMAX + (idx % W)] = px[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int idx = t + e * SC_THREADS;
      *reinterpret_cast<uint4*>(&us[(idx >> 4) * SC_THREADS + (idx & 15) * 8]) = pu[e];
    }
    if (has_delta) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = t + e * SC_THREADS;
        *reinterpret_cast<float4*>(&dls[(idx >> 5) * SC_THREADS + (idx & 31) * 4]) = pd[e];
      }
    }
  };

  prefetch(0);
  for (int c = 0; c < nchunks; ++c) {
    commit();
    __syncthreads();
    if (c + 1 < nchunks) prefetch(c + 1);
#pragma unroll 2
    for (int tt = 0; tt < SC_T; ++tt) {
      const int i = c * SC_T + tt;
      if (i >= p.L) break;
      const float* xr = xs + tt * SC_WMAX;
      float dt = bias;
      if (has_delta) dt += dls[tt * SC_THREADS + t];
#pragma unroll
      for (int r = 0; r < RMAX; ++r)
        if (r < p.R) dt = fmaf(w[r], xr[r], dt);
      if (p.softplus) dt = softplus_f(dt);
      const float uu = bf2f(us[tt * SC_THREADS + t]);
      const float du = dt * uu;
      const float* Bv = xr + p.R;
      const float* Cv = xr + p.R + 16;
      float y = 0.0f;
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        h[n] = fmaf(exp2f(dt * a2[n]), h[n], du * Bv[n]);
        y = fmaf(h[n], Cv[n], y);
      }
      y = fmaf(dsk, uu, y);
      const int l = pos_of(i);
      if (active && l < p.n_keep) yb[(size_t)l * p.ldy] = f2bf(y);
    }
    __syncthreads();
  }
}

extern "C" int acth_selective_scan(const ActhScanDesc* d, hipStream_t stream) {
  if (!d || !d->u || !d->xdbl || !d->A_log || !d->y0) return ACTH_EINVAL;
  if (d->R > 0 && (!d->dt_w || d->delta)) return ACTH_EINVAL;       // exactly one delta source
  if (d->R == 0 && !d->delta) return ACTH_EINVAL;
  if (d->N != 16 || d->R < 0 || d->R + 32 > SC_WMAX || d->L <= 0 || d->D <= 0 || d->nb <= 0) return ACTH_EINVAL;
  if (d->G < 1 || d->G > 65535 || (d->flip1 && d->G != 2) || (d->y1 && d->G != 2)) return ACTH_EINVAL;
  if (d->n_keep < 0 || d->n_keep > d->L || d->ldx < d->G * (d->R + 32)) return ACTH_EINVAL;
  if (d->D % 8 || d->ldu % 8 || (d->delta && (d->D % 4 || d->ld_delta % 4))) return ACTH_EINVAL;
  if (d->nb > 65535) return ACTH_EINVAL;
  if (d->n_keep == 0) return ACTH_OK;
  dim3 grid((d->D + SC_THREADS - 1) / SC_THREADS, d->G, d->nb);
  if (d->R <= 8) hipLaunchKernelGGL(scan_kernel<8>, grid, dim3(SC_THREADS), 0, stream, *d);
  else if (d->R <= 20) hipLaunchKernelGGL(scan_kernel<20>, grid, dim3(SC_THREADS), 0, stream, *d);
  else if (d->R <= 40) hipLaunchKernelGGL(scan_kernel<40>, grid, dim3(SC_THREADS), 0, stream, *d);
  else if (d->R <= 80) hipLaunchKernelGGL(scan_kernel<80>, grid, dim3(SC_THREADS), 0, stream, *d);
  else hipLaunchKernelGGL(scan_kernel<96>, grid, dim3(SC_THREADS), 0, stream, *d);
  ACTH_CHECK_LAUNCH();
  return ACTH_OK;
}
