/*
 * actalker_hip.h — C ABI of libactalker_hip.so, the MI355X (gfx950) kernels behind the
 * ACTalker denoising path.
 *
 * Boundary. The reference's drop-in points for this path are Python: the `unet_cls` dotted
 * path (config/inference.yaml:62 -> Inference.py:54-62) that selects
 * UNetSpatioTemporalConditionModel (unet_spatio_temporal_condition_mambaID_v10_two_ip.py:362),
 * and below it one native op, mamba-ssm 1.2.0's `selective_scan_fn` (called at
 * mamba_layer.py:1532-1538). Everything the reference runs through torch/cuDNN/SDPA under that
 * module is exposed here as plain-pointer entry points; the Python host package
 * (actalker_amd) binds them with ctypes and mirrors the reference's module interface.
 *
 * Conventions (all entry points):
 *   - device pointers, caller-allocated; activations are token-major rows x channels, bf16
 *     (raw 16-bit) unless a field says fp32; weights are (out, in) row-major bf16;
 *   - libactalker_hip_f16.so exports the same entry points built with fp16 activations (the
 *     reference's shipped weight_dtype, config/inference.yaml:66): there every "bf16" operand
 *     below is IEEE half; fp32 operands and all descriptors are unchanged;
 *   - stream-ordered on `stream`; no allocation, no host synchronisation (graph-capturable);
 *   - return ACTH_OK (0), ACTH_EINVAL (-1) for a rejected shape/alignment, or ACTH_ELAUNCH (-2)
 *     when the launch failed;
 *   - a call with no work (zero rows / an empty batch: M, B, nbatch, nb, Sq, n = 0, as torch ops accept empty
 *     tensors) returns ACTH_OK without launching and reads no pointer (an empty tensor's data pointer may
 *     be NULL). A negative value of that primary size stays ACTH_EINVAL; the attention entry points and
 *     acth_gather_blocks also check their other sizes (>= 0, F in 1..32, block_bytes % 16) before the
 *     no-work return, the others do not inspect
 *     the remaining fields of a call with no work.
 */
#ifndef ACTALKER_HIP_H
#define ACTALKER_HIP_H

#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACTH_OK 0
#define ACTH_EINVAL (-1)
#define ACTH_ELAUNCH (-2)

/* ---- dense contraction: nn.Linear, Conv2d 3x3 (stride 1/2, nearest-x2 upsample), Conv3d (3,1,1).
 * Replaces the cuDNN conv / cuBLAS GEMM calls under diffusers ResnetBlock2D,
 * TemporalResnetBlock, Downsample2D, Upsample2D, Attention.to_q/k/v/out, FeedForward (GEGLU),
 * SS2D_cond_v10 in/out projections and SS2D_Unit x_proj (mamba_layer.py:1521). */
typedef struct ActhGemmDesc {
  const void* A; const void* A2; int lda, lda2, K1;
  int amode;                 /* 0 dense rows, 1 conv3x3 NHWC, 2 temporal 3-tap over frames */
  int H, W, Ho, Wo, conv_stride, upsample, Cin;
  int F, S;
  const void* B; int ldb;
  int M, N, K;
  const float* bias;
  const float* rowbias; int rb_div, ldrb;
  const void* R; int ldr; const int* rmap; int r_div, r_mod;
  const void* MIX; int ldmix; float mix_alpha;
  float alpha;
  int act;                   /* 0 none, 1 silu, 2 geglu (interleaved 16-col granules), 3 gelu, 4 relu */
  int out_f32;
  void* C; int ldc;
  int orow_div, orow_stride, orow_off;
  int tile;                  /* bits 0-7: 0 auto; 1 128x128 (4 waves); 2 256x256, 3 256x160, 4 256x256 / 5 256x320 phased (8 waves); bits 16-23: row-block group of the phased kernels' tile order (0 auto) */
} ActhGemmDesc;
int acth_gemm(const ActhGemmDesc* d, hipStream_t stream);
int acth_gemm_desc_size(void);

/* ---- fused GEGLU feed-forward, C = 320 (FeedForward(activation_fn="geglu") of the level-0
 * BasicTransformerBlock.ff / TemporalBasicTransformerBlock.ff_in, .ff; attention.py:223-343, 418-473,
 * activations.py GEGLU): y = [mix_alpha*mix + (1-mix_alpha)*] (W2 (h*gelu(g)) + b2 [+ res]).
 * w1: (8C, C) bf16 [h|g] rows interleaved in 16-row granules (pack_geglu), b1 likewise (fp32);
 * w2: 0.5 x (C, 4C) bf16, each 16-column block permuted: column 8hi+e <- unit 8(e/4)+4hi+e%4 (modules.ffn_w2_perm). */
typedef struct ActhFfnDesc {
  const void* x; int ldx;
  const void* w1; int ldw1; const float* b1;
  const void* w2; int ldw2; const float* b2;
  const void* res; int ldres;
  const void* mix; int ldmix; float mix_alpha;
  void* y; int ldy;
  int M, C;
  /* optional fused input LayerNorm (ln != 0): the kernel normalises x per token (fp32 statistics by bf16 dot2,
   * ln_g / ln_b may be NULL = 1 / 0) before the up projection -- norm3 / norm_in of the block folded into
   * the FFN, so the normalised tensor never reaches HBM. Optional row vector add (add != NULL):
   * x <- bf16(x + add[row / add_div]) (add_div % 64 == 0) before the LayerNorm, and res <- bf16(res + add[row / add_div]) in the
   * epilogue (TemporalBasicTransformerBlock's "h + pos_emb" feeding norm_in and the ff_in residual). */
  const float* ln_g; const float* ln_b; float ln_eps; int ln;
  const void* add; int ldadd; int add_div;
} ActhFfnDesc;
int acth_geglu_ffn(const ActhFfnDesc* d, hipStream_t stream);
/* diagnostics: host_dst == NULL -> enable (1) / disable (0) per-workgroup phase stamps; else copy the
 * stamps of the first n_wgs workgroups (8 x u64 s_memtime each) of the last stamped launch */
int acth_debug_ffn_stamps(unsigned long long* host_dst, int n_wgs, int enable);

/* ---- spatial self-attention, head_dim 64 (AttnProcessor2_0, attention_processor.py:1528-1605) */
typedef struct ActhAttnDesc {
  const void* q; const void* k; const void* v; void* o;
  int ldq, ldk, ldv, ldo;
  long long bsq, bsk, bsv, bso;
  int nbatch, nheads, Sq, Skv;
  float scale;
} ActhAttnDesc;
int acth_flash_attn(const ActhAttnDesc* d, hipStream_t stream);

/* ---- temporal self-attention over F <= 32 frames (TemporalBasicTransformerBlock.attn1,
 * attention.py:446-448) on fused [q|k|v] rows ordered (b, f, s); F <= 32 covers the reference's shipped
 * n_sample_frames = 25 window (config/inference.yaml:4 -> Inference.py:573 frames_per_batch) */
typedef struct ActhTemporalAttnDesc {
  const void* qkv; int ldqkv; void* o; int ldo;
  int B, F, S, H;
  float scale;
} ActhTemporalAttnDesc;
int acth_temporal_attn(const ActhTemporalAttnDesc* d, hipStream_t stream);

/* ---- IP-adapter cross attention (IPAdapterAttnProcessor2_0, attention_processor.py:2747-2934):
 * out = vbase[ctx] + sa*mask_a[s]*softmax(q K^T*scale) V + sb*mask_b[s]*vb[ctx] */
typedef struct ActhIpAttnDesc {
  const void* q; int ldq;
  const void* kv; int ldkv; int nkeys;
  const void* vbase; int ldvbase;
  const void* vb; int ldvb;
  const float* mask_a; const float* mask_b;
  float sa, sb, scale;
  void* out; int ldo;
  int M, H, rows_per_ctx, S;
} ActhIpAttnDesc;
int acth_ip_attn(const ActhIpAttnDesc* d, hipStream_t stream);

/* ---- fused IP-adapter cross attention block (attn2 of BasicTransformerBlock /
 * TemporalBasicTransformerBlock with norm2 before and norm3 after, attention.py:223-343, 418-473;
 * IPAdapterAttnProcessor2_0, attention_processor.py:2747-2934). Replaces, per call, the norm2 LayerNorm,
 * the to_q GEMM, acth_ip_attn, the to_out GEMM (+ residual) and the norm3 LayerNorm:
 *   out = h + bo + Wo (v_id + sa ma[s] softmax(q K^T / 8) V + sb mb[s] v_vasa),  q = Wq LN2(h)
 *   n3  = LN3(out)
 * LN2 itself folds in too: n . K'_j = rstd (h . (g2 o K'_j) - mu sum(g2 o K'_j)) + b2 . K'_j, so the kernel
 * multiplies the raw rows of h and needs only their mean / variance.
 * with Wq and Wo folded into per-context keys / values by acth_ip_fold (32 audio keys per head):
 *   K'[ctx][h*32+j] = kscale * Wq_h^T k_{ctx,h,j},  V'[ctx][h*32+j] = Wo_h v_{ctx,h,j}   (C wide, bf16)
 *   (Wo passed transposed, so every fold read is coalesced)
 *   base[ctx] = bo + Wo v_id[ctx],  vbw[ctx] = Wo v_vasa[ctx]                              (fp32)
 * Contexts are consecutive blocks of rows_per_ctx rows (a frame, or a window for the temporal block). */
typedef struct ActhIpFoldDesc {
  const void* kv; int ldkv;        /* (nctx*32, >= 2C) bf16 [K | V] of the audio tokens, or NULL (no audio term) */
  const void* wq; int ldwq;        /* to_q.weight (C, C) bf16 */
  const void* wo; int ldwo;        /* to_out[0].weight TRANSPOSED (C, C) bf16: wo[d][c] = Wo[c][d] */
  const float* bo;                 /* to_out[0].bias (C) or NULL */
  const void* vid; int ldvid;      /* (nctx, C) bf16: to_v(ID token) */
  const void* vb; int ldvb;        /* (nctx, C) bf16: to_v_ip[1](VASA token), or NULL */
  const float* g2; const float* b2; /* norm2 weight / bias (C) fp32, or NULL (1 / 0): folded into K'' / gb */
  float kscale;                    /* folded into K' (log2(e) / 8: scores in exp2 units) */
  void* kp; void* vp;              /* (nctx*H*32, C) bf16 outputs (kv != NULL): K'' = g2 o K', V' */
  float* gb;                       /* (nctx*H*32, 2) fp32 output (kv != NULL): per key (sum_c K''_c, b2 . K') */
  float* base; float* vbw;         /* (nctx, C) fp32 outputs; vbw written when vb != NULL */
  int nctx, C, H;
} ActhIpFoldDesc;
int acth_ip_fold(const ActhIpFoldDesc* d, hipStream_t stream);

typedef struct ActhXattnDesc {
  const void* h; int ldh;          /* (M, C) bf16 residual stream */
  float eps2;                      /* norm2 eps (its weight / bias are folded into kp / gb) */
  const void* kp; const void* vp;  /* acth_ip_fold's K'' / V', or NULL (no audio term) */
  const float* gb;                 /* acth_ip_fold's per-key LN2 constants (with kp) */
  const float* base; int ldbase;   /* (nctx, C) fp32 */
  const float* vbw; int ldvbw;     /* (nctx, C) fp32 or NULL (no VASA term) */
  const float* mask_a; const float* mask_b;          /* per token position (period S) or NULL */
  float sa, sb;
  const float* g3; const float* b3; float eps3;      /* norm3 */
  void* out; int ldo;              /* (M, C) bf16: h + attn2 */
  void* n3; int ldn3;              /* (M, C) bf16: norm3(out) */
  int M, C, H, rows_per_ctx, S;    /* C = 320 (level 0); rows_per_ctx % 64 == 0, M % rows_per_ctx == 0 */
} ActhXattnDesc;
int acth_xattn(const ActhXattnDesc* d, hipStream_t stream);
/* diagnostics: host_dst == NULL -> enable (1) / disable (0) per-workgroup phase stamps; else copy the stamps
 * of the first n_wgs workgroups (6 x u64 s_memtime each) of the last stamped launch */
int acth_debug_xattn_stamps(unsigned long long* host_dst, int n_wgs, int enable);

/* ---- LayerNorm with optional fused row-vector pre-add */
typedef struct ActhLayerNormDesc {
  const void* x; int ldx;
  const void* add; int ldadd; int add_div;
  void* sum_out; int ldsum;
  const float* gamma; const float* beta; float eps;
  void* y; int ldy;
  int M, C;
} ActhLayerNormDesc;
int acth_layernorm(const ActhLayerNormDesc* d, hipStream_t stream);

/* ---- GroupNorm(G), stats over rows_per_stat tokens, optional channel-concat input;
 * y = act(GN(x) + res): act (field `silu`) 0 none, 1 SiLU, 2 ReLU; res (bf16 rows, C channels) optional
 * (ResNet-GN blocks of the VASA encoders, vasa_feature_v2.py:64-85 / 129-150) */
typedef struct ActhGroupNormDesc {
  const void* x; int ldx; const void* x2; int ldx2; int C1;
  int M, C, G, rows_per_stat;
  const float* gamma; const float* beta; float eps;
  int silu;
  void* y; int ldy;
  double* ws;
  const void* res; int ldres;
} ActhGroupNormDesc;
int acth_groupnorm(const ActhGroupNormDesc* d, hipStream_t stream);
/* ws: acth_groupnorm_workspace_size bytes, no clearing needed (each statistics block writes its own fp64
 * partial-sum slot; the apply pass adds them in a fixed order, so the output is bitwise reproducible) */
size_t acth_groupnorm_workspace_size(int M, int C, int G, int rows_per_stat);

/* ---- SS2D_cond_v10 scatter-back + sum + out_norm (mamba_layer.py:1963-1985) */
typedef struct ActhMambaCombineDesc {
  const void* xa; int ldxa; const void* ya0; const void* ya1; int ldya; int La; const int* pos_a; int mode_a;
  const void* xe; int ldxe; const void* ye0; const void* ye1; int ldye; int Le; const int* pos_e; int mode_e;
  const float* gamma; const float* beta; float eps;
  void* y; int ldy;
  int M, S, C;
} ActhMambaCombineDesc;
int acth_mamba_combine_ln(const ActhMambaCombineDesc* d, hipStream_t stream);

/* ---- selective scan. Replaces mamba_ssm.ops.selective_scan_interface.selective_scan_fn(u, delta,
 * A, B, C, D, z=None, delta_bias, delta_softplus) as called at mamba_layer.py:1532-1538.
 * Two uses: (1) fused SS2D mode: dt_proj folded in (R > 0, delta = NULL), G = 2 directions over
 * the same u channels (u_gstride = 0), direction 1 traversed in reverse (flip1 = 1), outputs to
 * y0 / y1; (2) op mode: explicit delta (R = 0), G groups of D channels (u_gstride = y_gstride = D),
 * forward traversal. xdbl rows hold per group [dt(R) | B(16) | C(16)] in fp32. */
typedef struct ActhScanDesc {
  const void* u; int ldu;
  const float* xdbl; int ldx;
  const float* dt_w;          /* (G, D, R) fp32, R > 0 */
  const float* dt_b;          /* (G, D) fp32 or NULL */
  const float* A_log;         /* (G*D, 16) fp32, A = -exp(A_log) */
  const float* Dskip;         /* (G*D) fp32 or NULL */
  void* y0; void* y1; int ldy;
  int nb, L, D, R, N, n_keep;
  const void* delta; int ld_delta; int delta_f32; int softplus;
  int G, u_gstride, y_gstride, flip1;
  int nchunks;                /* >1: two-pass chunked scan (needs ws); 0/1: single pass */
  int chunk_len;              /* derived by the library (ignored on input) */
  float* ws;                  /* acth_selective_scan_workspace_size(nb, G, D, nchunks) bytes */
  int xdbl_bf16;              /* 1: xdbl rows are bf16 (the reference's x_dbl dtype, mamba_layer.py:1521),
                                 per direction [dt (R rounded up to 4, padding ignored) | B(16) | C(16)];
                                 fused SS2D form only (R > 0, G = 2, flip1, single pass) */
  int scan_algo;              /* bf16 xdbl: 0 paired-lane kernel (default), 1 scan_quad_kernel */
} ActhScanDesc;
int acth_selective_scan(const ActhScanDesc* d, hipStream_t stream);
/* Both SS2D branches of SS2D_cond_v10 (audio d0, expression d1; mamba_layer.py:1955-1986) in one
 * launch when they share R, D, G, softplus and are single-pass; otherwise two launches. Each
 * descriptor means exactly what it means to acth_selective_scan. */
int acth_selective_scan2(const ActhScanDesc* d0, const ActhScanDesc* d1, hipStream_t stream);
size_t acth_selective_scan_workspace_size(int nb, int G, int D, int nchunks);

/* ---- direct 3x3 (pad 1, stride 1/2) / temporal (3,1,1) convolution for narrow channel counts
 * (PoseGuider InflatedConv3d, pose_guider.py:17-73; VAE Encoder conv_in / downsamplers, TemporalDecoder
 * conv_in / conv_out / time_conv_out).
 * x: NHWC bf16 rows; w: fp32 (taps*Cin, Cout), k = tap*Cin + c (tap = ky*3 + kx, or the frame tap);
 * y: rows (B*Ho*Wo | B*F*S, ldy), bf16 or fp32; act 0 none / 1 silu / 3 gelu (erf).
 * A Conv1d (k 3, pad 1, stride s) is the H = 1 case with the kernel in the middle row (Whisper conv1/conv2). */
typedef struct ActhConvDirectDesc {
  const void* x; int ldx;
  const float* w; const float* bias;
  void* y; int ldy;
  int mode;                  /* 0 spatial 3x3, 1 temporal 3-tap over F frames (rows (b*F + f)*S + s) */
  int B, H, W, Ho, Wo, stride;
  int pad0;                  /* mode 0: 0 = padding 1 all sides; 1 = bottom/right only (diffusers Downsample2D padding=0) */
  int F, S;
  int Cin, Cout, act, out_f32;
} ActhConvDirectDesc;
int acth_conv_direct(const ActhConvDirectDesc* d, hipStream_t stream);

/* ---- y(bf16) = softmax(scale * x(fp32)) per row (VAE mid-block single-head attention) */
int acth_softmax_rows(const float* x, int ldx, void* y, int ldy, int rows, int cols, float scale,
                      hipStream_t stream);

/* ---- small kernels */
int acth_timestep_embedding(const float* t, int n, int dim, int flip_sin_to_cos, float downscale_freq_shift,
                            float scale, float max_period, void* out, hipStream_t stream);
int acth_nchw_to_tokens(const void* x, int in_dt, void* y, int out_dt, int ldy, int B, int C, int HW,
                        hipStream_t stream);
int acth_tokens_to_nchw(const void* x, int in_dt, int ldx, void* y, int out_dt, int B, int C, int HW,
                        hipStream_t stream);
int acth_im2col3x3(const void* x, int B, int H, int W, int C, void* out, int Kpad, hipStream_t stream);
int acth_im2col(const void* x, int ldx, int B, int H, int W, int C, int kh, int kw, int stride, int pad,
                int Ho, int Wo, void* out, int Kpad, hipStream_t stream);
int acth_maxpool2d(const void* x, int ldx, int B, int H, int W, int C, int k, int stride, int pad, int Ho, int Wo,
                   void* y, int ldy, hipStream_t stream);
int acth_gather_rows(const void* src, int lds, int Ls, const int* idx, int n, void* dst, int ldd, int Ld,
                     int nb, int C, hipStream_t stream);
int acth_frame_mean(const void* x, int ldx, int B, int F, int T, int C, void* out, int ldo,
                    hipStream_t stream);
/* dst block i = src block idx[i], i < n (block_bytes each, a multiple of 16; src, dst 16-byte aligned; idx on the
 * device, entries in [0, n_src) -- not checked on the device; n <= 65535). The UNet's CFG-prefix sharing
 * (actalker_amd UNet.forward_tokens) copies the distinct batch elements' activations out to the full batch with it,
 * where the reference simply runs every CFG branch through the whole UNet (pipeline:712-729). */
int acth_gather_blocks(const void* src, int n_src, const int* idx, int n, long long block_bytes, void* dst,
                       hipStream_t stream);

/* ---- sampler loop (pipeline_svd_audio_adapter_motionexp_idembed_vasa_two_ip.py:684-756) */
int acth_window_input(const float* lat, const int* frame_idx, const float* img, const int* branch,
                      float in_scale, void* out, int U, int F, int S, int T, hipStream_t stream);
int acth_cfg_euler_accum(const float* noise, const long long* unit_off, const float* lat, const int* frame_idx,
                         float g1, float g2, float g3, float sigma, float sigma_next, float* acc, float* cnt,
                         int F, int S, hipStream_t stream);
int acth_div_counter(const float* acc, const float* cnt, float* out, int T, int S, hipStream_t stream);
int acth_version(void);
/* activation dtype the library was built for: 0 = bf16 (libactalker_hip.so), 1 = fp16 (libactalker_hip_f16.so);
 * the same C ABI is exported by both, so a host binding checks this once after loading */
int acth_act_dtype(void);
/* diagnostics: per-workgroup s_memtime phase stamps of the last phased-GEMM launch made with tile bit
 * 0x400 (entry, prologue landed, main loop done, epilogue done), n_wgs x 4 values copied to host */
int acth_debug_gemm_stamps(unsigned long long* host_dst, int n_wgs);

#ifdef __cplusplus
}
#endif
#endif /* ACTALKER_HIP_H */
