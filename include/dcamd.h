/*
 * dcamd.h -- C ABI of the MI355X-native Marigold-DC guided sampler (libdcamd.so, gfx950).
 *
 * The reference (tier4/depth_completion) has no native/FFI boundary: its hot path is the Python
 * operator API MarigoldDepthCompletionPipeline.__call__ (marigold_dc.py:467-985), executed by
 * diffusers/PyTorch CUDA kernels.  This header is the boundary the MI355X build inserts beneath
 * that API: plain device pointers, sizes and a hipStream_t (passed as void*), every entry point
 * returning an int status (0 = ok, 1 = bad argument, 2 = launch failure, 3 = alignment).  No
 * torch types cross it.  Layouts: bf16 tensors are NHWC "pixel rows" (row stride `ld*` in
 * elements, multiple of 8); fp32 for statistics, affine parameters and losses.
 *
 * Which reference call each group replaces is noted per function.
 */
#ifndef DCAMD_H
#define DCAMD_H

#ifdef __cplusplus
extern "C" {
#endif

int dc_abi_version(void);
/* sha256 prefix (16 hex digits) of the sources this library was built from (build provenance) */
const char* dc_build_id(void);

/* ---------------------------------------------------------------- matmul-shaped ops
 * Implicit-GEMM conv / linear on MFMA.  Replaces the cuDNN conv fwd/dgrad and cuBLAS GEMMs that
 * diffusers' UNet2DConditionModel (_predict_noise, marigold_dc.py:459-465) and AutoencoderTiny
 * (decode_prediction, marigold_dc.py:366; prepare_latents, :696-698) launch, and their autograd
 * input-gradients (losses.backward, marigold_dc.py:877).  Weight gradients are not computed: the
 * reference optimizer only holds latents and affine parameters (marigold_dc.py:777-781).
 * mode: 0 direct conv (stride/pad), 1 nearest-upsample hin->hout folded into the gather (Upsample2D),
 *       2 transposed stride-2 gather (input-gradient of a stride-2 3x3 conv, Downsample2D).
 * Epilogue order: acc + bias -> (+ rowbias[*rowbias_idx]) -> (+ resid) -> relu? -> (* [mask > 0]).
 */
/* GroupNorm statistics fused into the epilogue of the conv / linear that produces the normalised tensor
 * (diffusers ResnetBlock2D norm1 / norm2, Transformer2DModel.norm, conv_norm_out: every GroupNorm input of the
 * UNet is a conv or linear output, and so is every GroupNorm output-gradient).  The sums go into fixed-point
 * accumulators of dc_gn_acc_bytes(nb, groups) bytes (zero-filled before the producers run): per (frame, group)
 * two quantities, each an integer of 8 32-bit limbs (LSB 2^-120) plus a non-finite count, to which every block's
 * fp32 partial (its tile folded in a fixed order) is added with integer atomics -- the sum of the partials is
 * exact, so it does not depend on tile order or arrival order (bitwise reproducible); the partials are fp32.  dc_groupnorm_fwd_acc / dc_groupnorm_bwd_acc then normalise in one pass.
 *   mode 1 (forward): (sum y, sum y^2) of the stored bf16 outputs into t[0 .. nt-1] (one output may be both the
 *          direct input of one GroupNorm and the skip half (coff = c1) of an up-block concat);
 *   mode 2 (backward): the output is dL/d(GroupNorm(+SiLU) output); with the GroupNorm input x (x2: channels
 *          >= c1), its forward stats [nb][groups][2] (mean, rstd), gamma, beta the epilogue stores
 *          dy' = bf16(dy * silu'(bf16(xhat gamma + beta))) (silu; else dy) and adds (sum gamma dy',
 *          sum gamma dy' xhat) into t[0].
 * Frames are hw output rows each (the row index of a linear over nb * hw token rows works the same way). */
typedef struct dc_gn_target {
  long long* acc;
  int coff;         /* channel offset of this output inside the normalised tensor */
  int groups, cpg;
  int hw;
} dc_gn_target;
typedef struct dc_gn_fuse {
  int mode;         /* 1 forward, 2 backward */
  int nt;           /* targets used (1 or 2; mode 2: 1) */
  dc_gn_target t[2];
  const void* x;
  const void* x2;
  int ldx, ldx2, c1;
  const float* stats;
  const float* gamma;
  const float* beta;
  int silu;
} dc_gn_fuse;
long long dc_gn_acc_bytes(int nb, int groups);
/* LayerNorm of the input rows folded into a linear (BasicTransformerBlock norm3 -> ff.net.0.proj,
 * marigold_dc.py:460-465 through diffusers): with W' = bf16(W diag(gamma)) as the call's weight, csum[n] =
 * sum_k W'[n][k] and cbias[n] = sum_k W[n][k] beta[k] + bias[n] (dc_fold_layernorm), and the input rows' (mean, rstd)
 * in stats[rows][2] (dc_crossattn_fwd's ystats: the producer of norm3's input holds whole rows), the epilogue stores
 *   y = rstd (x . W'^T - mean csum) + cbias  =  LayerNorm(x) . W^T + bias   (up to rounding),
 * so the normalised rows are never written.  The input-gradient of the folded weight (W'^T) yields gamma * dL/dLN(x)
 * (dc_crossattn_bwd_ln / dc_layernorm_bwd with gamma NULL take it from there).
 * Contract: a linear (1x1, stride 1, pad 0, mode 0) with cin == ktot, no second source, no row list, no GroupNorm
 * fusion, bias NULL (cbias replaces it), geglu 0 or 1; the im2col tile variants (another choice runs the heuristic). */
typedef struct dc_ln_fuse {
  const float* csum;
  const float* cbias;
  const float* stats;
} dc_ln_fuse;
/* the folded weight and its column constants, on the host (the Python host and the native session share it):
 * w, gamma, beta fp32 (bf16-exact values), bias fp32 or NULL; wf bf16 [cout][k] out; csum, cbias fp32 [cout] out */
int dc_fold_layernorm(const float* w, int cout, int k, const float* gamma, const float* beta, const float* bias,
                      void* wf, float* csum, float* cbias);
/* FF2 (ff.net.2: y = x W2^T + b2, W2 [c][k2]) and the proj_out after it (z = y' Wp^T + bp, Wp [c][c], where
 * y' = y + r is FF2's residual sum) folded into one two-source linear over [x | r]:
 *   z = x (Wp W2)^T + r Wp^T + (Wp b2 + bp)
 * (BasicTransformerBlock's last residual and Transformer2DModel.proj_out, marigold_dc.py:460-465 through diffusers;
 * exact in real arithmetic: y' is not rounded to bf16 and Wp W2 is, the order of roundings changes).  w2, b2, wp, bp
 * fp32 (bf16-exact values); wf bf16 [c][k2 + c] = [bf16(Wp W2) | Wp] out; wd bf16 [k2 + c][c] = wf^T out (its input
 * gradient: columns < k2 are dL/dx, the GEGLU backward's input, the rest dL/dr); bias fp32 [c] out.  Products in
 * double, summed in k order, rows on up to 16 host threads (the same bits on every host). */
int dc_fold_linear_pair(const float* w2, const float* b2, int c, int k2, const float* wp, const float* bp, void* wf,
                        void* wd, float* bias);
/* 1 where the fused statistics pay for a GroupNorm of hw pixels x c channels (forward / backward): not where the
 * single-launch GroupNorm (one block per group, levels 2-3 of the UNet) runs it.  Both hosts plan with it. */
int dc_gn_fuse_pays(int hw, int c, int groups, int backward);

typedef struct dc_conv_desc {
  const void* x;   /* bf16 [nb*hin*win][ldx] */
  const void* x2;  /* optional second source for channels >= c1 (skip concat) */
  int ldx, ldx2, c1;
  int nb, hin, win, cin;
  int hout, wout;
  int kh, kw, stride, pad, mode;
  const void* w;   /* bf16 [cout][ktot], K order (ky, kx, cin), ktot % 64 == 0 */
  int ktot, cout;
  const float* bias;
  const void* rowbias;
  const int* rowbias_idx;
  int rowbias_ld;
  const void* resid;
  int ldr;
  const void* mask;
  int ldmask;
  int act;         /* 0 none, 1 relu */
  void* y;
  int ldy;
  float* ws;       /* split-K workspace (may be NULL: no split-K) */
  long long ws_bytes;
  /* GEGLU epilogues (diffusers GEGLU of the transformer FF, ff.net.0, fused into its two linears):
   * 1: the output columns are (h, gate) pairs interleaved 8 + 8 (FF1 rows permuted at load); y gets the raw
   *    pre-activation, y2[m][c/2 ..] = h * gelu(gate) (the [T][4C] input of FF2);
   * 2: the output is dL/d(h * gelu(gate)) (FF2 input-gradient, 4C channels); with the pre-activation in aux
   *    (interleaved layout) y gets (dL/dh, dL/dgate) interleaved 8 + 8 (the [T][8C] gradient of FF1's output) */
  int geglu;
  void* y2;
  int ldy2;
  const void* aux;
  int ldaux;
  int algo;        /* 0 = heuristic, 1..dc_conv_num_algos(): tile/ring variant (plan-time autotuned):
                      1-22, 37-42, 59-61 im2col tiles; 23-36 halo-tile direct 3x3; 43-54 weight-streaming skinny
                      conv / linear (few output pixels); 55-58 weight-resident persistent 3x3 (cin 64, cout <= 64).
                      A variant given a shape outside its contract runs the heuristic. */
  int splitk;      /* 0 = heuristic, >=1 explicit K split, -1..-4 stream-K over 256..1024 blocks (needs ws);
                      skinny variants: -2..-32 = that K split summed by a second (reduce) kernel; resident variants:
                      blocks per CU of the persistent grid (0 = as many as fit) */
  /* optional row list: only the nrows output pixels rows[0..nrows) (sorted indices into the nb*hout*wout
   * output rows) are computed and written; the others are left untouched (no GEGLU epilogue) */
  const int* rows;
  int nrows;
  /* optional fused GroupNorm statistics (above; NULL: none).  Needs cout % 8 == 0, no row list, no GEGLU. */
  const dc_gn_fuse* gn;
  /* optional LayerNorm of the input rows folded in (dc_ln_fuse above; NULL: none) */
  const dc_ln_fuse* ln;
  /* GEGLU 2 only: 0 = every column; 0 < geglu_n < cout (a multiple of 256): columns < geglu_n get the GEGLU backward
   * into y (ldy >= 2 geglu_n), columns >= geglu_n are stored plainly into y2[m][c - geglu_n] -- the input-gradient of
   * FF2 and proj_out folded into one linear (dc_fold_linear_pair) */
  int geglu_n;
} dc_conv_desc;

int dc_conv_num_algos(void);
int dc_conv_gemm(const dc_conv_desc* d, void* stream);

/* ---------------------------------------------------------------- normalisation
 * GroupNorm(+SiLU) fwd/bwd (ResnetBlock2D.norm1/norm2, Transformer2DModel.norm, conv_norm_out) and
 * LayerNorm fwd/bwd (BasicTransformerBlock.norm1/norm3).  stats: [nb][groups][2] (mean, rstd).
 */
long long dc_groupnorm_ws_bytes(int nb, int hw, int c, int groups);
int dc_groupnorm_fwd(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c, int groups,
                     float eps, const float* gamma, const float* beta, int silu, void* y, int ldy, float* stats,
                     float* ws, void* stream);
int dc_groupnorm_bwd(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c, int groups,
                     const float* gamma, const float* beta, int silu, const float* stats, const void* dy, int lddy,
                     void* dx, int lddx, const void* add1, int ldadd1, const void* add2, int ldadd2, float* ws,
                     void* stream);
/* one-pass GroupNorm from the fused statistics (dc_gn_fuse): acc as filled by the producers of x (and x2).
 * fwd: y = GN(x)(+SiLU), stats [nb][groups][2] (mean, rstd) written for the backward;
 * bwd: dyp = the producer's stored dy' (mode 2), dx = rstd (gamma dy' - mean_a - xhat mean_b) (+ add1)(+ add2). */
int dc_groupnorm_fwd_acc(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c, int groups,
                         float eps, const float* gamma, const float* beta, int silu, const long long* acc, void* y,
                         int ldy, float* stats, void* stream);
int dc_groupnorm_bwd_acc(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c, int groups,
                         const float* gamma, const float* stats, const long long* acc, const void* dyp, int lddy,
                         void* dx, int lddx, const void* add1, int ldadd1, const void* add2, int ldadd2,
                         void* stream);
int dc_layernorm_fwd(const void* x, int ldx, long long rows, int c, float eps, const float* gamma, const float* beta,
                     void* y, int ldy, float* stats, void* stream);
/* gamma NULL: dy is already gamma * dL/dy (the input-gradient of a dc_ln_fuse folded weight) */
int dc_layernorm_bwd(const void* x, int ldx, long long rows, int c, const float* gamma, const float* stats,
                     const void* dy, int lddy, void* dx, int lddx, const void* add, int ldadd, void* stream);

/* ---------------------------------------------------------------- attention (head dim 64)
 * Self-attention (Attention.attn1 via SDPA) fwd/bwd and the folded 2-key cross-attention
 * (attn2 with the constant empty-prompt context, marigold_dc.py:463, :663-674) fused with norm2.
 */
/* ws / ws_bytes: the fp32 scratch also given to dc_conv_gemm (its last 64 KB zero-filled counters); the
 * batch-1 level-0 shapes run stream-K kernels whose partial (m, l, O) / dK / dV / dQ slabs live there
 * (null: plain grid) */
int dc_attn_fwd(const void* qkv, int ld, int nb, int t, int heads, void* o, int ldo, float* lse, float* ws,
                long long ws_bytes, void* stream);
/* delta_ws: fp32 scratch of 2 nb heads t floats (ABI 21; was nb heads t): the dQ kernel fills it with the dK/dV kernel's
 * row constants, -rowsum(dO o O) then -8 lse */
int dc_attn_bwd(const void* qkv, int ld, const void* o, int ldo, const void* dout, int lddo, const float* lse, int nb,
                int t, int heads, float* delta_ws, void* dqkv, int ldd, float* ws, long long ws_bytes, void* stream);
/* folded cross-attention on MFMA (csrc/crossattn.hip): U, D fp32 [heads][c] (dc_fold_cross_attention) are
 * prepared once into bf16 hi / lo MFMA operand tables of dc_crossattn_tables_bytes(heads, c) bytes; heads <= 32,
 * c % 32 == 0, c <= 1280.  stats [rows][2] (mean, rstd of norm2), probs [rows][heads] (the sigmoids) are kept
 * for the backward. */
long long dc_crossattn_tables_bytes(int heads, int c);
int dc_crossattn_prepare(const float* U, const float* D, int heads, int c, void* tabs, void* stream);
/* ystats: NULL, or [rows][2] (mean, rstd with eps yeps) of the output rows y (norm3's statistics, dc_ln_fuse) */
int dc_crossattn_fwd(const void* x, int ldx, long long rows, int c, int heads, float eps, const float* gamma,
                     const float* beta, const void* tabs, const float* c0, void* y, int ldy, float* stats,
                     float* probs, float* ystats, float yeps, void* stream);
int dc_crossattn_bwd(const void* x, int ldx, long long rows, int c, int heads, const float* gamma, const void* tabs,
                     const float* stats, const float* probs, const void* dy, int lddy, void* dx, int lddx,
                     void* stream);
/* the same with its dy computed in the launch: dy = LayerNorm backward (norm3, BasicTransformerBlock) of dl, which is
 * gamma3 * dL/dLN3(x3) (the input-gradient of the folded ff.net.0.proj, dc_ln_fuse), over x3 with stats3 [rows][2]
 * (mean, rstd), plus add (the residual gradient): the arithmetic of dc_layernorm_bwd with gamma NULL, so the result
 * equals dc_layernorm_bwd followed by dc_crossattn_bwd bit for bit. */
int dc_crossattn_bwd_ln(const void* x, int ldx, long long rows, int c, int heads, const float* gamma, const void* tabs,
                        const float* stats, const float* probs, const void* dl, int lddl, const void* x3, int ldx3,
                        const float* stats3, const void* add, int ldadd, void* dx, int lddx, void* stream);

/* ---------------------------------------------------------------- elementwise
 * GEGLU (FeedForward.net[0]), nearest-upsample adjoint (Upsample2D / TAESD Upsample backward),
 * TAESD DecoderTiny input clamp tanh(x/3)*3 and its backward fused with the Tweedie-preview
 * backward, image preprocessing (MarigoldImageProcessor.preprocess, marigold_dc.py:687-692, plus
 * EncoderTiny's x.add(1).div(2)), layout conversion at the API boundary.
 */
int dc_geglu_fwd(const void* f, int ldf, long long rows, int c, void* y, int ldy, void* stream);
int dc_geglu_bwd(const void* f, int ldf, long long rows, int c, const void* dy, int lddy, void* df, int lddf,
                 void* stream);
int dc_upsample_adjoint(const void* dhi, int ldhi, int nb, int hhi, int whi, int c, int hlo, int wlo, void* dlo,
                        int ldlo, const void* mask, int ldmask, void* stream);
int dc_taesd_clamp_fwd(const void* x, int ldx, long long pixels, void* y, void* stream);
int dc_taesd_clamp_bwd(const void* x0, int ldx0, const void* dy, int lddy, long long pixels, const float* coef,
                       const int* step, void* gx_direct, void* dv, void* stream);
int dc_silu(const void* x, long long n, void* y, void* stream);
int dc_preprocess_image(const void* img_u8, int nb, int h, int w, int rh, int rw, int ph, int pw, int encoder_input,
                        void* out, void* stream);
int dc_nhwc_to_nchw(const void* x, int ldx, int nb, long long hw, int c, void* y, void* stream);
int dc_nchw_to_nhwc(const void* x, int nb, long long hw, int c, void* y, int ldy, void* stream);

/* ---------------------------------------------------------------- sparse guidance
 * Replaces marigold_dc.py:706-756 (sparse normalisation), :813-904 (Tweedie preview, learned
 * affine, l1+l2 loss and its gradient, grad-norm rescale, Adam, DDIM update) and :969-985
 * (final dense depth).  Per-step scalars are read from device tables indexed by *step so that a
 * captured hipGraph of one step can be replayed for every timestep.
 * norm: 0 const, 1 minmax, 2 percentile (host_lohi[2*nb] = quantiles); projection: 0 linear,
 * 1 log, 2 log10.  params[nb][8] = lo, hi, lo_p, hi_p, min_g, max_g, count, 0.
 * coef[step][4] = sqrt(a_t), sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev);
 * adam_tab[step][4] = lr_latent/bc1, sqrt(bc2), lr_affine/bc1, 0.
 * params[nb][8] (dc_sparse_setup) = lo, hi, lo_p, hi_p, min_g, max_g, count, projection + 4 inv: the losses
 * compare in the projected / inverted depth space it names (marigold_dc.py:843-860).
 */
/* interp: 0 bilinear, 1 nearest (the resize of _latent_to_affine, marigold_dc.py:366-370; stored in
 * params[7] bit 3 for every kernel that samples the decoded map) */
int dc_sparse_setup(const float* sparse, int nb, int h, int w, int norm, float min_depth, float max_depth,
                    const float* host_lohi, int projection, int inv, int interp, int* idx, float* gval, int* cnt,
                    float* params, void* stream);
int dc_preview(const void* x8, const void* v, int nb, int hw, const float* coef, const int* step, void* x0, void* tin,
               float* eps_norm, void* stream);
int dc_sparse_loss(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w, const int* idx,
                   const float* gval, const int* cnt, const float* params, const float* affine, float* dA,
                   float* daff_grad, float* loss, void* stream);
int dc_decode_tail_bwd(const void* dec_out, int ldo, const float* dA, int nb, int ph, int pw, int rh, int rw,
                       void* dout, void* stream);
/* opt: 0 Adam, 1 SGD, 2 Adagrad (marigold_dc.py:783-789); kld_mode: 0 off, 1 "simple", 2 "strict"
 * (utils.kld_stdnorm), weighted by kld_weight; for SGD / Adagrad adam_tab rows are [lr_lat, 0, lr_aff, 0] */
int dc_latent_update(void* x8, const void* v, const void* gdir, const void* gunet, int nb, int hw, const float* coef,
                     const float* adam_tab, const int* step, const float* eps_norm, void* m_lat, void* v_lat,
                     float* affine, float* m_aff, float* v_aff, const float* daff_grad, float* dbg, int opt,
                     int kld_mode, float kld_weight, float* ws, long long ws_bytes, void* stream);
/* ws (nb * ceil(hw / 256) floats; may be null): per-block partials of ||g||^2 for the two-launch form
 * (kld_mode 0 / 1); without it (or with the strict KL term) one block per frame does both passes */
int dc_step_advance(int* step, int nsteps, void* stream);  /* saturates at nsteps-1 */
/* initial latents (marigold_dc.py:661, 677-704): x8[..., 4:8] <- noise, or beta * noise + (1 - beta) * prev;
 * noise bf16 [noise_frames][4][hw] NCHW: noise_frames 1 = one draw shared by all nb frames (the reference's
 * single generator draw), noise_frames nb = one draw per frame (the per-seed draws of a seed ensemble) */
int dc_latent_init(const void* noise, int noise_frames, const void* prev, float beta, int nb, int hw, void* x8,
                   void* stream);
int dc_final_dense(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                   const float* params, const float* affine, int mode, float* dense, void* stream);
/* mode 0 learned affine (marigold_dc.py:323-331), 1 closed form (:332-336) */
/* plain DDIM step, train_latents=False (marigold_dc.py:905-909): x8[...,4:8] <- prev_sample(v, x) */
int dc_ddim_step(void* x8, const void* v, int nb, int hw, const float* coef, const int* step, void* stream);
/* compute_affine_params (marigold_dc.py:53-128) over the sparse pixels: affine[nb][2] = scale, shift */
int dc_closed_form_affine(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                          const int* idx, const float* gval, const int* cnt, const float* params, float* affine,
                          void* stream);
/* guided steps with closed_form=True (marigold_dc.py:332-336 inside :828-877): loss of the closed-form fit
 * of the preview and its gradient dA, the fit (s, t) included in the differentiation */
int dc_sparse_loss_cf(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                      const int* idx, const float* gval, const int* cnt, const float* params, float* dA, float* loss,
                      void* stream);
/* train_method="per-input" with learned affine (marigold_dc.py:911-967): train_steps Adam steps on
 * affine[nb][2] (scale, shift) against the fixed decode of the final latents */
int dc_affine_fit(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w, const int* idx,
                  const float* gval, const int* cnt, const float* params, int train_steps, float lr, int opt,
                  float* affine, float* loss, void* stream);
/* compute_loss with the full-image terms (marigold_dc.py:131-245: l1, l2, edge, smooth; flags 1 | 2 | 4 | 8)
 * on the dense map (replaces dc_sparse_loss when loss_funcs is not {l1, l2}): loss[nb], daff_grad[nb][2]
 * and the resize-adjoint gradient added into dA [nb][ph][pw].
 * imgs: the caller's uint8 [nb][3][h][w] (edge: gray = 0.299 R + 0.587 G + 0.114 B); gmap: dc_guide_map;
 * ws: dc_dense_loss_ws_bytes(nb, h, w) bytes.
 * flag 16: closed-form affine (marigold_dc.py:332-336): `affine` is dc_closed_form_stats' [nb][8], the map
 *          is scale * A + shift, daff_grad receives (Gs, E) for dc_closed_form_adjoint;
 * flag 32: no clamp(0, 1) (the per-input loop, marigold_dc.py:927-929);
 * flag 64: dA untouched (may be null): only loss and daff_grad (per-input training). */
long long dc_dense_loss_ws_bytes(int nb, int h, int w);
int dc_guide_map(const int* idx, const float* gval, const int* cnt, int nb, int h, int w, float* gmap, void* stream);
int dc_dense_loss(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                  const unsigned char* imgs, const float* gmap, const int* cnt, const float* params,
                  const float* affine, int flags, float* ws, float* dA, float* daff_grad, float* loss, void* stream);
/* closed_form=True guided steps with full-image losses: the fit of the preview with its statistics
 * st8[nb][8] = (scale, shift, mean A, mean guide, var + eps, count, 0, 0) (compute_affine_params,
 * marigold_dc.py:53-128), and, after dc_dense_loss(flags | 16), the fit's share of dL/dA at the sparse
 * pixels added into dA (grad2 = dc_dense_loss' daff_grad) */
int dc_closed_form_stats(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                         const int* idx, const float* gval, const int* cnt, const float* params, float* st8,
                         void* stream);
int dc_closed_form_adjoint(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                           const int* idx, const float* gval, const int* cnt, const float* params, const float* st8,
                           const float* grad2, float* dA, void* stream);
/* per-input training with full-image losses: one optimiser step (opt 0 Adam, 1 SGD, 2 Adagrad; `it` the
 * 1-based step) of affine[nb][2] from grad2[nb][2] (dc_dense_loss flags | 32 | 64), state[nb][4] zeroed
 * before the first step (marigold_dc.py:911-967) */
int dc_affine_step(int nb, const float* grad2, int it, float lr, int opt, float* state, float* affine, void* stream);
int dc_memset_async(void* ptr, int value, long long bytes, void* stream);

/* ---------------------------------------------------------------- sparse-aware decode row sets
 * With the point losses the guided step reads the decoded map only at the resize taps of the sparse
 * pixels (marigold_dc.py:195-205 via _latent_to_affine's resize, :366-370); the decoder's full-resolution
 * convs then run on row lists (dc_conv_desc.rows) of the taps' receptive fields.
 * dc_tap_mask: byte mask [nb][ph][pw] of the taps; dc_dilate_mask: 3x3 dilation (in != out);
 * dc_mask_count then dc_mask_rows: sorted pixel indices of a mask (count[0] of them, padded up to pad_to
 * with the last index), ws of dc_mask_rows_ws_bytes(total) bytes. */
int dc_tap_mask(const int* idx, const int* cnt, const float* params, int nb, int ph, int pw, int rh, int rw, int h,
                int w, unsigned char* mask, void* stream);
int dc_dilate_mask(const unsigned char* in, int nb, int ph, int pw, unsigned char* out, void* stream);
long long dc_mask_rows_ws_bytes(long long total);
int dc_mask_count(const unsigned char* mask, long long total, int* ws, int* count, void* stream);
int dc_mask_rows(const unsigned char* mask, long long total, const int* ws, const int* count, int pad_to, int* rows,
                 void* stream);
/* rows[count[0] .. pad_to) = rows[count[0] - 1]: dc_mask_rows' padding as its own launch (rows listed with pad_to 0
 * before the host knows the padded size) */
int dc_pad_rows(int* rows, const int* count, int pad_to, void* stream);

/* ---------------------------------------------------------------- AutoencoderKL (--vae original)
 * decode_prediction's vae.decode(z / scaling_factor) (marigold_dc.py:366 via diffusers) for the 4 latent
 * channels of a [P][ldx] bf16 row buffer -> y [P][8], and its backward chained into the Tweedie preview
 * (as dc_taesd_clamp_bwd does for TAESD's tanh clamp).  The VAE mid-block attention (1 head of C = 512
 * channels, diffusers Attention via SDPA) runs as dc_conv_gemm GEMMs around a row softmax:
 * dc_softmax_rows: P = softmax(S * scale) per row (columns >= cols of P zeroed up to ldp);
 * dc_softmax_rows_bwd: dS = P (dP - rowsum(P dP)) * scale; dc_transpose: y[c][r] = x[r][c], rows padded
 * with zeros up to ldy. */
int dc_latent_scale_fwd(const void* x, int ldx, long long pixels, float scale, void* y, void* stream);
int dc_latent_scale_bwd(const void* dy, int lddy, long long pixels, float scale, const float* coef, const int* step,
                        void* gx_direct, void* dv, void* stream);
int dc_softmax_rows(const void* s, int lds, long long rows, int cols, float scale, void* p, int ldp, void* stream);
int dc_softmax_rows_bwd(const void* p, int ldp, const void* dp, int lddp, long long rows, int cols, float scale,
                        void* ds, int ldds, void* stream);
int dc_transpose(const void* x, int ldx, int rows, int cols, void* y, int ldy, void* stream);

/* ---------------------------------------------------------------- evaluation (analyze.py)
 * One batch of analyze.py:233-290 (utils.mae / utils.rmse, utils.py:692-740): mask = sparse > 0, both maps
 * clamped to [min_depth, max_depth]; res[(1 + nbins)][3] = (sum |d - s|, sum (d - s)^2, count) overall and
 * per bin (bins[nbins][2] = lo, hi, inclusive, on the clamped sparse depth; utils.calc_bins).  dense /
 * sparse: fp32 device arrays of `total` elements; ws: dc_depth_metrics_ws_bytes() bytes. */
long long dc_depth_metrics_ws_bytes(void);
int dc_depth_metrics(const float* dense, const float* sparse, long long total, float min_depth, float max_depth,
                     const float* bins, int nbins, double* ws, double* res, void* stream);

/* ---------------------------------------------------------------- seed ensemble (BASELINE C5)
 * The S seeds of each frame run as S frames of one guided call (per-frame noise, dc_latent_init).
 * dense fp32 [frames*seeds][hw] frame-major (frame f's seeds are rows f*seeds ..), guide fp32 [frames][hw]
 * (metres, > 0 = valid).  out[f] = scale_f * mean_seeds(dense) + shift_f with (scale_f, shift_f) =
 * compute_affine_params(mean, guide, guide > 0) (marigold_dc.py:53-128; fp64 sums, same centring);
 * affine (optional) [frames][2] gets (scale, shift).  ws >= dc_ensemble_ws_bytes(frames, hw), 8-B aligned. */
long long dc_ensemble_ws_bytes(int frames, long long hw);
int dc_ensemble_fit(const float* dense, int frames, int seeds, long long hw, const float* guide, float* out,
                    float* affine, void* ws, long long ws_bytes, void* stream);


/* ---------------------------------------------------------------- host-side tables (CPU, shared by both hosts)
 * Computed on the CPU by the library so that the Python host and the native session feed the kernels the same
 * bits.  dc_schedule_tables: the DDIMScheduler of Marigold v1-0 (scaled_linear betas 0.00085..0.012, v_prediction,
 * set_alpha_to_one=False) with timestep_spacing="trailing" (predict.py:491-494; marigold_dc.py:800, 823-826,
 * 902-904): timesteps[steps] (int64), coef[steps][4] as for dc_preview, and adam[steps][4] as for
 * dc_latent_update (opt 0: torch.optim.Adam bias corrections, marigold_dc.py:783, 897; 1 / 2: [lr_lat, 0,
 * lr_aff, 0]).  dc_timestep_embedding: diffusers get_timestep_embedding(flip_sin_to_cos=True, shift 0), fp32
 * out[n][dim] (UNet2DConditionModel.time_proj, marigold_dc.py:459-465).  dc_fold_cross_attention: attn2 of a
 * BasicTransformerBlock with the constant 2-token empty-prompt context (marigold_dc.py:663-674) folded into
 * U[heads][c], D[heads][cout], c0[cout]; weights fp32 host arrays in diffusers layout. */
int dc_schedule_tables(int steps, double lr_latent, double lr_scaling, int opt, long long* timesteps, float* coef,
                       float* adam);
int dc_timestep_embedding(const long long* timesteps, int n, int dim, float* out);
int dc_fold_cross_attention(const float* wq, const float* wk, const float* wv, const float* wo, const float* bo,
                            const float* ctx, int ntok, int inner, int c, int cross, int cout, int heads, float* U,
                            float* D, float* c0);
/* dc_conv_pick: the dc_conv_gemm variant for a conv shape from a tuned table (tools/tune_gemm.py; both hosts call
 * it, so they launch the same variant).  keys[n][12] = (mode, nb, hin, win, cin, hout, wout, cout, kh, stride,
 * two_sources, ktot) in table order, choices[n][2] = (algo, splitk), key[12] the shape.  An exact match wins;
 * otherwise the nearest tuned shape with the same (mode, kh, stride, two_sources) in
 * 4 |log2 M - log2 M'| + |log2 N - log2 N'| + |log2 K - log2 K'| (M = nb hout wout, N = cout, K = ktot; first
 * in table order on ties).  out[2] = (algo, splitk); returns 0, or 1 when no entry qualifies (out = (0, 0): the
 * library heuristic). */
int dc_conv_pick(const int* keys, const int* choices, int n, const int* key, int* out);

/* ---------------------------------------------------------------- native session
 * The whole guided sampler behind an opaque handle, for hosts that are not Python: the same weight packing,
 * buffers and launch sequence as the Python pipeline (results equal bitwise), one guided step captured as a
 * hipGraph and replayed per timestep.  Replaces MarigoldDepthCompletionPipeline.from_pretrained + __call__
 * (predict.py:474-503, marigold_dc.py:467-985) for the predict.py default path: guided per-step optimisation
 * of the latents and the learned affine, l1 + l2 point losses, TAESD; norm const / minmax; any projection,
 * inv, interpolation and optimiser.  Every call returns a status; dc_session_error() gives the message (the
 * reference's ValueError text where one applies).  Tensors are device pointers: images uint8 [n][3][H][W],
 * sparse depth fp32 [n][1][H][W] (0 = missing), latents bf16 [n][4][h][w] (dc_latent_hw), noise bf16
 * [noise_n][4][h][w] (noise_n 1: one draw shared by every frame, as the reference draws it; n: per frame),
 * affine fp32 [n][2] (learned scale, shift), dense fp32 [n][1][H][W] metres.  `stream` orders the session's
 * work after the caller's and the caller's after the session's (the session launches on a stream of its own). */
typedef struct dc_session dc_session;
typedef struct dc_sample_params {
  float max_depth, min_depth;  /* (120, 0): predict.py:101-114 */
  int norm;                    /* 0 const, 1 minmax */
  int projection;              /* 0 linear, 1 log, 2 log10 */
  int inv;
  int interp;                  /* 0 bilinear, 1 nearest */
  int steps;                   /* DDIM steps (50) */
  int resolution;              /* processing resolution (768) */
  int opt;                     /* 0 Adam, 1 SGD, 2 Adagrad */
  double lr_latent, lr_scaling;  /* (0.05, 0.005) */
  float beta;                  /* warm start beta * noise + (1 - beta) * prev (0.9) */
  int use_graph;               /* 1: replay one captured guided step */
} dc_sample_params;
void dc_sample_params_default(dc_sample_params* p);
int dc_latent_hw(int H, int W, int resolution, int* h, int* w);
int dc_create(dc_session** out, int device);
int dc_destroy(dc_session* s);
const char* dc_session_error(const dc_session* s);
/* dir: unet/config.json + unet/diffusion_pytorch_model.safetensors, taesd/ (or vae/)
 * diffusion_pytorch_model.safetensors, empty_text_embedding.safetensors ("embedding" [1][2][cross]);
 * tuned_table: the GEMM variant table (depth_completion_amd/tuned_gfx950.json) or NULL (library heuristic) */
int dc_load_weights(dc_session* s, const char* dir, const char* tuned_table);
/* preprocess + TAESD encoder (marigold_dc.py:687-698) */
int dc_encode(dc_session* s, const void* imgs_u8, int n, int H, int W, int resolution, void* latents, void* stream);
/* the guided denoising loop (marigold_dc.py:661-909) from image latents; prev (may be NULL): pred_latents_prev */
int dc_guided_sample(dc_session* s, const void* img_latents, const void* noise, int noise_n, const void* prev,
                     const float* sparses, int n, int H, int W, const dc_sample_params* p, void* latents_out,
                     float* affine_out, void* stream);
/* final decode + learned-affine de-normalisation (marigold_dc.py:969-985) */
int dc_decode_dense(dc_session* s, const void* latents, const float* affine, const float* sparses, int n, int H,
                    int W, const dc_sample_params* p, float* dense_out, void* stream);
/* all of __call__ (encode + guided sample + final decode); latents_out may be NULL */
int dc_complete(dc_session* s, const void* imgs_u8, const float* sparses, int n, int H, int W, const void* noise,
                int noise_n, const void* prev, const dc_sample_params* p, float* dense_out, void* latents_out,
                void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DCAMD_H */
