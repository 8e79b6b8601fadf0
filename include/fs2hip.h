/* fs2hip.h — C-ABI of libfs2hip.so, the gfx950 (MI355X) kernels of the FastSpeech2 +
 * TacoSpawn-GMM training step.
 *
 * The reference (sarulab-speech/Mid-Attribute-Speaker-Generation) is pure PyTorch: it has no
 * FFI.  Each entry point below replaces a *sequence of ATen ops* of the reference's
 * `nn.Module`s; the citation on each names the reference lines it replaces
 * (paths relative to the reference root).  The Python host in
 * mid-attribute-speaker-generation_amd/ mirrors the reference module API on top of these.
 *
 * Conventions (all entry points):
 *   - plain device pointers, int64 sizes, a dtype enum where storage type varies,
 *     `stream` = hipStream_t (as void*), return 0 on success, <0 on error;
 *     `fs2_last_error()` describes the last failure of the calling thread.
 *   - no allocation, no host synchronisation: callers pass workspaces (size queries are
 *     provided), so every call can be captured into a hipGraph.
 *   - activations are (rows, channels) row-major = the reference's (B, T, C) layout;
 *     row r of a batch of sequences of length seq_len is frame r % seq_len of utterance
 *     r / seq_len.  Padding masks are given as per-utterance lengths (int64), a row being
 *     padding when (r % seq_len) >= lens[r / seq_len] (utils/tools.py:155-163).
 *   - dropout is counter-based (Philox4x32-10 keyed by seed, site, element index): the
 *     backward entry points regenerate the forward mask from the same (seed, site).  The
 *     seed is read from DEVICE memory (`const uint64_t* seed`, NULL when p == 0), so a
 *     captured HIP graph of the step draws a new seed per replay (fs2_seed_next).
 */
#ifndef FS2HIP_H
#define FS2HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { FS2_OK = 0, FS2_ERR_ARG = -1, FS2_ERR_LAUNCH = -2, FS2_ERR_DTYPE = -3 };
enum { FS2_F32 = 0, FS2_BF16 = 1 };
/* GEMM epilogue flags */
enum {
  FS2_EPI_BIAS = 1,          /* y += bias[n]                                   */
  FS2_EPI_RELU = 2,          /* y = max(y, 0)                                  */
  FS2_EPI_ADD_AUX = 4,       /* y += aux[m, n]   (residual-gradient fusion)    */
  FS2_EPI_RELU_MASK_AUX = 8, /* y *= (aux[m, n] > 0)   (ReLU backward fusion)  */
  FS2_EPI_OUT_BF16 = 16,     /* bf16 path: store y as bf16 (default fp32)       */
  FS2_EPI_AUX_BF16 = 32,     /* bf16 path: aux is bf16 (default fp32)           */
  /* fs2_conv_gemm_ex only (vocoder, hifigan/models.py), applied after BIAS / ADD_AUX:  */
  FS2_EPI_LRELU = 64,        /* y = y >= 0 ? y : alpha * y                      */
  FS2_EPI_ACC_Y = 128,       /* y = (y + y_old[m, n]) * scale  (y read, then written) */
  FS2_EPI_Y2 = 256,          /* y2[m, n] = y >= 0 ? y : alpha2 * y  (compute dtype) */
  FS2_EPI_SKIP_NOSTORE = 512 /* with lens: skipped row tiles store nothing (y, y2 keep their
                                contents there) -- for consumers that never read those rows */
};

const char* fs2_last_error(void);
int fs2_abi_version(void);

/* ---------------------------------------------------------------- convolution / linear
 * Conv1d over time as an implicit GEMM on (rows, c_in) activations:
 *   y[r, o] = sum_{j, c} wk[o, j*c_in + c] * x[r + j - pad, c]      (zero outside the utterance)
 * dtype FS2_F32: x, wk fp32 (exact f32 MFMA); FS2_BF16: x, wk bf16 (bf16 MFMA, fp32
 * accumulate), y fp32 or bf16 (FS2_EPI_OUT_BF16).
 * A Linear layer is taps=1, pad=0.  Forward uses wk = fs2_conv_weight_prep's w_fwd; the
 * data gradient is the same call on dy with w_bwd (flipped taps, transposed channels).
 * Replaces nn.Conv1d / nn.Linear forward and their input-gradient:
 *   transformer/SubLayers.py:39-41,53,85-89 ; model/modules.py:289-296 ;
 *   transformer/Layers.py:59-64 ; model/fastspeech2.py:25-28,109.
 * lens (nullable, device int64[rows / seq_len]): row r = b*seq_len + t is padding when
 * t >= lens[b].  With lens, output tiles made only of padding rows are not computed: they
 * are written as if their rows were zero and there were no bias (aux under ADD_AUX, 0
 * otherwise) -- for the FFT blocks, whose padded rows are masked (Layers.py:25,28) or carry
 * zero gradient.  fs2_conv_wgrad skips 64-row k-tiles made only of padding rows (their dy
 * rows must be zero).  The fp32 path ignores lens.                                     */
int fs2_conv_gemm(int dtype, const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                  int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps, int pad,
                  const int64_t* lens, const float* bias, int flags, const void* aux,
                  int64_t ld_aux, void* stream);

/* bf16 Conv1d / Linear with the FFT block's post-LayerNorm fused into the epilogue
 * (c_out = 256, the LayerNorm width; x, wk bf16 as fs2_conv_gemm):
 *   z[r, :] = dropout(conv(x)[r, :] + bias, p_in) + res[r, :]      (res nullable)
 *   out = (z - mean) * rstd * gamma + beta, out_t = bf16(out) (nullable), xhat, rstd saved;
 *   rows t >= lens[b] are written as 0 (xhat / rstd left unwritten there).
 * Bitwise equal to fs2_conv_gemm (fp32 y, FS2_EPI_BIAS) followed by fs2_ln_fwd(y, res, ...,
 * p_out = 0, no head): one kernel instead of two, and y never goes to memory.  The dropout
 * mask is fs2_ln_fwd's (seed, site_in), so fs2_ln_bwd is its backward.
 * Replaces transformer/SubLayers.py:54-55 (fc, dropout, residual, layer_norm) and :88-91
 * (w_2, dropout, residual, layer_norm).                                                  */
int fs2_conv_gemm_ln(const void* x, int64_t ldx, const void* wk, int64_t rows, int64_t seq_len,
                     int64_t c_in, int64_t c_out, int taps, int pad, const int64_t* lens,
                     const float* bias, const float* res, const float* gamma, const float* beta,
                     float* out, void* out_t, float* xhat, float* rstd, float p_in,
                     const uint64_t* seed, uint64_t site_in, void* stream);

/* bf16 Linear / Conv1d (c_out = 256) whose output is the upstream gradient of a post-
 * LayerNorm, with that LayerNorm's backward in the epilogue:
 *   dout[r, :] = conv(x)[r, :] + aux[r, :]                (aux: fp32 residual gradient, nullable)
 *   then fs2_ln_bwd(dout, xhat, rstd, gamma, ..., p_in, site_in, dres, dres_add, dy_t = the bf16
 *   dy copy, dgamma / dbeta / dbias_in accumulated; p_out = 0, no head, no ReLU input).
 * Against fs2_conv_gemm(FS2_EPI_ADD_AUX) followed by fs2_ln_bwd (the contract its test
 * checks): dres equal to fp32 rounding (the row arithmetic is compiled in another kernel and
 * contracted differently), the bf16 dy copy within 1 bf16 ulp, and the parameter gradients
 * summed from per-32-row block partials in another in-block order.
 * ws: fs2_ln_bwd_ws_bytes(rows, 256).  In the FFT-block backward x is the attention input
 * gradient (dqkv) and the LayerNorm is the PREVIOUS block's FFN post-LN: block i's QKV data
 * gradient and block i-1's first backward op in one launch (transformer/SubLayers.py:38-40,91). */
int fs2_conv_gemm_ln_bwd(const void* x, int64_t ldx, const void* wk, int64_t rows,
                         int64_t seq_len, int64_t c_in, int64_t c_out, int taps, int pad,
                         const int64_t* lens, const float* aux, const float* xhat,
                         const float* rstd, const float* gamma, float* dgamma, float* dbeta,
                         float* dbias_in, float p_in, const uint64_t* seed, uint64_t site_in,
                         float* dres, int dres_add, void* dy_t, float* ws, int64_t ws_bytes,
                         void* stream);

/* Dilated Conv1d with the vocoder epilogue (HiFi-GAN generator, hifigan/models.py:19-178):
 *   v[r, o] = sum_{j, c} wk[o, j*c_in + c] * x[r + j*dilation - pad, c]   (zero outside the
 *   utterance of seq_len rows), then BIAS, ADD_AUX, ACC_Y, LRELU in that order; y stored
 *   (skipped when y is NULL) and, with FS2_EPI_Y2, a second output y2 = leaky_relu(v, alpha2)
 *   in the compute dtype (bf16 for FS2_BF16, fp32 for FS2_F32; ld = c_out): the input copy
 *   of the next convolution (models.py:95-97,157,167).  pad <= (taps-1)*dilation.
 *   ConvTranspose1d(k = 2s, stride s, pad s/2) runs as taps=3, pad=1 over s*c_out phase
 *   columns (see fs2_convT_weight_prep).  lens (optional, device, one per utterance): as
 *   fs2_conv_gemm -- bf16 row tiles made only of rows t >= lens[b] skip the product (their
 *   outputs are the epilogue of a zero accumulator); rows t < lens[b] are exact.  The
 *   vocoder passes its valid length plus the network's receptive radius, so the kept samples
 *   equal the padded-batch result bitwise.  fs2_conv_gemm(...) == fs2_conv_gemm_ex(...,
 *   dilation 1, lens, alpha 0, scale 1, y2 NULL, alpha2 0).                              */
int fs2_conv_gemm_ex(int dtype, const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                     int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps, int pad,
                     int dilation, const int64_t* lens, const float* bias, int flags,
                     const void* aux, int64_t ld_aux, float alpha, float scale, void* y2,
                     float alpha2, void* stream);

/* ConvTranspose1d(c_in -> c_out, k = 2*stride, stride, padding = stride/2) weight
 * w (c_in, c_out, k) (hifigan/models.py:127-137) as the equivalent 3-tap Conv1d weight
 * wc (stride*c_out, c_in, 3) over input frames q-1, q, q+1 producing output samples
 * stride*q + ph (column ph*c_out + o):
 *   wc[ph*c_out + o, c, d+1] = w[c, o, ph + stride/2 - stride*d]  if that tap is in [0, k)
 * (else 0), and bias_c[ph*c_out + o] = bias[o].  Feed wc to fs2_conv_weight_prep.        */
int fs2_convT_weight_prep(const float* w, const float* bias, int64_t c_in, int64_t c_out,
                          int stride, float* wc, float* bias_c, void* stream);

/* Fused HiFi-GAN ResBlock1 (hifigan/models.py:21-53) for the narrow stages: one launch runs
 * the block's three (leaky_relu 0.1, dilated conv k, leaky_relu 0.1, conv k, residual add)
 * pairs on an LDS-resident row tile (R = 256 rows at 32 channels, 128 at 64) and folds the
 * stage's running average: v = acc ? (xs + out) * scale : out * scale; xs = v when store_xs;
 * hc = bf16(leaky_relu(v, alpha2)) when hc is given.  x (rows, C) fp32; w1 / w2: HOST arrays
 * of 3 device pointers to fs2_conv_weight_prep bf16 weights (C, k*C); b1 / b2: host arrays
 * of 3 fp32 bias pointers; dil: host array of 3 dilations.  seq_len % R == 0 (tiles inside
 * one utterance; zero padding at its edges as each Conv1d).  lens (optional): tiles made
 * only of rows t >= lens[b] store nothing.  fs2_resblock1_supported() returns 1 when a shape
 * qualifies (channels 32 / 64, receptive radius <= 64 rows), else 0 (not an error code). */
int fs2_resblock1_supported(int64_t channels, int64_t seq_len, int kernel_size, const int* dil);
int fs2_resblock1_fused(const void* x, int64_t rows, int64_t seq_len, int64_t channels,
                        int kernel_size, const int* dil, const void* const* w1,
                        const void* const* w2, const float* const* b1, const float* const* b2,
                        float* xs, int acc, float scale, int store_xs, void* hc, float alpha2,
                        const int64_t* lens, void* stream);

/* HiFi-GAN output head (hifigan/models.py:167-169, utils/model.py:74-90):
 *   wav[r] = tanh(bias + sum_{j<7, c} w[0, c, j] * x[r + j - 3, c])   (zero outside the
 *   utterance), x (rows, c_in) in the compute dtype; wav fp32 and, when pcm is not NULL,
 *   pcm[r] = (int16) (wav[r] * max_wav_value) truncated toward zero as numpy's astype.
 *   lens (optional, device, samples per utterance): rows t >= lens[b] are written as 0.     */
int fs2_vocoder_post(int dtype, const void* x, int64_t rows, int64_t seq_len, int64_t c_in,
                     const int64_t* lens, const float* w, const float* bias, float max_wav_value,
                     float* wav, int16_t* pcm, void* stream);

/* ---------------------------------------------------------------- language discriminator
 * The --use_clf branch (train.py:168-197): GE2E SpeechEmbedder (speech_embedder_net.py:65-162)
 * and GE2ELoss's BCE term (165-186), fp32.
 * One LSTM layer (nn.LSTM, batch_first, gates i,f,g,o, h0 = c0 = 0) over n_seq sequences of
 * `steps` rows (row n*steps + t): gx = x W_ih^T + bias (bias = b_ih + b_hh; one GEMM), then
 * the recurrence, one launch per step issued from C.  w_ih (4H, c_in) and w_hh (4H, H)
 * natural; hidden a multiple of 256.  Saves h_all, c_all (rows, H) and the activated gates
 * act (rows, 4H).                                                                         */
int fs2_lstm_layer_fwd(const float* x, int64_t n_seq, int64_t steps, int64_t c_in, int64_t hidden,
                       const float* w_ih, const float* bias, const float* w_hh, float* gx,
                       float* h_all, float* c_all, float* act, void* stream);
/* Backward through time: dh_out (rows, H; NULL = 0) is the gradient of the layer's outputs;
 * writes dgates (rows, 4H; pre-activation gate gradients) and, when dx is given,
 * dx = dgates W_ih (rows, c_in; w_ih_t = W_ih^T (c_in, 4H)); w_hh_t = W_hh^T (H, 4H).
 * dc_ws: 2*n_seq*H floats.
 * Weight gradients are not formed (train.py never steps the discriminator).            */
int fs2_lstm_layer_bwd(const float* dh_out, int64_t n_seq, int64_t steps, int64_t c_in,
                       int64_t hidden, const float* w_ih_t, const float* w_hh_t, const float* act,
                       const float* c_all, float* dgates, float* dc_ws, float* dx, void* stream);
/* The whole L-layer stack (the GE2E LSTM_stack, nn.LSTM(num_layers = L)) as a wavefront:
 * launch s runs layer l at step s - l, so the stack takes steps + L - 1 launches; the inputs
 * of layers >= 1 are folded into their step kernels.  Layer-major buffers: h_all, c_all
 * (L, rows, H), act (L, rows, 4H); weights w_ih0 (4H, c_in), w_ih_up (L-1, 4H, H) = W_ih of
 * layers 1.., w_hh (L, 4H, H), bias (L, 4H) = b_ih + b_hh; gx (rows, 4H) workspace.  Same
 * results as fs2_lstm_layer_fwd layer by layer, within fp32 summation order.              */
int fs2_lstm_stack_fwd(const float* x, int64_t n_seq, int64_t steps, int64_t c_in,
                       int64_t hidden, int layers, const float* w_ih0, const float* w_ih_up,
                       const float* w_hh, const float* bias, float* gx, float* h_all,
                       float* c_all, float* act, void* stream);
/* Backward of the stack: dh_out (rows, H; NULL = 0) is the top layer's output gradient;
 * writes dgates (L, rows, 4H) and, with dx, dx = dgates_0 W_ih0 (rows, c_in).  Transposed
 * weights: w_ih0_t (c_in, 4H), w_ih_up_t (L-1, H, 4H), w_hh_t (L, H, 4H).
 * dc_ws: L * 2 * n_seq * H floats.                                                      */
int fs2_lstm_stack_bwd(const float* dh_out, int64_t n_seq, int64_t steps, int64_t c_in,
                       int64_t hidden, int layers, const float* w_ih0_t, const float* w_ih_up_t,
                       const float* w_hh_t, const float* act, const float* c_all, float* dgates,
                       float* dc_ws, float* dx, void* stream);
/* Embedding + domain-classifier head on the last LSTM frame (x row n at x + n*ldx, 256 wide):
 * projection 256->64, L2 norm (emb), Linear 64->64, dropout, ReLU, Linear 64->64, dropout,
 * ReLU, Linear 64->1 (logit).  w*t are the transposed weights (forward), w* the natural
 * ones (backward).  With dx: dx = d(head)/dx for the given demb / dlogit (NULL = 0), the
 * dropout masks regenerated from (seed, site).                                           */
int fs2_clf_head(const float* x, int64_t ldx, int64_t n, const float* wp, const float* wpt,
                 const float* bp, const float* w0, const float* w0t, const float* b0,
                 const float* w1, const float* w1t, const float* b1, const float* w2,
                 const float* b2, float p_drop, const uint64_t* seed, uint64_t site, float* emb,
                 float* logit, const float* demb, const float* dlogit, float* dx, int64_t lddx,
                 void* stream);
/* BCEWithLogits per row (loss_rows, nullable) and dlogit = g[0] * scale * (sigmoid - y)
 * (g nullable = 1).                                                                      */
int fs2_bce_logits(const float* logit, const float* y, int64_t n, float* loss_rows,
                   const float* g, float scale, float* dlogit, void* stream);
/* (batch, t_src, c) rows -> (batch, t_dst, c): copy the first min(t_src, t_dst) frames,
 * zero the rest (the 150-frame chunking of train.py:178-183 and its gradient).          */
int fs2_rows_repad(const float* src, int64_t batch, int64_t t_src, int64_t t_dst, int64_t c,
                   float* dst, void* stream);
/* y[b*rep + k] = meta[b*ld + col] (per-chunk language labels, train.py:184).             */
int fs2_repeat_col(const float* meta, int64_t batch, int64_t ld, int col, int rep, float* y,
                   void* stream);

/* Weight re-layout (and cast for bf16) of a (c_out, c_in, taps) fp32 master weight:
 *   w_fwd[o, j*c_in + c]        = w[o, c, j]
 *   w_bwd[c, j*c_out + o]       = w[o, c, taps-1-j]      (either output may be NULL)     */
int fs2_conv_weight_prep(int dtype, const float* w, int64_t c_out, int64_t c_in, int taps,
                         void* w_fwd, void* w_bwd, void* stream);
/* The same for every layer of the model in one launch: jobs (device, int64) holds
 * n_jobs rows {w, c_out, c_in, taps, w_fwd, w_bwd, first, end}: the job's tiles
 * [first, end) of ceil(c_out/64) * ceil(c_in/CT) tiles, numbered consecutively over the
 * jobs, CT = fs2_weight_prep_tile_channels(dtype); n_tiles = end of the last job; taps <= 9. */
int fs2_weight_prep_tile_channels(int dtype);
int fs2_weight_prep_batch(int dtype, const int64_t* jobs, int n_jobs, int64_t n_tiles,
                          void* stream);

/* Kernel-selection knobs for benchmarking (0 = automatic choice, the default).  Variants that
 * measured slower or neutral were removed in round 4 (their A/B records stay in profiles/):
 *   FS2_TUNE_GEMM_STAGES   fwd/dX LDS stages (1..4) of the tap-major kernel
 *   FS2_TUNE_WGRAD_STAGES  weight-gradient LDS stages (1..4) of the tap-major wgrad kernel
 *   FS2_TUNE_WGRAD_TILE    weight-gradient tile width (64 or 128) of the tap-major wgrad kernel
 *   FS2_TUNE_WGRAD_SPLITS  weight-gradient row splits (1..64) of the split-K wgrad kernels
 *   FS2_TUNE_LEGACY_GEMM   1 = the register-staged bf16 kernels of round 1 (A/B against round 1)
 *   FS2_TUNE_NT_GROUP      fwd/dX n-tiles per L2 tile group
 *   FS2_TUNE_NT_HALO       fwd/dX Conv1d (taps > 1) halo kernel: 0 = automatic (8-wave 256 x 128
 *                          tiles for the wide c_in <= 256 forward shapes, else 4-wave tiles by
 *                          grid size), 1 = 4-wave tiles only, 2 = force 128-wide 4-wave tiles,
 *                          -1 = off (tap-major kernel)
 *   FS2_TUNE_WGRAD_HALO    weight gradient of Conv1d taps 3/5/9: 0 = the slab-free band kernel
 *                          where its 32 x 32 output tiles fill the chip, else the split-K halo
 *                          kernel (default), 1 = the split-K halo kernel, -1 = tap-major kernel
 *   FS2_TUNE_HALO_SPLITK   64x64 halo fwd/dX on an under-filled grid (long-K encoder data
 *                          gradient): 0 = automatic channel-block split (128x64 tiles when
 *                          T % 128 == 0), -1 = off, -2 = 64x64 tiles only, n = n splits
 *   FS2_TUNE_ATTN          bf16 attention: 0 = two 16-row groups per wave in the forward
 *                          and dQ (delta fused) kernels at T >= 256, one 16-key group per wave
 *                          at two workgroups per CU in dK/dV (automatic), -1 = one group
 *                          everywhere, 1 = as 0 with the one-workgroup-per-CU dK/dV build,
 *                          2 = two groups in dK/dV too, 3 = dK/dV at three workgroups per CU
 *   FS2_TUNE_NT_TILE       tap-major fwd/dX kernel (k = 1 projections, odd shapes): 0 = tile
 *                          by grid size, 1 / 2 / 3 = force 128x128 / 128x64 / 64x64
 *   FS2_TUNE_LN_TILE       fs2_conv_gemm_ln(_bwd) row tile: 0 = 64 x 256 (default), 1 = 128 x 256
 *   FS2_TUNE_WGRAD_K1      k = 1 weight gradient: 0 = the grouped split-K kernel of
 *                          fs2_conv_wgrad_k1_multi with one job (default), -1 = the tap-major kernel
 *   FS2_TUNE_NT_K1         k = 1 projections on the tap-major kernel: 0 = buffer-descriptor
 *                          staging build (default), -1 = the general tap-walking build (A/B)
 *   FS2_TUNE_ATTN_DMA      bf16 attention at T >= 256: 0 = K / V (Q / dO) tiles by LDS-DMA into
 *                          a 2-slot ring, exp2-folded softmax (default), 1 = 3-slot forward ring
 *                          at one workgroup per CU, -1 = the register-staged kernels (A/B)
 *   FS2_TUNE_TAPREG        fwd/dX Conv1d taps 5 / 9 (C_in % 64 == 0, T and rows % 128 == 0):
 *                          0 = the tap-register halo kernel where its grid fills the chip
 *                          (default: 4-wave 128 x 64 tiles at 3 blocks per CU, 128 x 128 at 2 for
 *                          c_out <= 256), -1 = off (the halo kernels above), 1 = force the
 *                          128 x 64 tiles, 3 = force 128 x 128
 *   FS2_TUNE_WGRAD_BAND    band weight gradient (taps 9, and taps 3 / 5 whose channels are not
 *                          64-multiples): 0 = default, 3 = only on grids of >= 128 tiles,
 *                          4 = the band kernel for taps 3 / 5 with 64-multiple channels too
 *   FS2_TUNE_ATTN_XCD      LDS-DMA attention kernels: 0 = the blocks of one (utterance, head) on
 *                          one XCD (K / V reuse in its L2; default), -1 = the launch grid's order
 *   FS2_TUNE_WGRAD_K1M_STAGES  grouped k = 1 weight gradient LDS ring: 0 = 4 slots, 2 / 3 slots
 *   FS2_TUNE_WGRAD_WIDE    weight gradient of Conv1d taps 3/5/9 (T % 64 == 0) on the wide-tile
 *                          kernel (64 x 64 x taps tiles, row splits to ~256 blocks): 0 = where a
 *                          channel count is not a 64-multiple (default), 1 = wherever eligible,
 *                          -1 = off (band / split-K halo kernels), n > 1 = everywhere, n splits
 * Process-wide; query workspace sizes after setting.                                 */
enum { FS2_TUNE_GEMM_STAGES = 0, FS2_TUNE_WGRAD_STAGES = 1, FS2_TUNE_WGRAD_TILE = 2,
       FS2_TUNE_WGRAD_SPLITS = 3, FS2_TUNE_LEGACY_GEMM = 4, FS2_TUNE_NT_GROUP = 5,
       FS2_TUNE_NT_HALO = 6, FS2_TUNE_WGRAD_HALO = 7, FS2_TUNE_HALO_SPLITK = 8,
       FS2_TUNE_ATTN = 9, FS2_TUNE_NT_TILE = 10, FS2_TUNE_LN_TILE = 11, FS2_TUNE_WGRAD_K1 = 12,
       FS2_TUNE_NT_K1 = 13, FS2_TUNE_ATTN_DMA = 14, FS2_TUNE_TAPREG = 15,
       FS2_TUNE_WGRAD_BAND = 16, FS2_TUNE_ATTN_XCD = 17, FS2_TUNE_WGRAD_K1M_STAGES = 18,
       FS2_TUNE_WGRAD_WIDE = 19, FS2_TUNE_COUNT = 20 };
int fs2_set_tuning(int knob, int value);

/* ---------------------------------------------------------------- one FFT block per call
 * transformer/Layers.py:21-30 (FFTBlock.forward: MultiHeadAttention SubLayers.py:29-57, then
 * PositionwiseFeedForward SubLayers.py:85-93, post-LN, padded rows masked) and its backward,
 * bf16, issued from C: the same entry points in the same order as the per-kernel host path
 * (model.FFTBlock.fwd / bwd), so the results are bitwise those.  `blk` is a host int64 table of
 * FS2_FB_WORDS words (pointers as integers): geometry, the bf16 compute-layout weights
 * (fs2_conv_weight_prep: QKV fused as one (3 h d_k, d) Linear), the fp32 biases / LayerNorm
 * affines, and the fp32 gradient buffers they accumulate into.                               */
enum { FS2_FB_D = 0, FS2_FB_HEADS, FS2_FB_DK, FS2_FB_DINNER, FS2_FB_TAPS, FS2_FB_PAD, FS2_FB_SITE,
       FS2_FB_WQKV_F, FS2_FB_WQKV_B, FS2_FB_BQKV, FS2_FB_WFC_F, FS2_FB_WFC_B, FS2_FB_BFC,
       FS2_FB_W1_F, FS2_FB_W1_B, FS2_FB_B1, FS2_FB_W2_F, FS2_FB_W2_B, FS2_FB_B2,
       FS2_FB_LN1_G, FS2_FB_LN1_B, FS2_FB_LN2_G, FS2_FB_LN2_B,
       FS2_FB_GQKV_W, FS2_FB_GQKV_B, FS2_FB_GFC_W, FS2_FB_GFC_B, FS2_FB_G1_W, FS2_FB_G1_B,
       FS2_FB_G2_W, FS2_FB_G2_B, FS2_FB_GLN1_G, FS2_FB_GLN1_B, FS2_FB_GLN2_G, FS2_FB_GLN2_B,
       FS2_FB_WORDS };
enum { FS2_FA_X2 = 0, FS2_FA_X2_T = 1 };
/* Forward: x (rows, d) fp32 residual stream and its bf16 copy x_t -> the activation region
 * `act` (fs2_fft_block_act_bytes; saved for the backward) whose FS2_FA_X2 / FS2_FA_X2_T
 * tensors (byte offsets: fs2_fft_block_act_offset) are the block output and its copy.
 * fuse_ln: the post-LNs in the fc / w_2 GEMM epilogues (fs2_conv_gemm_ln).  p: dropout rate
 * (0 = off), seed device int64[1].                                                          */
int64_t fs2_fft_block_act_bytes(const int64_t* blk, int64_t rows, int64_t batch, int64_t seq_len,
                                int fuse_ln);
int64_t fs2_fft_block_act_offset(const int64_t* blk, int64_t rows, int64_t batch,
                                 int64_t seq_len, int fuse_ln, int which);
int fs2_fft_block_fwd(const int64_t* blk, const float* x, const void* x_t, void* act, int64_t rows,
                      int64_t batch, int64_t seq_len, const int64_t* lens, float p,
                      const uint64_t* seed, int fuse_ln, void* stream);
/* Backward from dx2 (the output gradient) or from (carry_dy2_t, carry_dx1), the block's LN2
 * backward already done by the following block.  dx (rows, d) fp32: the input gradient, or,
 * with prev_blk (the block before this one, its act region), that block's LN2 backward runs in
 * this block's QKV data-gradient epilogue (fs2_conv_gemm_ln_bwd) and writes prev_dy2_t (bf16)
 * / prev_dx1 (fp32) -- its carry -- instead (dx is then scratch).  tmp: fs2_fft_block_tmp_bytes.
 * The weight gradients run on side_stream (NULL: stream) with side_ws
 * (>= fs2_fft_block_side_ws_bytes); act, tmp and the carry buffers are read there after the
 * call returns: keep them until that stream is joined.                                      */
int64_t fs2_fft_block_tmp_bytes(const int64_t* blk, int64_t rows, int64_t batch, int64_t seq_len);
int64_t fs2_fft_block_side_ws_bytes(const int64_t* blk, int64_t rows);
int fs2_fft_block_bwd(const int64_t* blk, void* act, const void* x_t, int fuse_ln, float p,
                      const float* dx2, const void* carry_dy2_t, float* carry_dx1,
                      const int64_t* prev_blk, void* prev_act, int prev_fuse_ln, float prev_p,
                      void* tmp, float* dx, void* prev_dy2_t, float* prev_dx1, int64_t rows,
                      int64_t batch, int64_t seq_len, const int64_t* lens, const uint64_t* seed,
                      float* side_ws, int64_t side_ws_bytes, void* stream, void* side_stream);

/* ---------------------------------------------------------------- mel head per call
 * model/fastspeech2.py:91-93 (mel_linear, then postnet(output) + output; PostNet
 * transformer/Layers.py:67-137: Conv1d(k) + BatchNorm1d (batch statistics, running update,
 * num_batches_tracked), tanh on all but the last, dropout) and its backward, bf16, issued from C
 * in the order of model.MelHeadFn / PostNet (bitwise those).  `mh` is a host int64 table of
 * FS2_MH_WORDS words: geometry, mel_linear's bf16 compute-layout weights, fp32 bias and
 * gradient buffers, then FS2_MHL_WORDS words per PostNet layer.                             */
enum { FS2_MH_NMEL = 0, FS2_MH_DIN, FS2_MH_DIM, FS2_MH_TAPS, FS2_MH_PAD, FS2_MH_LAYERS, FS2_MH_SITE,
       FS2_MH_LIN_WF, FS2_MH_LIN_WB, FS2_MH_LIN_B, FS2_MH_GLIN_W, FS2_MH_GLIN_B, FS2_MH_LAYER0 };
enum { FS2_MHL_W_F = 0, FS2_MHL_W_B, FS2_MHL_B, FS2_MHL_BN_G, FS2_MHL_BN_B, FS2_MHL_BN_RM,
       FS2_MHL_BN_RV, FS2_MHL_BN_NBT, FS2_MHL_GW, FS2_MHL_GB, FS2_MHL_GBN_G, FS2_MHL_GBN_B,
       FS2_MHL_WORDS };
enum { FS2_MH_MAX_LAYERS = 8, FS2_MH_WORDS = FS2_MH_LAYER0 + FS2_MH_MAX_LAYERS * FS2_MHL_WORDS };
enum { FS2_MHA_OUT = 0, FS2_MHA_POST = 1 };
/* Forward: x_t (rows, d_in) bf16 decoder output -> act (fs2_mel_head_act_bytes) holding the
 * mel_linear output (FS2_MHA_OUT) and postnet(out) + out (FS2_MHA_POST), fp32 (rows, n_mel),
 * byte offsets from fs2_mel_head_act_offset.  Backward from d_out and / or d_post (either may be
 * NULL, not both): dx (rows, d_in) fp32 is written; tmp: fs2_mel_head_tmp_bytes; weight
 * gradients on side_stream with side_ws (>= fs2_mel_head_side_ws_bytes), reading act / tmp /
 * x_t after the call returns: keep them until that stream is joined.                       */
int64_t fs2_mel_head_act_bytes(const int64_t* mh, int64_t rows);
int64_t fs2_mel_head_act_offset(const int64_t* mh, int64_t rows, int which);
int64_t fs2_mel_head_tmp_bytes(const int64_t* mh, int64_t rows);
int64_t fs2_mel_head_side_ws_bytes(const int64_t* mh, int64_t rows);
int fs2_mel_head_fwd(const int64_t* mh, const void* x_t, void* act, int64_t rows, int64_t seq_len,
                     float p, const uint64_t* seed, void* stream);
int fs2_mel_head_bwd(const int64_t* mh, void* act, const void* x_t, const float* d_out,
                     const float* d_post, void* tmp, float* dx, int64_t rows, int64_t seq_len,
                     float p, const uint64_t* seed, float* side_ws, int64_t side_ws_bytes,
                     void* stream, void* side_stream);

/* ---------------------------------------------------------------- variance predictor per call
 * model/modules.py:197-250 (2 x (Conv1d(k) -> ReLU -> LayerNorm -> dropout) -> Linear(., 1),
 * padded rows masked to 0) and its backward, bf16, in the order of model.VariancePredictor.fwd
 * / .bwd (bitwise those).  `vp`: host int64 table of FS2_VP_WORDS words.  Forward: x_t (rows,
 * d) bf16 -> act (fs2_variance_predictor_act_bytes) whose FS2_VPA_PRED tensor is the (rows,)
 * fp32 prediction.  Backward from dpred (rows,) fp32: the input gradient is ADDED into dx_acc
 * (rows, d) fp32; tmp / side_ws / side_stream as the mel head.                              */
enum { FS2_VP_D = 0, FS2_VP_FILTER, FS2_VP_TAPS, FS2_VP_PAD1, FS2_VP_PAD2, FS2_VP_SITE,
       FS2_VP_W1_F, FS2_VP_W1_B, FS2_VP_B1, FS2_VP_LN1_G, FS2_VP_LN1_B,
       FS2_VP_W2_F, FS2_VP_W2_B, FS2_VP_B2, FS2_VP_LN2_G, FS2_VP_LN2_B, FS2_VP_LIN_W, FS2_VP_LIN_B,
       FS2_VP_G1_W, FS2_VP_G1_B, FS2_VP_GLN1_G, FS2_VP_GLN1_B, FS2_VP_G2_W, FS2_VP_G2_B,
       FS2_VP_GLN2_G, FS2_VP_GLN2_B, FS2_VP_GLIN_W, FS2_VP_GLIN_B, FS2_VP_WORDS };
enum { FS2_VPA_PRED = 0 };
int64_t fs2_variance_predictor_act_bytes(const int64_t* vp, int64_t rows);
int64_t fs2_variance_predictor_act_offset(const int64_t* vp, int64_t rows, int which);
int64_t fs2_variance_predictor_tmp_bytes(const int64_t* vp, int64_t rows);
int64_t fs2_variance_predictor_side_ws_bytes(const int64_t* vp, int64_t rows);
int fs2_variance_predictor_fwd(const int64_t* vp, const void* x_t, void* act, int64_t rows,
                               int64_t seq_len, const int64_t* lens, float p, const uint64_t* seed,
                               void* stream);
int fs2_variance_predictor_bwd(const int64_t* vp, void* act, const void* x_t, const float* dpred,
                               void* tmp, float* dx_acc, int64_t rows, int64_t seq_len,
                               const int64_t* lens, float p, const uint64_t* seed, float* side_ws,
                               int64_t side_ws_bytes, void* stream, void* side_stream);

/* Stand-in for one gradient all-reduce of the data-parallel step, for pricing the collective
 * schedule at N ranks on one GPU (train.CollectiveModel; not on the training path):
 * `blocks` workgroups read and write back `bytes` of buf[0..n) (values unchanged), paced to
 * last duration_ns -- a ring all-reduce's CU occupancy, HBM traffic and duration without the
 * interconnect.  Replaces no reference code (the reference's only collective is
 * nn.DataParallel, train.py:67-68). */
int fs2_collective_standin(float* buf, int64_t n, int64_t bytes, int blocks, int64_t duration_ns,
                           void* stream);

/* Weight (and optionally bias) gradient, accumulated into the fp32 master-gradient layout:
 *   dw[o, c, j] += sum_r dy[r, o] * x[r + j - pad, c]
 *   db[o]       += sum_r dy[r, o]                          (db may be NULL)
 * bf16, taps 3 / 5 / 9, T % 64 == 0: 64 x 64 x taps output tiles shared by 8 waves, the rows
 * split into ~256 / tiles ranges whose fp32 slabs in `ws` are summed in split order; other
 * shapes: split-K slabs with an in-order reduction.  Bitwise reproducible for the same inputs
 * AND the same lens: with lens, 64-row bands / k-tiles made only of rows past each length
 * are skipped, which changes which split sums which rows (results then agree to fp32
 * rounding with the lens-free call on zero padding rows, not bitwise).
 * `ws_bytes` >= fs2_conv_wgrad_ws_bytes(...).
 * Replaces the weight/bias half of ConvolutionBackward / AddmmBackward.                */
int64_t fs2_conv_wgrad_ws_bytes(int64_t rows, int64_t c_in, int64_t c_out, int taps);
int fs2_conv_wgrad(int dtype, const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                   float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                   int pad, const int64_t* lens, float* ws, int64_t ws_bytes, void* stream);

/* Several k = 1 weight gradients over the same rows in one launch (+ one split reduce):
 * for each job j of `jobs` (HOST memory, n_jobs <= 4 rows of 8 int64:
 * {dy, ldy, x, ldx, dw, db, c_in, c_out}, pointers as integers, db may be 0)
 *   dw_j[o, c] += sum_r dy_j[r, o] * x_j[r, c],   db_j[o] += sum_r dy_j[r, o].
 * The FFT block's QKV, fc and w_2 weight gradients (SubLayers.py:39-55,88) run as one grid;
 * lens (optional): 64-row k-tiles made only of padding rows are skipped.  Fixed reduction
 * order (bitwise reproducible).  ws_bytes >= fs2_conv_wgrad_k1_multi_ws_bytes(...).           */
int64_t fs2_conv_wgrad_k1_multi_ws_bytes(const int64_t* jobs, int n_jobs, int64_t rows);
int fs2_conv_wgrad_k1_multi(int dtype, const int64_t* jobs, int n_jobs, int64_t rows,
                            int64_t seq_len, const int64_t* lens, float* ws, int64_t ws_bytes,
                            void* stream);

/* Column sums (bias / LayerNorm-affine / BatchNorm gradients):
 *   out[c] (+)= sum_r x[r, c]   in a fixed order (partials in ws, then in-order sum).   */
int64_t fs2_colsum_ws_bytes(int64_t rows, int64_t cols);
int fs2_colsum(int dtype, const void* x, int64_t ldx, int64_t rows, int64_t cols, float* out,
               int accumulate, float* ws, int64_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- attention
 * Fused key-padding-masked softmax attention over the packed projection buffer
 * qkv (rows, 3*heads*d_head) = [Q | K | V], head h at column block h (SubLayers.py:39-52,
 * Modules.py:14-25: scores / temperature -> masked_fill(-inf) -> softmax -> @V).
 * o (rows, heads*d_head) in the reference's (B, T, h*d_v) order; lse (batch*heads, seq_len)
 * is saved for the backward.  scale = 1/temperature.  Only d_head = 128 is supported.   */
int fs2_attn_fwd(int dtype, const void* qkv, void* o, float* lse, const int64_t* lens,
                 int64_t batch, int64_t seq_len, int heads, int d_head, float scale, void* stream);
/* d_qkv (rows, 3*heads*d_head) = gradient of the packed projections.
 * ws_bytes >= fs2_attn_bwd_ws_bytes(batch, seq_len, heads).                            */
int64_t fs2_attn_bwd_ws_bytes(int64_t batch, int64_t seq_len, int heads);
int fs2_attn_bwd(int dtype, const void* qkv, const void* o, const void* d_o, const float* lse,
                 void* d_qkv, const int64_t* lens, int64_t batch, int64_t seq_len, int heads,
                 int d_head, float scale, float* ws, int64_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- LayerNorm family
 * Row LayerNorm (d = 256) with the fusions of the reference's call sites:
 *   z   = dropout(y; p_in, site_in) + res          (res may be NULL)
 *   u   = LN(z) * gamma + beta                      (eps 1e-5)
 *   out = padded(row) ? 0 : dropout(u; p_out, site_out)
 * and optionally a per-row dot with a Linear(256 -> 1): dot_out[r] = padded ? 0 : out.w + b.
 *   SubLayers.py:54-55,91-93 + Layers.py:25,28   (p_in = dropout, res = residual, masked)
 *   model/modules.py:209-250                      (p_out = dropout, dot = linear_layer)
 * xhat/rstd are saved for the backward (not written for masked rows outside dot mode,
 * whose backward is zero).  out_t: optional extra copy in `dtype`.                    */
int fs2_ln_fwd(int dtype, const float* y, const float* res, const float* gamma, const float* beta,
               float* out, void* out_t, float* xhat, float* rstd, const int64_t* lens,
               int64_t seq_len, int64_t rows, int d, float p_in, float p_out,
               const uint64_t* seed, uint64_t site_in, uint64_t site_out, const float* dot_w,
               const float* dot_b,
               float* dot_out, void* stream);
/* Backward of fs2_ln_fwd.  Upstream gradient is dout (per element) or, in dot mode,
 * ddot (per row).  Produces dy (gradient w.r.t. y before dropout, times (relu_y > 0) when
 * relu_y != NULL), optionally adds dz into dres (dres_add 1: +=, 0: =), and accumulates dgamma, dbeta and
 * (dot mode) dw_dot/db_dot into fp32 gradients; dbias_in (nullable) += sum over rows of
 * dy — the bias gradient of the layer that produced y, fused here instead of a separate
 * column sum.  dy may be NULL when the dtype copy dy_t is requested.
 * ws >= fs2_ln_bwd_ws_bytes(rows, d).                                                 */
int64_t fs2_ln_bwd_ws_bytes(int64_t rows, int d);
int fs2_ln_bwd(int dtype, const float* dout, const float* ddot, const float* dot_w,
               const float* xhat, const float* rstd, const float* gamma, const float* beta,
               const int64_t* lens, int64_t seq_len, int64_t rows, int d, float p_in, float p_out,
               const uint64_t* seed, uint64_t site_in, uint64_t site_out, const float* relu_y,
               float* dy,
               void* dy_t, float* dres, int dres_add, float* dgamma, float* dbeta, float* dw_dot,
               float* db_dot, float* dbias_in, float* ws, int64_t ws_bytes, void* stream);
/* The parameter-gradient half of fs2_ln_bwd on its own: fs2_ln_bwd called with dgamma, dbeta,
 * dw_dot, db_dot and dbias_in all NULL leaves its per-block partial sums in ws; this sums
 * them into the given gradients (+=, fixed order) -- e.g. on another stream, off the data-
 * gradient chain.  has_ddot: fs2_ln_bwd was called with ddot (the dw_dot / db_dot partials
 * exist).  ws must hold fs2_ln_bwd's partials of the same rows.                          */
int fs2_ln_bwd_final(int64_t rows, int d, const float* ws, int has_ddot, float* dgamma,
                     float* dbeta, float* dw_dot, float* db_dot, float* dbias_in, void* stream);

/* ---------------------------------------------------------------- BatchNorm (PostNet)
 * Training-mode BatchNorm1d over all rows (padded frames included) + optional tanh +
 * dropout (transformer/Layers.py:129-137).  Stats in one pass: per 64-row block its column
 * sum and centred second moment, combined exactly (M2 = sum_b [M2_b + n_b (mean_b - mean)^2])
 * in a fixed order; running stats updated with momentum, unbiased variance.  c % 8 == 0;
 * fs2_bn_bwd also c <= 4096.  ws: fs2_bn_ws_bytes(rows, c) bytes, for either call.
 * out / dz may be NULL when the bf16 copy (out_t / dz_t) is requested.               */
int64_t fs2_bn_ws_bytes(int64_t rows, int64_t c);
int fs2_bn_fwd(int dtype, const float* z, int64_t rows, int64_t c, const float* gamma,
               const float* beta, float eps, float momentum, float* running_mean,
               float* running_var, float* mean, float* rstd, int act_tanh, float p,
               const uint64_t* seed, uint64_t site, const float* res, float* out, void* out_t,
               float* ws,
               int64_t ws_bytes, int64_t* num_batches_tracked, void* stream);
/* (num_batches_tracked: nullable device int64, incremented with the running statistics --
 *  BatchNorm1d's counter update, Layers.py:129-137, without a launch of its own.)        */
/* Eval-mode BatchNorm1d (transformer/Layers.py:129-137 under model.eval()): normalise with
 * the running statistics, no dropout, no statistics update; mean / rstd (c floats each)
 * receive running_mean and 1/sqrt(running_var + eps).                                 */
int fs2_bn_eval_fwd(int dtype, const float* z, int64_t rows, int64_t c, const float* gamma,
                    const float* beta, float eps, const float* running_mean,
                    const float* running_var, float* mean, float* rstd, int act_tanh,
                    const float* res, float* out, void* out_t, void* stream);
int fs2_bn_bwd(int dtype, const float* dout, const float* z, const float* mean, const float* rstd,
               const float* gamma, const float* beta, int64_t rows, int64_t c, int act_tanh,
               float p, const uint64_t* seed, uint64_t site, float* dz, void* dz_t,
               float* dgamma,
               float* dbeta, float* ws, int64_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- embeddings, adaptor
 * Encoder input: word_emb[text] + accent_emb[accent] + posenc[t] (transformer/Models.py:101-103). */
int fs2_encoder_embed_fwd(const int64_t* texts, const int64_t* accents, const float* word_emb,
                          const float* accent_emb, const float* posenc, int64_t batch,
                          int64_t seq_len, int d, float* out, void* out_t, void* stream);
/* out[i] = table[ids[i]]  (nn.Embedding lookup, e.g. speaker_emb, fastspeech2.py:81).  */
int fs2_embedding_fwd(const int64_t* ids, const float* table, int64_t n, int d, float* out,
                      void* stream);
/* mask[b, t] = t >= lens[b]  (get_mask_from_lengths, utils/tools.py:155-163), 1 byte.   */
int fs2_length_mask(const int64_t* lens, int64_t batch, int64_t max_len, uint8_t* mask,
                    void* stream);
/* dtable[ids[i]] += dout[i]  for ids[i] != padding_idx (padding_idx < 0: none); dtable
 * has n_table rows.  Fixed summation order (chunk partials in ws, no atomics).
 * ws_bytes >= fs2_embedding_bwd_ws_bytes(n, d, n_table) (also for fs2_bucket_embed_bwd). */
int64_t fs2_embedding_bwd_ws_bytes(int64_t n, int d, int64_t n_table);
int fs2_embedding_bwd(const float* dout, const int64_t* ids, int64_t n, int d, int padding_idx,
                      float* dtable, int64_t n_table, float* ws, int64_t ws_bytes, void* stream);
/* out[b, t] = x[b, t] + table[ids[b]] over all t (model/fastspeech2.py:81-84).        */
int fs2_rowvec_add_fwd(const float* x, const int64_t* ids, const float* table, int64_t batch,
                       int64_t seq_len, int d, float* out, void* out_t, void* stream);
int fs2_rowvec_add_bwd(const float* dout, const int64_t* ids, int64_t batch, int64_t seq_len,
                       int d, float* dtable, void* stream);
/* out = x + table[bucketize(values, bins)] (model/modules.py:80-100, torch.bucketize
 * right=False: #bins < v).  values_dtype: FS2_F32 or 2 = f64.  idx (int32) saved.     */
int fs2_bucket_embed_fwd(const float* x, const void* values, int values_dtype, const float* bins,
                         int n_bins, const float* table, int64_t rows, int d, float* out,
                         void* out_t, int32_t* idx, void* stream);
int fs2_bucket_embed_bwd(const float* dout, const int32_t* idx, int64_t rows, int d,
                         float* dtable, int64_t n_table, float* ws, int64_t ws_bytes, void* stream);
int fs2_bucketize(const void* values, int values_dtype, const float* bins, int n_bins,
                  int64_t n, int32_t* idx, void* stream);

/* LengthRegulator (model/modules.py:161-194, utils/tools.py:363-381).
 * fs2_lr_index: cum[b, i] = inclusive scan of max(trunc(d), 0); mel_len[b] = cum[b, Ts-1]
 * (uncropped).  dur_dtype: 0 = int64, 1 = f32.                                       */
int fs2_lr_index(const void* durations, int dur_dtype, int64_t batch, int64_t src_len,
                 int32_t* cum, int64_t* mel_len, void* stream);
/* Inference durations (model/modules.py:132-135):
 * out = clamp(round_half_even(exp(log_d) - 1) * d_control, min = 0), f32 (NaN propagates). */
int fs2_duration_round(const float* log_d, int64_t n, float d_control, float* out, void* stream);
/* src[b, t] = i with cum[i-1] <= t < cum[i], or -1 past mel_len (bit-exact index map). */
int fs2_lr_source(const int32_t* cum, int64_t batch, int64_t src_len, int64_t out_len,
                  int32_t* src, void* stream);
/* out[b, t] = x[b, src[b, t]] (+ posenc[t] for every t < out_len when posenc != NULL) */
int fs2_lr_expand_fwd(const float* x, const int32_t* cum, int64_t batch, int64_t src_len,
                      int64_t out_len, int d, const float* posenc, float* out, void* out_t,
                      void* stream);
/* dx[b, i] = sum of dout[b, t] over the frames phoneme i was copied to (segmented, in order). */
int fs2_lr_expand_bwd(const float* dout, const int32_t* cum, int64_t batch, int64_t src_len,
                      int64_t out_len, int d, float* dx, void* stream);

/* ---------------------------------------------------------------- losses, GMM
 * FastSpeech2Loss (model/loss.py:19-92): masked L1 (mel, postnet), masked MSE (pitch,
 * energy, log-duration vs log(d+1)) with device-side valid counts (no masked_select
 * sync).  Masks are the reference's bool tensors (1 byte, true = padding): src_pad
 * (batch, src_len), mel_pad (batch, mel_len); mel_tgt is cropped to mel_len frames.
 * losses[6] = total, mel, postnet, pitch, energy, duration.  denoms (nullable, device):
 * [mel elements, phonemes] overriding the local counts (data-parallel normalisation).
 * The backward reads the denominators the forward left in ws; g_losses[6] (device) are the
 * upstream gradients of the six outputs.                                               */
int64_t fs2_fs2loss_ws_bytes(int64_t batch, int64_t mel_len);
int fs2_fs2loss_fwd(const float* mel_out, const float* post_out, const float* mel_tgt,
                    int64_t tgt_len, const float* p_pred, const float* e_pred,
                    const float* logd_pred, const float* p_tgt, const float* e_tgt,
                    const int64_t* d_tgt, const uint8_t* src_pad, const uint8_t* mel_pad,
                    int64_t batch, int64_t src_len, int64_t mel_len, int n_mel,
                    const float* denoms, float* losses, float* ws, int64_t ws_bytes, void* stream);
int fs2_fs2loss_bwd(const float* mel_out, const float* post_out, const float* mel_tgt,
                    int64_t tgt_len, const float* p_pred, const float* e_pred,
                    const float* logd_pred, const float* p_tgt, const float* e_tgt,
                    const int64_t* d_tgt, const uint8_t* src_pad, const uint8_t* mel_pad,
                    int64_t batch, int64_t src_len, int64_t mel_len, int n_mel, const float* ws,
                    const float* g_losses, float* d_mel_out, float* d_post_out, float* d_p,
                    float* d_e, float* d_logd, void* stream);

/* SpeakerMetaEncoder (model/fastspeech2.py:306-341): pi = softmax(W m + b),
 * sigma = softplus(W m + b), mu = W m + b.  sigma_pre saved for the backward.          */
int fs2_gmm_head_fwd(const float* meta, int64_t batch, int in_dim, int k, int d,
                     const float* w_pi, const float* b_pi, const float* w_sigma,
                     const float* b_sigma, const float* w_mu, const float* b_mu, float* pi,
                     float* sigma, float* mu, float* sigma_pre, void* stream);
/* log p(e_b) of MixtureSameFamily(Categorical(pi), Independent(Normal(mu, sigma), 1))
 * (torch.distributions semantics incl. the probs clamp); resp (batch, k) saved;
 * mean_out (nullable) = sum_b logp_b / batch  = SpeakerMetaEncLoss (model/loss.py:102-104);
 * denom (nullable, device) replaces batch by the global batch (data parallel).       */
int fs2_gmm_logprob(const float* e, const float* pi, const float* mu, const float* sigma,
                    int64_t batch, int k, int d, float* logp, float* resp, float* mean_out,
                    const float* denom, void* stream);
/* out[3] = [sum_b min(mel_lens, mel_len) * n_mel, sum_b min(src_lens, src_len), batch]:
 * this rank's loss denominators, all-reduced into the global ones (data parallel).  */
int fs2_dp_counts(const int64_t* src_lens, const int64_t* mel_lens, int64_t batch,
                  int64_t src_len, int64_t mel_len, int n_mel, float* out, void* stream);
/* Backward of  L = sum_b g_b * logp_b  through the GMM head into fp32 weight grads (+=). */
int fs2_gmm_head_bwd(const float* meta, const float* e, const float* pi, const float* mu,
                     const float* sigma, const float* sigma_pre, const float* resp,
                     const float* g_logp, int64_t batch, int in_dim, int k, int d,
                     float* dw_pi, float* db_pi, float* dw_sigma, float* db_sigma, float* dw_mu,
                     float* db_mu, void* stream);
/* Draw one embedding per row: component ~ Categorical(pi), e = mu + sigma * N(0,1)
 * (model/fastspeech2.py:176-180 speaker_gen; Philox + Box-Muller).                    */
int fs2_gmm_sample(const float* pi, const float* mu, const float* sigma, int64_t batch, int k,
                   int d, uint64_t seed, uint64_t offset, float* out, int32_t* comp, void* stream);

/* ---------------------------------------------------------------- mid-attribute GMMs
 * model/distributions.py (off the training step).
 * Mixtures are (k, d) rows of mu / sd (Normal scale) plus k weights.
 *
 * InterpolateGMM (12-77).  fs2_gmm_w2_cost: cost[i*kb+j] = the reference's _w2sq (64-77)
 * incl. its elementwise-diagonal quirk, ||mu_a-mu_b||^2 + sum(va + vb - 2 sa^3 sb), double.
 * fs2_ot_emd: exact transport plan (replaces ot.emd, 22: the f32 weights taken as float64,
 * b rescaled to a's mass), one-thread
 * transportation simplex; status[0] = iterations or -1 at max_iter.  k <= 16.
 * fs2_gmm_interpolate (23-62): pi[n] = plan.flat[n] / sum (n = i*kb + j), component
 * n = j*ka + i: mu = (1-t) mu_a[i] + t mu_b[j], sd = ((1-t) sd_a[i] + t sd_b[j])^2.      */
int fs2_gmm_w2_cost(const float* mu_a, const float* sd_a, int ka, const float* mu_b,
                    const float* sd_b, int kb, int d, double* cost, void* stream);
int fs2_ot_emd(const float* a, const float* b, const double* cost, int ka, int kb,
               int max_iter, double* plan, int* status, void* stream);
int fs2_gmm_interpolate(const double* plan, const float* mu_a, const float* sd_a, int ka,
                        const float* mu_b, const float* sd_b, int kb, int d, double t, float* pi,
                        float* mu, float* sd, void* stream);
/* BarycenterGMM (79-192).  m mixtures of k components (one per metadata combination).
 * fs2_gmm_barycenter_positions: k^m (<= 4096) or -1.  fs2_gmm_barycenter (136-163): mean and
 * 60-step fixed-point std of every position of product(range(k), repeat=m), fp32 in the
 * reference's operation order (rate: m floats).  fs2_gmm_bary_mix (165-184): nearest
 * barycenter of each of the m*k original components, weights rate_i * pi_ij (rate: m
 * doubles) summed per barycenter in first-use order, normalised; n_used[0] = number of
 * components written to used / pi_out / mu_out / sd_out (capacity m*k).  m*k <= 64.      */
int64_t fs2_gmm_barycenter_positions(int m, int k);
int fs2_gmm_barycenter(const float* mu, const float* sd, int m, int k, int d, const float* rate,
                       int iters, float* bmean, float* bstd, void* stream);
int64_t fs2_gmm_bary_mix_ws_bytes(int m, int k);
int fs2_gmm_bary_mix(const float* pi, const float* mu, const float* sd, int m, int k, int d,
                     const double* rate, const float* bmean, const float* bstd, int* n_used,
                     int* used, float* pi_out, float* mu_out, float* sd_out, double* ws,
                     int64_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- optimiser
 * clip_grad_norm_ + Adam over one flat fp32 parameter buffer (train.py:202,
 * model/optimizer.py:10-51).  fs2_grad_norm writes norm_coef[0] = ||g||_2 and
 * norm_coef[1] = min(1, max_norm / (norm + 1e-6)); fs2_adam_step multiplies g by
 * norm_coef[1] on the fly (no extra pass over the gradients).                         */
int64_t fs2_grad_norm_ws_bytes(int64_t n);
int fs2_grad_norm(const float* g, int64_t n, float max_norm, float* norm_coef, float* ws,
                  int64_t ws_bytes, void* stream);
int fs2_adam_step(float* p, const float* g, float* m, float* v, int64_t n, const float* norm_coef,
                  float lr, float beta1, float beta2, float eps, float bias_corr1,
                  float bias_corr2_sqrt, const float* hyper, void* stream);
/* Device-side ScheduledOptim.step_and_update_lr (model/optimizer.py:33-51): steps (device,
 * int64[2] = [current_step, adam t]) are incremented (current_step only when advance_lr;
 * step() without the LR update passes 0) and hyper (device, float[3]) set to
 * [lr, 1 - beta1^t, sqrt(1 - beta2^t)], lr = init_lr * min(s^-0.5, warmup^-1.5 * s) *
 * rate^#{anneal < s}; fs2_adam_step reads hyper when it is non-NULL.  anneal_steps_host is
 * a host array (<= 3 entries, copied into the launch).  Together with fs2_seed_next
 * (state = device uint64[3] {base, counter, current seed}; current = splitmix64 of the
 * incremented counter) the whole step is a fixed launch sequence: graph-capturable.     */
int fs2_sched_step(int64_t* steps, float* hyper, double init_lr, int64_t n_warmup,
                   const int64_t* anneal_steps_host, int n_anneal, double anneal_rate, double beta1,
                   double beta2, int advance_lr, void* stream);
int fs2_seed_next(uint64_t* state, void* stream);
/* Stream ordering: work queued on `waiter` after this call starts only after everything
 * queued on `signaler` so far (event record + stream wait; host-side, not a launch).  */
int fs2_stream_wait(void* waiter, void* signaler);
int fs2_fill(float* x, int64_t n, float value, void* stream);
/* y = bf16(x), round to nearest even (compute copies for the bf16 path)              */
int fs2_cast_bf16(const float* x, void* y, int64_t n, void* stream);
int fs2_add_i64(int64_t* x, int64_t n, int64_t value, void* stream); /* BN num_batches_tracked */
int fs2_scale(float* x, int64_t n, float value, void* stream);
/* x[i] = src[0] * scale / (den ? den[0] : 1)  (device scalar broadcast, no host sync) */
int fs2_fill_from(float* x, int64_t n, const float* src, float scale, const float* den,
                  void* stream);
int fs2_add(float* out, const float* a, const float* b, int64_t n, void* stream); /* out = a + b */

/* ---------------------------------------------------------------- debug: stale-read poisoning
 * Not part of the reference's surface: a harness for the bitwise-determinism tests
 * (tests/test_stale_reads.py).  fs2_debug_poison(byte), byte in [0, 255] (or the FS2_POISON
 * environment variable, read once): every workspace an entry point receives and the library's
 * reused split-K partials are filled with that byte before each use; -1 turns it off (the
 * default).  fs2_debug_alloc / fs2_debug_free have the signatures of
 * torch.cuda.memory.CUDAPluggableAllocator: no caching and no device synchronisation; a block
 * is filled with the poison byte (0xff when off) at allocation (done before the call returns)
 * and again on its stream at its free, and freed blocks are quarantined (not reused) until 6 GB of them pile up.  With both, a
 * kernel that reads memory nothing wrote this step, or memory freed before it ran, reads the
 * poison, so its results depend on the byte instead of on what ran earlier in the process.
 * With poisoning on, every fs2_stream_wait also fills the LDS of every CU with the byte on the
 * waiting stream (one 160 KiB block per CU), so a kernel reading LDS it did not write reads it.
 * fs2_debug_race(delay_us, main_stream, mode): mode 0 -- every stream other than main_stream
 * is held back delay_us after each fs2_stream_wait it receives (a one-lane sleep kernel), so
 * side-stream work trails the main stream and a buffer freed or overwritten on the main stream
 * before a side-stream reader ran is poisoned by then; mode 1 -- the main stream is held back
 * after each event a side stream waits on, so a side-stream read of a main-stream result that
 * was not waited for reads stale data.  Either way a missing ordering or lifetime guard fails
 * deterministically.  Mode 2 -- a seeded random schedule: at each wait the waiter and the
 * signaler are each held back with probability 1/2 by a random 0..delay_us (an LCG from seed),
 * so one seed replays one interleaving.  delay_us 0: off.  fs2_debug_lds_dma_oob(src, out, stream): one wave
 * LDS-DMAs 16 B per lane from src (64 x 16 B) into LDS pre-filled with 0xAB bytes, lanes 32-63
 * at an out-of-range offset, and copies the 1 KiB image to out (the padding-row contract of
 * every LDS-DMA kernel: out-of-range lanes land zeros).  fs2_debug_snap(buf, cap): the variance
 * predictor backward appends copies of its intermediates (dh2, the LN2 partials, du1, dh1, the
 * LN1 partials), in stream order, to buf; fs2_debug_snap_used() is the byte count so far
 * (cap + 1 after an overflow); buf NULL turns it off.  fs2_debug_coherence(x, n, rounds,
 * blocks, bad, stream): per round, `blocks` blocks read the n uint32 of x, one block writes
 * x[i] = tag + i, and `blocks` blocks read x again, adding to bad[block] the elements that
 * are not tag + i (bad: blocks + 1 uint32, zeroed by the caller) -- a stale line in some
 * XCD's L2 after a kernel boundary on one stream shows up as a nonzero count.             */
int fs2_debug_poison(int byte);
void* fs2_debug_alloc(int64_t size, int device, void* stream);
void fs2_debug_free(void* ptr, int64_t size, int device, void* stream);
int fs2_debug_race(int delay_us, void* main_stream, int mode, int seed);
int fs2_debug_lds_dma_oob(const float* src, void* out, void* stream);
int fs2_debug_snap(void* buf, int64_t cap);
int fs2_debug_coherence(void* x, int64_t n, int rounds, int blocks, void* bad, void* stream);
int64_t fs2_debug_snap_used(void);

#ifdef __cplusplus
}
#endif
#endif /* FS2HIP_H */
