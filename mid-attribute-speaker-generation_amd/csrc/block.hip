// One FFT block's forward and backward issued from C (host code only; every kernel is one of
// the library's own entry points, called in the order model.FFTBlock.fwd / .bwd call them, so
// the results are bitwise those of the per-kernel path).  The Python host spends ~5-6 us per
// ctypes launch with its allocations and argument conversion (4.6 ms
// of host enqueue for 348 launches); here a block is one call: ~5 launches forward, ~10
// backward on two streams with their event waits.
//
// transformer/Layers.py:21-30 (FFTBlock.forward), transformer/SubLayers.py:29-57,85-93
// (MultiHeadAttention, PositionwiseFeedForward) and their autograd backward.
//
// Activations live in one caller-allocated region per block and step (fs2_fft_block_act_bytes);
// the backward's temporaries in another (fs2_fft_block_tmp_bytes).  Both are read by
// weight-gradient kernels on the side stream after the call returns: the caller keeps them
// alive until it joins that stream.
#include <math.h>
#include <string.h>

#include "common.hpp"

using namespace fs2;

namespace {

struct Blk {
  int64_t d, heads, dk, dinner, taps, pad, site;
  int64_t n3, hd;
  const void *wq_f, *wq_b, *wfc_f, *wfc_b, *w1_f, *w1_b, *w2_f, *w2_b;
  const float *bq, *bfc, *b1, *b2, *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  float *gq_w, *gq_b, *gfc_w, *gfc_b, *g1_w, *g1_b, *g2_w, *g2_b;
  float *gln1_g, *gln1_b, *gln2_g, *gln2_b;
};

template <typename T>
T* P(int64_t v) {
  return reinterpret_cast<T*>((uintptr_t)v);
}

Blk unpack(const int64_t* w) {
  Blk b;
  b.d = w[FS2_FB_D];
  b.heads = w[FS2_FB_HEADS];
  b.dk = w[FS2_FB_DK];
  b.dinner = w[FS2_FB_DINNER];
  b.taps = w[FS2_FB_TAPS];
  b.pad = w[FS2_FB_PAD];
  b.site = w[FS2_FB_SITE];
  b.hd = b.heads * b.dk;
  b.n3 = 3 * b.hd;
  b.wq_f = P<const void>(w[FS2_FB_WQKV_F]);
  b.wq_b = P<const void>(w[FS2_FB_WQKV_B]);
  b.bq = P<const float>(w[FS2_FB_BQKV]);
  b.wfc_f = P<const void>(w[FS2_FB_WFC_F]);
  b.wfc_b = P<const void>(w[FS2_FB_WFC_B]);
  b.bfc = P<const float>(w[FS2_FB_BFC]);
  b.w1_f = P<const void>(w[FS2_FB_W1_F]);
  b.w1_b = P<const void>(w[FS2_FB_W1_B]);
  b.b1 = P<const float>(w[FS2_FB_B1]);
  b.w2_f = P<const void>(w[FS2_FB_W2_F]);
  b.w2_b = P<const void>(w[FS2_FB_W2_B]);
  b.b2 = P<const float>(w[FS2_FB_B2]);
  b.ln1_g = P<const float>(w[FS2_FB_LN1_G]);
  b.ln1_b = P<const float>(w[FS2_FB_LN1_B]);
  b.ln2_g = P<const float>(w[FS2_FB_LN2_G]);
  b.ln2_b = P<const float>(w[FS2_FB_LN2_B]);
  b.gq_w = P<float>(w[FS2_FB_GQKV_W]);
  b.gq_b = P<float>(w[FS2_FB_GQKV_B]);
  b.gfc_w = P<float>(w[FS2_FB_GFC_W]);
  b.gfc_b = P<float>(w[FS2_FB_GFC_B]);
  b.g1_w = P<float>(w[FS2_FB_G1_W]);
  b.g1_b = P<float>(w[FS2_FB_G1_B]);
  b.g2_w = P<float>(w[FS2_FB_G2_W]);
  b.g2_b = P<float>(w[FS2_FB_G2_B]);
  b.gln1_g = P<float>(w[FS2_FB_GLN1_G]);
  b.gln1_b = P<float>(w[FS2_FB_GLN1_B]);
  b.gln2_g = P<float>(w[FS2_FB_GLN2_G]);
  b.gln2_b = P<float>(w[FS2_FB_GLN2_B]);
  return b;
}

int64_t al(int64_t bytes) { return (bytes + 255) / 256 * 256; }

// the forward's activation region: offsets (bytes) of its tensors
struct ActLayout {
  int64_t qkv, o, lse, x1, x1_t, xh1, rs1, h, x2, x2_t, xh2, rs2, y, total;
};
ActLayout act_layout(const Blk& b, int64_t rows, int64_t batch, int64_t T, int fuse) {
  ActLayout L;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = o;
    o += al(bytes);
    return at;
  };
  L.qkv = take(rows * b.n3 * 2);
  L.o = take(rows * b.hd * 2);
  L.lse = take(batch * b.heads * T * 4);
  L.x1 = take(rows * b.d * 4);
  L.x1_t = take(rows * b.d * 2);
  L.xh1 = take(rows * b.d * 4);
  L.rs1 = take(rows * 4);
  L.h = take(rows * b.dinner * 2);
  L.x2 = take(rows * b.d * 4);
  L.x2_t = take(rows * b.d * 2);
  L.xh2 = take(rows * b.d * 4);
  L.rs2 = take(rows * 4);
  L.y = fuse ? -1 : take(rows * b.d * 4);  // fp32 GEMM output before a separate LayerNorm
  L.total = o;
  return L;
}

// the backward's temporaries
struct TmpLayout {
  int64_t dx1, dy2_t, dh, dy1_t, dout, dqkv, ws, ws_bytes, ln_ws[3], ln_ws_bytes, total;
};
TmpLayout tmp_layout(const Blk& b, int64_t rows, int64_t batch, int64_t T) {
  TmpLayout L;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = o;
    o += al(bytes);
    return at;
  };
  L.dx1 = take(rows * b.d * 4);
  L.dy2_t = take(rows * b.d * 2);
  L.dh = take(rows * b.dinner * 2);
  L.dy1_t = take(rows * b.d * 2);
  L.dout = take(rows * b.hd * 2);
  L.dqkv = take(rows * b.n3 * 2);
  const int64_t w1 = fs2_ln_bwd_ws_bytes(rows, (int)b.d), w2 = fs2_attn_bwd_ws_bytes(batch, T, (int)b.heads);
  L.ws_bytes = al(w1 > w2 ? w1 : w2);
  L.ws = take(L.ws_bytes);
  // the LayerNorm backwards' column partials (LN2, LN1, the previous block's LN2), reduced into
  // the parameter gradients on the side stream after the call returns: a region each
  L.ln_ws_bytes = al(w1);
  for (int i = 0; i < 3; ++i) L.ln_ws[i] = take(L.ln_ws_bytes);
  L.total = o;
  return L;
}

template <typename T>
T* at(void* base, int64_t off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}

#define FS2_TRY(call)              \
  do {                             \
    const int rc_ = (call);        \
    if (rc_ != FS2_OK) return rc_; \
  } while (0)

}  // namespace

extern "C" {

int64_t fs2_fft_block_act_bytes(const int64_t* blk, int64_t rows, int64_t batch, int64_t seq_len,
                                int fuse_ln) {
  return act_layout(unpack(blk), rows, batch, seq_len, fuse_ln).total;
}

int64_t fs2_fft_block_act_offset(const int64_t* blk, int64_t rows, int64_t batch,
                                 int64_t seq_len, int fuse_ln, int which) {
  const ActLayout L = act_layout(unpack(blk), rows, batch, seq_len, fuse_ln);
  switch (which) {
    case FS2_FA_X2: return L.x2;
    case FS2_FA_X2_T: return L.x2_t;
    default: return -1;
  }
}

int64_t fs2_fft_block_tmp_bytes(const int64_t* blk, int64_t rows, int64_t batch, int64_t seq_len) {
  return tmp_layout(unpack(blk), rows, batch, seq_len).total;
}

int64_t fs2_fft_block_side_ws_bytes(const int64_t* blk, int64_t rows) {
  const Blk b = unpack(blk);
  const int64_t w9 = fs2_conv_wgrad_ws_bytes(rows, b.d, b.dinner, (int)b.taps);
  const int64_t jobs[24] = {0, b.d,  0, b.dinner, 0, 0, b.dinner, b.d,
                            0, b.d,  0, b.hd,     0, 0, b.hd,     b.d,
                            0, b.n3, 0, b.d,      0, 1, b.d,      b.n3};
  const int64_t w1 = fs2_conv_wgrad_k1_multi_ws_bytes(jobs, 3, rows);
  return w9 > w1 ? w9 : w1;
}

int fs2_fft_block_fwd(const int64_t* blk, const float* x, const void* x_t, void* act, int64_t rows,
                      int64_t batch, int64_t seq_len, const int64_t* lens, float p,
                      const uint64_t* seed, int fuse_ln, void* stream) {
  FS2_CHECK_ARG(blk && x && x_t && act && rows == batch * seq_len && seq_len > 0,
                "fs2_fft_block_fwd: bad arguments");
  const Blk b = unpack(blk);
  const ActLayout L = act_layout(b, rows, batch, seq_len, fuse_ln);
  const int64_t T = seq_len;
  const uint64_t* sd = p > 0.f ? seed : nullptr;
  FS2_CHECK_ARG(!(p > 0.f) || seed, "fs2_fft_block_fwd: dropout without seed");
  lds_poison(as_stream(stream));
  void* qkv = at<void>(act, L.qkv);
  void* o = at<void>(act, L.o);
  float* lse = at<float>(act, L.lse);
  float* x1 = at<float>(act, L.x1);
  void* x1_t = at<void>(act, L.x1_t);
  float* xh1 = at<float>(act, L.xh1);
  float* rs1 = at<float>(act, L.rs1);
  void* h = at<void>(act, L.h);
  float* x2 = at<float>(act, L.x2);
  void* x2_t = at<void>(act, L.x2_t);
  float* xh2 = at<float>(act, L.xh2);
  float* rs2 = at<float>(act, L.rs2);
  // QKV projection -> attention (SubLayers.py:39-52, Modules.py:14-25)
  FS2_TRY(fs2_conv_gemm(FS2_BF16, x_t, b.d, b.wq_f, qkv, b.n3, rows, T, b.d, b.n3, 1, 0, lens, b.bq,
                        FS2_EPI_BIAS | FS2_EPI_OUT_BF16, nullptr, b.n3, stream));
  const float scale = (float)(1.0 / sqrt((double)b.dk));
  FS2_TRY(fs2_attn_fwd(FS2_BF16, qkv, o, lse, lens, batch, T, (int)b.heads, (int)b.dk, scale, stream));
  // fc -> dropout -> + residual -> LayerNorm, masked (SubLayers.py:53-55, Layers.py:25)
  if (fuse_ln) {
    FS2_TRY(fs2_conv_gemm_ln(o, b.hd, b.wfc_f, rows, T, b.hd, b.d, 1, 0, lens, b.bfc, x, b.ln1_g,
                             b.ln1_b, x1, x1_t, xh1, rs1, p, sd, (uint64_t)b.site, stream));
  } else {
    float* y = at<float>(act, L.y);
    FS2_TRY(fs2_conv_gemm(FS2_BF16, o, b.hd, b.wfc_f, y, b.d, rows, T, b.hd, b.d, 1, 0, lens, b.bfc,
                          FS2_EPI_BIAS, nullptr, b.d, stream));
    FS2_TRY(fs2_ln_fwd(FS2_BF16, y, x, b.ln1_g, b.ln1_b, x1, x1_t, xh1, rs1, lens, T, rows, (int)b.d,
                       p, 0.f, sd, (uint64_t)b.site, 0, nullptr, nullptr, nullptr, stream));
  }
  // Conv1d(k) -> ReLU -> Conv1d(1) -> dropout -> + residual -> LayerNorm (SubLayers.py:85-93)
  FS2_TRY(fs2_conv_gemm(FS2_BF16, x1_t, b.d, b.w1_f, h, b.dinner, rows, T, b.d, b.dinner, (int)b.taps,
                        (int)b.pad, lens, b.b1, FS2_EPI_BIAS | FS2_EPI_RELU | FS2_EPI_OUT_BF16, nullptr,
                        b.dinner, stream));
  if (fuse_ln) {
    FS2_TRY(fs2_conv_gemm_ln(h, b.dinner, b.w2_f, rows, T, b.dinner, b.d, 1, 0, lens, b.b2, x1,
                             b.ln2_g, b.ln2_b, x2, x2_t, xh2, rs2, p, sd, (uint64_t)(b.site + 1),
                             stream));
  } else {
    float* y = at<float>(act, L.y);
    FS2_TRY(fs2_conv_gemm(FS2_BF16, h, b.dinner, b.w2_f, y, b.d, rows, T, b.dinner, b.d, 1, 0, lens,
                          b.b2, FS2_EPI_BIAS, nullptr, b.d, stream));
    FS2_TRY(fs2_ln_fwd(FS2_BF16, y, x1, b.ln2_g, b.ln2_b, x2, x2_t, xh2, rs2, lens, T, rows, (int)b.d,
                       p, 0.f, sd, (uint64_t)(b.site + 1), 0, nullptr, nullptr, nullptr, stream));
  }
  return FS2_OK;
}

int fs2_fft_block_bwd(const int64_t* blk, void* act, const void* x_t, int fuse_ln, float p,
                      const float* dx2, const void* carry_dy2_t, float* carry_dx1,
                      const int64_t* prev_blk, void* prev_act, int prev_fuse_ln, float prev_p,
                      void* tmp, float* dx, void* prev_dy2_t, float* prev_dx1, int64_t rows,
                      int64_t batch, int64_t seq_len, const int64_t* lens, const uint64_t* seed,
                      float* side_ws, int64_t side_ws_bytes, void* stream, void* side_stream) {
  FS2_CHECK_ARG(blk && act && x_t && tmp && dx && rows == batch * seq_len && seq_len > 0,
                "fs2_fft_block_bwd: bad arguments");
  FS2_CHECK_ARG((dx2 != nullptr) != (carry_dy2_t != nullptr && carry_dx1 != nullptr),
                "fs2_fft_block_bwd: give dx2 or the carried (dy2_t, dx1), not both");
  FS2_CHECK_ARG(!prev_blk || (prev_act && prev_dy2_t && prev_dx1),
                "fs2_fft_block_bwd: the previous block's LN2 backward needs its buffers");
  FS2_CHECK_ARG(!(p > 0.f || (prev_blk && prev_p > 0.f)) || seed, "fs2_fft_block_bwd: dropout without seed");
  const Blk b = unpack(blk);
  const ActLayout L = act_layout(b, rows, batch, seq_len, fuse_ln);
  const TmpLayout W = tmp_layout(b, rows, batch, seq_len);
  const int64_t T = seq_len;
  const uint64_t* sd = p > 0.f ? seed : nullptr;
  void* side = side_stream ? side_stream : stream;
  FS2_CHECK_ARG(side_ws && side_ws_bytes >= fs2_fft_block_side_ws_bytes(blk, rows),
                "fs2_fft_block_bwd: side-stream workspace too small");
  lds_poison(as_stream(stream));
  const void* qkv = at<void>(act, L.qkv);
  const void* o = at<void>(act, L.o);
  const float* lse = at<float>(act, L.lse);
  const void* x1_t = at<void>(act, L.x1_t);
  const float* xh1 = at<float>(act, L.xh1);
  const float* rs1 = at<float>(act, L.rs1);
  const void* h = at<void>(act, L.h);
  const float* xh2 = at<float>(act, L.xh2);
  const float* rs2 = at<float>(act, L.rs2);
  float* ws = at<float>(tmp, W.ws);
  const void* dy2_t;
  float* dx1;
  if (carry_dy2_t) {  // this block's LN2 backward ran in the following block's QKV epilogue
    dy2_t = carry_dy2_t;
    dx1 = carry_dx1;
  } else {  // LN2 (masked; dropout before the residual add): dx1 starts as dz2
    dx1 = at<float>(tmp, W.dx1);
    void* d2 = at<void>(tmp, W.dy2_t);
    FS2_TRY(fs2_ln_bwd(FS2_BF16, dx2, nullptr, nullptr, xh2, rs2, b.ln2_g, b.ln2_b, lens, T, rows,
                       (int)b.d, p, 0.f, sd, (uint64_t)(b.site + 1), 0, nullptr, nullptr, d2, dx1, 0,
                       nullptr, nullptr, nullptr, nullptr, nullptr, at<float>(tmp, W.ln_ws[0]),
                       W.ln_ws_bytes, stream));
    dy2_t = d2;
  }
  // a LayerNorm backward's parameter gradients (dgamma, dbeta, the fused bias gradient): the
  // column reduction of its partials, off the main chain on the side stream (called after a
  // stream_wait that orders it behind the partials)
  auto ln_final = [&](int slot, float* dg, float* db, float* dbias) {
    return fs2_ln_bwd_final(rows, (int)b.d, at<float>(tmp, W.ln_ws[slot]), 0, dg, db, nullptr,
                            nullptr, dbias, side);
  };
  // grouped k = 1 weight gradients (w_2, fc, QKV), issued together at the end of the block
  int64_t jobs[24] = {(int64_t)(uintptr_t)dy2_t, b.d, (int64_t)(uintptr_t)h, b.dinner,
                      (int64_t)(uintptr_t)b.g2_w, 0, b.dinner, b.d};
  // dh = (dy2 W2) * (h > 0), then w_1's weight gradient on the side stream and its data gradient
  void* dh = at<void>(tmp, W.dh);
  FS2_TRY(fs2_conv_gemm(FS2_BF16, dy2_t, b.d, b.w2_b, dh, b.dinner, rows, T, b.d, b.dinner, 1, 0, lens,
                        nullptr, FS2_EPI_RELU_MASK_AUX | FS2_EPI_OUT_BF16 | FS2_EPI_AUX_BF16, h,
                        b.dinner, stream));
  if (side != stream) FS2_TRY(fs2_stream_wait(side, stream));
  if (!carry_dy2_t) FS2_TRY(ln_final(0, b.gln2_g, b.gln2_b, b.g2_b));
  FS2_TRY(fs2_conv_wgrad(FS2_BF16, dh, b.dinner, x1_t, b.d, b.g1_w, b.g1_b, rows, T, b.d, b.dinner,
                         (int)b.taps, (int)b.pad, lens, side_ws, side_ws_bytes, side));
  FS2_TRY(fs2_conv_gemm(FS2_BF16, dh, b.dinner, b.w1_b, dx1, b.d, rows, T, b.dinner, b.d, (int)b.taps,
                        (int)b.pad, lens, nullptr, FS2_EPI_ADD_AUX, dx1, b.d, stream));
  // LN1 -> fc -> attention -> QKV
  void* dy1_t = at<void>(tmp, W.dy1_t);
  FS2_TRY(fs2_ln_bwd(FS2_BF16, dx1, nullptr, nullptr, xh1, rs1, b.ln1_g, b.ln1_b, lens, T, rows,
                     (int)b.d, p, 0.f, sd, (uint64_t)b.site, 0, nullptr, nullptr, dy1_t, dx, 0, nullptr,
                     nullptr, nullptr, nullptr, nullptr, at<float>(tmp, W.ln_ws[1]), W.ln_ws_bytes,
                     stream));
  const int64_t j2[8] = {(int64_t)(uintptr_t)dy1_t, b.d, (int64_t)(uintptr_t)o, b.hd,
                         (int64_t)(uintptr_t)b.gfc_w, 0, b.hd, b.d};
  memcpy(jobs + 8, j2, sizeof j2);
  void* dout = at<void>(tmp, W.dout);
  FS2_TRY(fs2_conv_gemm(FS2_BF16, dy1_t, b.d, b.wfc_b, dout, b.hd, rows, T, b.d, b.hd, 1, 0, lens,
                        nullptr, FS2_EPI_OUT_BF16, nullptr, b.hd, stream));
  void* dqkv = at<void>(tmp, W.dqkv);
  const float scale = (float)(1.0 / sqrt((double)b.dk));
  FS2_TRY(fs2_attn_bwd(FS2_BF16, qkv, o, dout, lse, dqkv, lens, batch, T, (int)b.heads, (int)b.dk,
                       scale, ws, W.ws_bytes, stream));
  const int64_t j3[8] = {(int64_t)(uintptr_t)dqkv, b.n3, (int64_t)(uintptr_t)x_t, b.d,
                         (int64_t)(uintptr_t)b.gq_w, (int64_t)(uintptr_t)b.gq_b, b.d, b.n3};
  memcpy(jobs + 16, j3, sizeof j3);
  // the grouped k = 1 weight gradients and the LN1 parameter reduction go to the side stream
  // after the QKV data gradient is issued, not before it: the w_2 data gradient of the next
  // block then runs beside the band weight gradient rather than beside the grouped k = 1
  // kernel (same kernels and per-buffer order; -0.04 ms/step same-box, profiles/r6_k1_late_ab.txt)
  auto k1_side = [&]() -> int {
    if (side != stream) FS2_TRY(fs2_stream_wait(side, stream));
    FS2_TRY(ln_final(1, b.gln1_g, b.gln1_b, b.gfc_b));
    return fs2_conv_wgrad_k1_multi(FS2_BF16, jobs, 3, rows, T, lens, side_ws, side_ws_bytes, side);
  };
  if (prev_blk) {
    // the previous block's FFN post-LN backward in this block's QKV data-gradient epilogue
    const Blk pb = unpack(prev_blk);
    const ActLayout PL = act_layout(pb, rows, batch, seq_len, prev_fuse_ln);
    FS2_TRY(fs2_conv_gemm_ln_bwd(dqkv, b.n3, b.wq_b, rows, T, b.n3, b.d, 1, 0, lens, dx,
                                 at<float>(prev_act, PL.xh2), at<float>(prev_act, PL.rs2), pb.ln2_g,
                                 nullptr, nullptr, nullptr, prev_p, prev_p > 0.f ? seed : nullptr,
                                 (uint64_t)(pb.site + 1), prev_dx1, 0, prev_dy2_t,
                                 at<float>(tmp, W.ln_ws[2]), W.ln_ws_bytes, stream));
    FS2_TRY(k1_side());
    return fs2_ln_bwd_final(rows, (int)pb.d, at<float>(tmp, W.ln_ws[2]), 0, pb.gln2_g, pb.gln2_b,
                            nullptr, nullptr, pb.g2_b, side);
  }
  FS2_TRY(fs2_conv_gemm(FS2_BF16, dqkv, b.n3, b.wq_b, dx, b.d, rows, T, b.n3, b.d, 1, 0, lens, nullptr,
                        FS2_EPI_ADD_AUX, dx, b.d, stream));
  return k1_side();
}

}  // extern "C"
