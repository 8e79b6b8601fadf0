// The mel head (mel_linear + PostNet + residual) and one VariancePredictor, forward and
// backward, issued from C (host code only), as block.hip does for an FFT block: every kernel
// is one of the library's own entry points, called in the order model.MelHeadFn /
// model.PostNet / model.VariancePredictor call them, so the results are bitwise those of the
// per-kernel path.
//
// model/fastspeech2.py:91-93 (mel_linear, postnet(output) + output), transformer/Layers.py:67-137
// (PostNet: 5 x Conv1d(k=5) + BatchNorm1d, tanh on all but the last, dropout 0.5),
// model/modules.py:197-250 (VariancePredictor: 2 x (Conv1d(k=3) -> ReLU -> LN -> dropout) ->
// Linear(., 1), masked) and their autograd backward.
//
// Activations live in one caller-allocated region per call site and step (fs2_*_act_bytes);
// the backward's temporaries in another (fs2_*_tmp_bytes).  Side-stream weight gradients read
// both after the call returns: the caller keeps them until it joins that stream.
#include <string.h>

#include "common.hpp"

using namespace fs2;

namespace {

template <typename T>
T* P(int64_t v) {
  return reinterpret_cast<T*>((uintptr_t)v);
}

template <typename T>
T* at(void* base, int64_t off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}

int64_t al(int64_t bytes) { return (bytes + 255) / 256 * 256; }

struct Take {
  int64_t o = 0;
  int64_t operator()(int64_t bytes) {
    const int64_t at = o;
    o += al(bytes);
    return at;
  }
};

#define FS2_TRY(call)              \
  do {                             \
    const int rc_ = (call);        \
    if (rc_ != FS2_OK) return rc_; \
  } while (0)

// BatchNorm1d defaults (PostNet builds them with eps / momentum unset, Layers.py:87-124)
constexpr float kBnEps = 1e-5f, kBnMomentum = 0.1f;

// ------------------------------------------------------------------ mel head
struct MhLayer {
  const void *w_f, *w_b;
  const float *b, *bn_g, *bn_b;
  float *rm, *rv;
  int64_t* nbt;
  float *gw, *gb, *gbn_g, *gbn_b;
};

struct Mh {
  int64_t n_mel, d_in, dim, taps, pad, layers, site;
  const void *lin_wf, *lin_wb;
  const float* lin_b;
  float *glin_w, *glin_b;
  MhLayer l[FS2_MH_MAX_LAYERS];
  int64_t c_in(int i) const { return i == 0 ? n_mel : dim; }
  int64_t c_out(int i) const { return i == layers - 1 ? n_mel : dim; }
};

bool unpack(const int64_t* w, Mh& m) {
  m.n_mel = w[FS2_MH_NMEL];
  m.d_in = w[FS2_MH_DIN];
  m.dim = w[FS2_MH_DIM];
  m.taps = w[FS2_MH_TAPS];
  m.pad = w[FS2_MH_PAD];
  m.layers = w[FS2_MH_LAYERS];
  m.site = w[FS2_MH_SITE];
  m.lin_wf = P<const void>(w[FS2_MH_LIN_WF]);
  m.lin_wb = P<const void>(w[FS2_MH_LIN_WB]);
  m.lin_b = P<const float>(w[FS2_MH_LIN_B]);
  m.glin_w = P<float>(w[FS2_MH_GLIN_W]);
  m.glin_b = P<float>(w[FS2_MH_GLIN_B]);
  if (m.layers < 1 || m.layers > FS2_MH_MAX_LAYERS || m.n_mel <= 0 || m.dim <= 0 || m.d_in <= 0)
    return false;
  for (int i = 0; i < m.layers; ++i) {
    const int64_t* q = w + FS2_MH_LAYER0 + i * FS2_MHL_WORDS;
    MhLayer& L = m.l[i];
    L.w_f = P<const void>(q[FS2_MHL_W_F]);
    L.w_b = P<const void>(q[FS2_MHL_W_B]);
    L.b = P<const float>(q[FS2_MHL_B]);
    L.bn_g = P<const float>(q[FS2_MHL_BN_G]);
    L.bn_b = P<const float>(q[FS2_MHL_BN_B]);
    L.rm = P<float>(q[FS2_MHL_BN_RM]);
    L.rv = P<float>(q[FS2_MHL_BN_RV]);
    L.nbt = P<int64_t>(q[FS2_MHL_BN_NBT]);
    L.gw = P<float>(q[FS2_MHL_GW]);
    L.gb = P<float>(q[FS2_MHL_GB]);
    L.gbn_g = P<float>(q[FS2_MHL_GBN_G]);
    L.gbn_b = P<float>(q[FS2_MHL_GBN_B]);
  }
  return true;
}

int64_t bn_ws(const Mh& m, int64_t rows) {
  const int64_t a = fs2_bn_ws_bytes(rows, m.dim), b = fs2_bn_ws_bytes(rows, m.n_mel);
  return al(a > b ? a : b);
}

// forward region: mel_linear output + copy, per layer (z, mean, rstd, bf16 output copy: the
// next layer's input), the PostNet output (+ residual), BatchNorm scratch
struct MhAct {
  int64_t out, out_t, z[FS2_MH_MAX_LAYERS], mean[FS2_MH_MAX_LAYERS], rstd[FS2_MH_MAX_LAYERS],
      a_t[FS2_MH_MAX_LAYERS], post, ws, ws_bytes, total;
};
MhAct mh_act(const Mh& m, int64_t rows) {
  MhAct A;
  Take take;
  A.out = take(rows * m.n_mel * 4);
  A.out_t = take(rows * m.n_mel * 2);
  for (int i = 0; i < m.layers; ++i) {
    A.z[i] = take(rows * m.c_out(i) * 4);
    A.mean[i] = take(m.c_out(i) * 4);
    A.rstd[i] = take(m.c_out(i) * 4);
    A.a_t[i] = i < m.layers - 1 ? take(rows * m.c_out(i) * 2) : -1;
  }
  A.post = take(rows * m.n_mel * 4);
  A.ws_bytes = bn_ws(m, rows);
  A.ws = take(A.ws_bytes);
  A.total = take.o;
  return A;
}

// backward temporaries: dm (fp32) and its copy, one bf16 dz per layer (read by the side
// stream), the fp32 running gradient, BatchNorm scratch
struct MhTmp {
  int64_t dm, dm_t, dz_t[FS2_MH_MAX_LAYERS], d, ws, ws_bytes, total;
};
MhTmp mh_tmp(const Mh& m, int64_t rows) {
  MhTmp W;
  Take take;
  W.dm = take(rows * m.n_mel * 4);
  W.dm_t = take(rows * m.n_mel * 2);
  for (int i = 0; i < m.layers; ++i) W.dz_t[i] = take(rows * m.c_out(i) * 2);
  W.d = take(rows * m.dim * 4);
  W.ws_bytes = bn_ws(m, rows);
  W.ws = take(W.ws_bytes);
  W.total = take.o;
  return W;
}

// ------------------------------------------------------------------ variance predictor
struct Vp {
  int64_t d, filt, taps, pad1, pad2, site;
  const void *w1_f, *w1_b, *w2_f, *w2_b;
  const float *b1, *ln1_g, *ln1_b, *b2, *ln2_g, *ln2_b, *lin_w, *lin_b;
  float *g1_w, *g1_b, *gln1_g, *gln1_b, *g2_w, *g2_b, *gln2_g, *gln2_b, *glin_w, *glin_b;
};

Vp unpack_vp(const int64_t* w) {
  Vp v;
  v.d = w[FS2_VP_D];
  v.filt = w[FS2_VP_FILTER];
  v.taps = w[FS2_VP_TAPS];
  v.pad1 = w[FS2_VP_PAD1];
  v.pad2 = w[FS2_VP_PAD2];
  v.site = w[FS2_VP_SITE];
  v.w1_f = P<const void>(w[FS2_VP_W1_F]);
  v.w1_b = P<const void>(w[FS2_VP_W1_B]);
  v.b1 = P<const float>(w[FS2_VP_B1]);
  v.ln1_g = P<const float>(w[FS2_VP_LN1_G]);
  v.ln1_b = P<const float>(w[FS2_VP_LN1_B]);
  v.w2_f = P<const void>(w[FS2_VP_W2_F]);
  v.w2_b = P<const void>(w[FS2_VP_W2_B]);
  v.b2 = P<const float>(w[FS2_VP_B2]);
  v.ln2_g = P<const float>(w[FS2_VP_LN2_G]);
  v.ln2_b = P<const float>(w[FS2_VP_LN2_B]);
  v.lin_w = P<const float>(w[FS2_VP_LIN_W]);
  v.lin_b = P<const float>(w[FS2_VP_LIN_B]);
  v.g1_w = P<float>(w[FS2_VP_G1_W]);
  v.g1_b = P<float>(w[FS2_VP_G1_B]);
  v.gln1_g = P<float>(w[FS2_VP_GLN1_G]);
  v.gln1_b = P<float>(w[FS2_VP_GLN1_B]);
  v.g2_w = P<float>(w[FS2_VP_G2_W]);
  v.g2_b = P<float>(w[FS2_VP_G2_B]);
  v.gln2_g = P<float>(w[FS2_VP_GLN2_G]);
  v.gln2_b = P<float>(w[FS2_VP_GLN2_B]);
  v.glin_w = P<float>(w[FS2_VP_GLIN_W]);
  v.glin_b = P<float>(w[FS2_VP_GLIN_B]);
  return v;
}

// forward region: h1 (fp32, the ReLU mask), u1 (fp32 LN output, unused downstream but written
// by the LN kernel) + copy, xhat1, rstd1, h2, xhat2, rstd2, the LN2 output (written, unused),
// pred
struct VpAct {
  int64_t h1, u1, u1_t, xh1, rs1, h2, u2, xh2, rs2, pred, total;
};
VpAct vp_act(const Vp& v, int64_t rows) {
  VpAct A;
  Take take;
  A.h1 = take(rows * v.filt * 4);
  A.u1 = take(rows * v.filt * 4);
  A.u1_t = take(rows * v.filt * 2);
  A.xh1 = take(rows * v.filt * 4);
  A.rs1 = take(rows * 4);
  A.h2 = take(rows * v.filt * 4);
  A.u2 = take(rows * v.filt * 4);
  A.xh2 = take(rows * v.filt * 4);
  A.rs2 = take(rows * 4);
  A.pred = take(rows * 4);
  A.total = take.o;
  return A;
}

// backward temporaries; the two LayerNorm backwards' column partials each have a region (their
// reductions into the parameter gradients run later, on the side stream)
struct VpTmp {
  int64_t dh2_t, du1, dh1_t, ws[2], ws_bytes, total;
};
VpTmp vp_tmp(const Vp& v, int64_t rows) {
  VpTmp W;
  Take take;
  W.dh2_t = take(rows * v.filt * 2);
  W.du1 = take(rows * v.filt * 4);
  W.dh1_t = take(rows * v.filt * 2);
  W.ws_bytes = al(fs2_ln_bwd_ws_bytes(rows, (int)v.filt));
  W.ws[0] = take(W.ws_bytes);
  W.ws[1] = take(W.ws_bytes);
  W.total = take.o;
  return W;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ mel head
int64_t fs2_mel_head_act_bytes(const int64_t* mh, int64_t rows) {
  Mh m;
  if (!mh || !unpack(mh, m)) return -1;
  return mh_act(m, rows).total;
}

int64_t fs2_mel_head_act_offset(const int64_t* mh, int64_t rows, int which) {
  Mh m;
  if (!mh || !unpack(mh, m)) return -1;
  const MhAct A = mh_act(m, rows);
  switch (which) {
    case FS2_MHA_OUT: return A.out;
    case FS2_MHA_POST: return A.post;
    default: return -1;
  }
}

int64_t fs2_mel_head_tmp_bytes(const int64_t* mh, int64_t rows) {
  Mh m;
  if (!mh || !unpack(mh, m)) return -1;
  return mh_tmp(m, rows).total;
}

int64_t fs2_mel_head_side_ws_bytes(const int64_t* mh, int64_t rows) {
  Mh m;
  if (!mh || !unpack(mh, m)) return -1;
  int64_t w = fs2_conv_wgrad_ws_bytes(rows, m.d_in, m.n_mel, 1);
  for (int i = 0; i < m.layers; ++i) {
    const int64_t v = fs2_conv_wgrad_ws_bytes(rows, m.c_in(i), m.c_out(i), (int)m.taps);
    if (v > w) w = v;
  }
  return w;
}

int fs2_mel_head_fwd(const int64_t* mh, const void* x_t, void* act, int64_t rows, int64_t seq_len,
                     float p, const uint64_t* seed, void* stream) {
  Mh m;
  FS2_CHECK_ARG(mh && unpack(mh, m), "fs2_mel_head_fwd: bad descriptor");
  FS2_CHECK_ARG(x_t && act && seq_len > 0 && rows % seq_len == 0, "fs2_mel_head_fwd: bad arguments");
  FS2_CHECK_ARG(!(p > 0.f) || seed, "fs2_mel_head_fwd: dropout without seed");
  const MhAct A = mh_act(m, rows);
  const int64_t T = seq_len;
  const uint64_t* sd = p > 0.f ? seed : nullptr;
  lds_poison(as_stream(stream));
  float* ws = at<float>(act, A.ws);
  // mel_linear (fastspeech2.py:91) and its bf16 copy: the PostNet's input and residual
  float* out = at<float>(act, A.out);
  void* out_t = at<void>(act, A.out_t);
  FS2_TRY(fs2_conv_gemm(FS2_BF16, x_t, m.d_in, m.lin_wf, out, m.n_mel, rows, T, m.d_in, m.n_mel, 1,
                        0, nullptr, m.lin_b, FS2_EPI_BIAS, nullptr, m.n_mel, stream));
  FS2_TRY(fs2_cast_bf16(out, out_t, rows * m.n_mel, stream));
  // PostNet (Layers.py:126-137): conv -> BatchNorm (batch statistics, running update) ->
  // tanh (not the last) -> dropout; the last adds the residual
  const void* a = out_t;
  for (int i = 0; i < m.layers; ++i) {
    const MhLayer& L = m.l[i];
    const bool last = i == m.layers - 1;
    float* z = at<float>(act, A.z[i]);
    FS2_TRY(fs2_conv_gemm(FS2_BF16, a, m.c_in(i), L.w_f, z, m.c_out(i), rows, T, m.c_in(i), m.c_out(i),
                          (int)m.taps, (int)m.pad, nullptr, L.b, FS2_EPI_BIAS, nullptr, m.c_out(i),
                          stream));
    void* a_t = last ? nullptr : at<void>(act, A.a_t[i]);
    FS2_TRY(fs2_bn_fwd(last ? FS2_F32 : FS2_BF16, z, rows, m.c_out(i), L.bn_g, L.bn_b, kBnEps,
                       kBnMomentum, L.rm, L.rv, at<float>(act, A.mean[i]), at<float>(act, A.rstd[i]),
                       last ? 0 : 1, p, sd, (uint64_t)(m.site + i), last ? out : nullptr,
                       last ? at<float>(act, A.post) : nullptr, a_t, ws, A.ws_bytes, L.nbt, stream));
    a = a_t;
  }
  return FS2_OK;
}

int fs2_mel_head_bwd(const int64_t* mh, void* act, const void* x_t, const float* d_out,
                     const float* d_post, void* tmp, float* dx, int64_t rows, int64_t seq_len,
                     float p, const uint64_t* seed, float* side_ws, int64_t side_ws_bytes,
                     void* stream, void* side_stream) {
  Mh m;
  FS2_CHECK_ARG(mh && unpack(mh, m), "fs2_mel_head_bwd: bad descriptor");
  FS2_CHECK_ARG(act && x_t && tmp && dx && seq_len > 0 && rows % seq_len == 0,
                "fs2_mel_head_bwd: bad arguments");
  FS2_CHECK_ARG(d_out || d_post, "fs2_mel_head_bwd: no output gradient");
  FS2_CHECK_ARG(!(p > 0.f) || seed, "fs2_mel_head_bwd: dropout without seed");
  FS2_CHECK_ARG(side_ws && side_ws_bytes >= fs2_mel_head_side_ws_bytes(mh, rows),
                "fs2_mel_head_bwd: side-stream workspace too small");
  lds_poison(as_stream(stream));
  const MhAct A = mh_act(m, rows);
  const MhTmp W = mh_tmp(m, rows);
  const int64_t T = seq_len;
  const uint64_t* sd = p > 0.f ? seed : nullptr;
  void* side = side_stream ? side_stream : stream;
  float* ws = at<float>(tmp, W.ws);
  // dm = d_out + d_post: the mel_linear output feeds both outputs (fastspeech2.py:91-93)
  const float* dm = d_out;
  if (d_post) {
    float* acc = at<float>(tmp, W.dm);
    if (d_out) {
      FS2_TRY(fs2_add(acc, d_out, d_post, rows * m.n_mel, stream));
    } else {
      const hipError_t e = hipMemcpyAsync(acc, d_post, rows * m.n_mel * 4, hipMemcpyDeviceToDevice,
                                          as_stream(stream));
      if (e != hipSuccess) return FS2_ERR_LAUNCH;
    }
    // PostNet backward, last layer first; its input gradient is added into dm
    const float* d = d_post;
    for (int i = (int)m.layers - 1; i >= 0; --i) {
      const MhLayer& L = m.l[i];
      const bool last = i == m.layers - 1;
      void* dz_t = at<void>(tmp, W.dz_t[i]);
      FS2_TRY(fs2_bn_bwd(FS2_BF16, d, at<float>(act, A.z[i]), at<float>(act, A.mean[i]),
                         at<float>(act, A.rstd[i]), L.bn_g, L.bn_b, rows, m.c_out(i), last ? 0 : 1, p,
                         sd, (uint64_t)(m.site + i), nullptr, dz_t, L.gbn_g, L.gbn_b, ws, W.ws_bytes,
                         stream));
      const void* a = i == 0 ? at<void>(act, A.out_t) : at<void>(act, A.a_t[i - 1]);
      if (side != stream) FS2_TRY(fs2_stream_wait(side, stream));
      FS2_TRY(fs2_conv_wgrad(FS2_BF16, dz_t, m.c_out(i), a, m.c_in(i), L.gw, L.gb, rows, T,
                             m.c_in(i), m.c_out(i), (int)m.taps, (int)m.pad, nullptr, side_ws,
                             side_ws_bytes, side));
      if (i > 0) {
        float* dn = at<float>(tmp, W.d);
        FS2_TRY(fs2_conv_gemm(FS2_BF16, dz_t, m.c_out(i), L.w_b, dn, m.c_in(i), rows, T, m.c_out(i),
                              m.c_in(i), (int)m.taps, (int)m.pad, nullptr, nullptr, 0, nullptr,
                              m.c_in(i), stream));
        d = dn;
      } else {
        FS2_TRY(fs2_conv_gemm(FS2_BF16, dz_t, m.c_out(i), L.w_b, acc, m.c_in(i), rows, T, m.c_out(i),
                              m.c_in(i), (int)m.taps, (int)m.pad, nullptr, nullptr, FS2_EPI_ADD_AUX,
                              acc, m.c_in(i), stream));
      }
    }
    dm = acc;
  }
  // mel_linear: weight + bias gradient on the side stream, data gradient into dx
  void* dm_t = at<void>(tmp, W.dm_t);
  FS2_TRY(fs2_cast_bf16(dm, dm_t, rows * m.n_mel, stream));
  if (side != stream) FS2_TRY(fs2_stream_wait(side, stream));
  FS2_TRY(fs2_conv_wgrad(FS2_BF16, dm_t, m.n_mel, x_t, m.d_in, m.glin_w, m.glin_b, rows, T, m.d_in,
                         m.n_mel, 1, 0, nullptr, side_ws, side_ws_bytes, side));
  return fs2_conv_gemm(FS2_BF16, dm_t, m.n_mel, m.lin_wb, dx, m.d_in, rows, T, m.n_mel, m.d_in, 1, 0,
                       nullptr, nullptr, 0, nullptr, m.d_in, stream);
}

// ------------------------------------------------------------------ variance predictor
int64_t fs2_variance_predictor_act_bytes(const int64_t* vp, int64_t rows) {
  return vp ? vp_act(unpack_vp(vp), rows).total : -1;
}

int64_t fs2_variance_predictor_act_offset(const int64_t* vp, int64_t rows, int which) {
  if (!vp) return -1;
  const VpAct A = vp_act(unpack_vp(vp), rows);
  return which == FS2_VPA_PRED ? A.pred : -1;
}

int64_t fs2_variance_predictor_tmp_bytes(const int64_t* vp, int64_t rows) {
  return vp ? vp_tmp(unpack_vp(vp), rows).total : -1;
}

int64_t fs2_variance_predictor_side_ws_bytes(const int64_t* vp, int64_t rows) {
  if (!vp) return -1;
  const Vp v = unpack_vp(vp);
  const int64_t a = fs2_conv_wgrad_ws_bytes(rows, v.d, v.filt, (int)v.taps);
  const int64_t b = fs2_conv_wgrad_ws_bytes(rows, v.filt, v.filt, (int)v.taps);
  return a > b ? a : b;
}

int fs2_variance_predictor_fwd(const int64_t* vp, const void* x_t, void* act, int64_t rows,
                               int64_t seq_len, const int64_t* lens, float p, const uint64_t* seed,
                               void* stream) {
  FS2_CHECK_ARG(vp && x_t && act && seq_len > 0 && rows % seq_len == 0,
                "fs2_variance_predictor_fwd: bad arguments");
  FS2_CHECK_ARG(!(p > 0.f) || seed, "fs2_variance_predictor_fwd: dropout without seed");
  const Vp v = unpack_vp(vp);
  const VpAct A = vp_act(v, rows);
  const int64_t T = seq_len;
  const uint64_t* sd = p > 0.f ? seed : nullptr;
  lds_poison(as_stream(stream));
  float* h1 = at<float>(act, A.h1);
  void* u1_t = at<void>(act, A.u1_t);
  float* h2 = at<float>(act, A.h2);
  // Conv1d -> ReLU -> LN -> dropout (modules.py:207-229)
  FS2_TRY(fs2_conv_gemm(FS2_BF16, x_t, v.d, v.w1_f, h1, v.filt, rows, T, v.d, v.filt, (int)v.taps,
                        (int)v.pad1, nullptr, v.b1, FS2_EPI_BIAS | FS2_EPI_RELU, nullptr, v.filt,
                        stream));
  FS2_TRY(fs2_ln_fwd(FS2_BF16, h1, nullptr, v.ln1_g, v.ln1_b, at<float>(act, A.u1), u1_t,
                     at<float>(act, A.xh1), at<float>(act, A.rs1), nullptr, 1, rows, (int)v.filt, 0.f,
                     p, sd, 0, (uint64_t)v.site, nullptr, nullptr, nullptr, stream));
  // Conv1d (padding 1, modules.py:230) -> ReLU -> LN -> dropout -> Linear(., 1), masked
  FS2_TRY(fs2_conv_gemm(FS2_BF16, u1_t, v.filt, v.w2_f, h2, v.filt, rows, T, v.filt, v.filt,
                        (int)v.taps, (int)v.pad2, nullptr, v.b2, FS2_EPI_BIAS | FS2_EPI_RELU, nullptr,
                        v.filt, stream));
  return fs2_ln_fwd(FS2_F32, h2, nullptr, v.ln2_g, v.ln2_b, at<float>(act, A.u2), nullptr,
                    at<float>(act, A.xh2), at<float>(act, A.rs2), lens, T, rows, (int)v.filt, 0.f, p,
                    sd, 0, (uint64_t)(v.site + 1), v.lin_w, v.lin_b, at<float>(act, A.pred), stream);
}

int fs2_variance_predictor_bwd(const int64_t* vp, void* act, const void* x_t, const float* dpred,
                               void* tmp, float* dx_acc, int64_t rows, int64_t seq_len,
                               const int64_t* lens, float p, const uint64_t* seed, float* side_ws,
                               int64_t side_ws_bytes, void* stream, void* side_stream) {
  FS2_CHECK_ARG(vp && act && x_t && dpred && tmp && dx_acc && seq_len > 0 && rows % seq_len == 0,
                "fs2_variance_predictor_bwd: bad arguments");
  FS2_CHECK_ARG(!(p > 0.f) || seed, "fs2_variance_predictor_bwd: dropout without seed");
  FS2_CHECK_ARG(side_ws && side_ws_bytes >= fs2_variance_predictor_side_ws_bytes(vp, rows),
                "fs2_variance_predictor_bwd: side-stream workspace too small");
  lds_poison(as_stream(stream));
  const Vp v = unpack_vp(vp);
  const VpAct A = vp_act(v, rows);
  const VpTmp W = vp_tmp(v, rows);
  const int64_t T = seq_len;
  const uint64_t* sd = p > 0.f ? seed : nullptr;
  void* side = side_stream ? side_stream : stream;
  float* ws2 = at<float>(tmp, W.ws[0]);
  float* ws1 = at<float>(tmp, W.ws[1]);
  const void* u1_t = at<void>(act, A.u1_t);
  // LN2 (+ Linear, masked; ReLU mask; conv2 bias gradient) backward; its parameter gradients
  // (LN2 affine, Linear, conv2 bias) reduced on the side stream
  void* dh2_t = at<void>(tmp, W.dh2_t);
  // debug snapshots (fs2_debug_snap): the LN2 backward's inputs before and after it runs
  auto snap_in = [&]() {
    snap(dpred, rows * 4, as_stream(stream));
    snap(at<float>(act, A.xh2), rows * v.filt * 4, as_stream(stream));
    snap(at<float>(act, A.rs2), rows * 4, as_stream(stream));
    snap(at<float>(act, A.h2), rows * v.filt * 4, as_stream(stream));
    snap(v.lin_w, v.filt * 4, as_stream(stream));
    snap(v.ln2_g, v.filt * 4, as_stream(stream));
    snap(v.ln2_b, v.filt * 4, as_stream(stream));
  };
  snap_in();
  FS2_TRY(fs2_ln_bwd(FS2_BF16, nullptr, dpred, v.lin_w, at<float>(act, A.xh2), at<float>(act, A.rs2),
                     v.ln2_g, v.ln2_b, lens, T, rows, (int)v.filt, 0.f, p, sd, 0,
                     (uint64_t)(v.site + 1), at<float>(act, A.h2), nullptr, dh2_t, nullptr, 1,
                     nullptr, nullptr, nullptr, nullptr, nullptr, ws2, W.ws_bytes, stream));
  snap_in();
  snap(dh2_t, rows * v.filt * 2, as_stream(stream));
  snap(ws2, W.ws_bytes, as_stream(stream));
  if (side != stream) FS2_TRY(fs2_stream_wait(side, stream));
  FS2_TRY(fs2_ln_bwd_final(rows, (int)v.filt, ws2, 1, v.gln2_g, v.gln2_b, v.glin_w, v.glin_b, v.g2_b,
                           side));
  FS2_TRY(fs2_conv_wgrad(FS2_BF16, dh2_t, v.filt, u1_t, v.filt, v.g2_w, nullptr, rows, T, v.filt,
                         v.filt, (int)v.taps, (int)v.pad2, nullptr, side_ws, side_ws_bytes, side));
  float* du1 = at<float>(tmp, W.du1);
  FS2_TRY(fs2_conv_gemm(FS2_BF16, dh2_t, v.filt, v.w2_b, du1, v.filt, rows, T, v.filt, v.filt,
                        (int)v.taps, (int)v.pad2, nullptr, nullptr, 0, nullptr, v.filt, stream));
  // LN1 (ReLU mask; conv1 bias gradient) backward
  void* dh1_t = at<void>(tmp, W.dh1_t);
  FS2_TRY(fs2_ln_bwd(FS2_BF16, du1, nullptr, nullptr, at<float>(act, A.xh1), at<float>(act, A.rs1),
                     v.ln1_g, v.ln1_b, nullptr, 1, rows, (int)v.filt, 0.f, p, sd, 0, (uint64_t)v.site,
                     at<float>(act, A.h1), nullptr, dh1_t, nullptr, 1, nullptr, nullptr, nullptr,
                     nullptr, nullptr, ws1, W.ws_bytes, stream));
  snap(du1, rows * v.filt * 4, as_stream(stream));
  snap(dh1_t, rows * v.filt * 2, as_stream(stream));
  snap(ws1, W.ws_bytes, as_stream(stream));
  if (side != stream) FS2_TRY(fs2_stream_wait(side, stream));
  FS2_TRY(fs2_ln_bwd_final(rows, (int)v.filt, ws1, 0, v.gln1_g, v.gln1_b, nullptr, nullptr, v.g1_b,
                           side));
  FS2_TRY(fs2_conv_wgrad(FS2_BF16, dh1_t, v.filt, x_t, v.d, v.g1_w, nullptr, rows, T, v.d, v.filt,
                         (int)v.taps, (int)v.pad1, nullptr, side_ws, side_ws_bytes, side));
  return fs2_conv_gemm(FS2_BF16, dh1_t, v.filt, v.w1_b, dx_acc, v.d, rows, T, v.filt, v.d,
                       (int)v.taps, (int)v.pad1, nullptr, nullptr, FS2_EPI_ADD_AUX, dx_acc, v.d,
                       stream);
}

}  // extern "C"
