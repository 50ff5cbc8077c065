// extern "C" boundary (include/mec.h).
#include "../../include/mec.h"

#include <algorithm>
#include <cstdlib>
#include <exception>
#include <new>

#include "models.h"

namespace mec {
const char* last_error();

size_t blob_floats(int kind) {
  switch (kind) {
    case KIND_SPEECH: {
      const int d[6] = {56, 512, 512, 256, 128, 64};
      size_t s = 112;
      for (int i = 0; i < 5; ++i) s += (size_t)d[i] * d[i + 1] + 5 * d[i + 1];
      return s + 64 * 7 + 7;
    }
    case KIND_TEXT: {
      size_t s = (size_t)30522 * 768 + 512 * 768 + 2 * 768 + 2 * 768;
      const size_t layer = 4 * ((size_t)768 * 768 + 768) + 2 * 768 + ((size_t)3072 * 768 + 3072) +
                           ((size_t)768 * 3072 + 768) + 2 * 768;
      return s + 12 * layer + (size_t)768 * 768 + 768 + 7 * 768 + 7;
    }
    case KIND_IMAGE: {
      size_t s = 64 * 3 * 49 + 4 * 64;
      const int L[4][3] = {{64, 3, 1}, {128, 4, 2}, {256, 6, 2}, {512, 3, 2}};
      int cin = 64;
      for (int l = 0; l < 4; ++l)
        for (int b = 0; b < L[l][1]; ++b) {
          const int w = L[l][0];
          s += (size_t)w * cin + 4 * w + (size_t)w * w * 9 + 4 * w + (size_t)4 * w * w + 16 * w;
          if (b == 0) s += (size_t)4 * w * cin + 16 * w;
          cin = 4 * w;
        }
      return s + (size_t)512 * 2048 + 512 + 7 * 512 + 7;
    }
    case KIND_IMAGE_MBV2: {
      size_t s = 32 * 27 + 4 * 32;
      const int set[7][4] = {{1, 16, 1, 1}, {6, 24, 2, 2}, {6, 32, 3, 2}, {6, 64, 4, 2}, {6, 96, 3, 1}, {6, 160, 3, 2}, {6, 320, 1, 1}};
      int cin = 32;
      for (int i = 0; i < 7; ++i)
        for (int r = 0; r < set[i][2]; ++r) {
          const size_t t = set[i][0], hid = cin * t, cout = set[i][1];
          if (t != 1) s += hid * cin + 4 * hid;
          s += hid * 9 + 4 * hid + cout * hid + 4 * cout;
          cin = (int)cout;
        }
      return s + (size_t)1280 * 320 + 4 * 1280 + (size_t)512 * 1280 + 512 + 7 * 512 + 7;
    }
    case KIND_FUSION: {
      size_t s = 0;
      const int d[3] = {64, 768, 512};
      for (int m = 0; m < 3; ++m) s += (size_t)256 * d[m] + 256 + 512;
      s += 3 * ((size_t)768 * 256 + 768 + 256 * 256 + 256 + 512);
      s += 3 * ((size_t)256 * 256 + 256 + 512);
      s += (size_t)256 * 768 + 256 + 3 * 256 + 3 + 64 * 21 + 64 + 3 * 64 + 3;
      s += (size_t)256 * 263 + 256 + 512 + 128 * 256 + 128 + 7 * 128 + 7;
      return s;
    }
    case KIND_AUDIO: return 5;  // [sample_rate, n_fft, hop, n_mels, n_mfcc]
    default: return 0;
  }
}
}  // namespace mec

using namespace mec;

struct mec_model {
  Model* impl;
};

#define API_GUARD(body)                                  \
  try {                                                  \
    body                                                 \
  } catch (const std::bad_alloc&) {                      \
    set_error("host allocation failed");                 \
    return -1;                                           \
  } catch (const std::exception& e) {                    \
    set_error(e.what());                                 \
    return -1;                                           \
  }

static hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Image entry points take either backbone (ResNet50 or MobileNetV2).
static ImageNet* image_net(mec_model* m) {
  if (!m || !m->impl) { set_error("null model handle"); return nullptr; }
  if (m->impl->kind != KIND_IMAGE && m->impl->kind != KIND_IMAGE_MBV2) {
    set_error("model handle has the wrong kind for this call");
    return nullptr;
  }
  if (hipSetDevice(m->impl->device) != hipSuccess) { set_error("hipSetDevice failed"); return nullptr; }
  return static_cast<ImageNet*>(m->impl);
}

template <class T>
static T* as(mec_model* m, int kind) {
  if (!m || !m->impl) { set_error("null model handle"); return nullptr; }
  if (m->impl->kind != kind) { set_error("model handle has the wrong kind for this call"); return nullptr; }
  if (hipSetDevice(m->impl->device) != hipSuccess) { set_error("hipSetDevice failed"); return nullptr; }
  return static_cast<T*>(m->impl);
}

extern "C" {

const char* mec_version(void) { return "mec-hip 0.1 (gfx950)"; }
const char* mec_last_error(void) { return last_error(); }

long long mec_blob_size(int kind) {
  const size_t n = blob_floats(kind);
  return n ? (long long)n : -1;
}

int mec_create(int kind, const float* host_blob, size_t n, int device, mec_model** out) {
  return mec_create_ex(kind, host_blob, n, device, MEC_PREC_F16, out);
}

int mec_create_ex(int kind, const float* host_blob, size_t n, int device, int precision, mec_model** out) {
  return mec_create_opt(kind, host_blob, n, device, precision, nullptr, out);
}

int mec_create_opt(int kind, const float* host_blob, size_t n, int device, int precision, const char* opts,
                   mec_model** out) {
  API_GUARD({
    if (!out) { set_error("mec_create: out is null"); return -1; }
    if (precision != MEC_PREC_F16 && precision != MEC_PREC_FP32 && precision != MEC_PREC_FP32X3) {
      set_error("mec_create: precision must be MEC_PREC_F16, MEC_PREC_FP32 or MEC_PREC_FP32X3");
      return -1;
    }
    *out = nullptr;
    const size_t want = blob_floats(kind);
    if (!want) { set_error("mec_create: unknown kind"); return -1; }
    if (!host_blob || n != want) {
      set_error("mec_create: blob has " + std::to_string(n) + " floats, expected " + std::to_string(want));
      return -1;
    }
    // "key=value,key=value": this handle's knobs, applied over the process defaults before its weights are
    // packed (so creation-time knobs such as x3_headroom take effect)
    Options o = default_options();
    if (opts && *opts) {
      std::string all(opts);
      size_t pos = 0;
      while (pos <= all.size()) {
        const size_t end = std::min(all.find(',', pos), all.size());
        const std::string kv = all.substr(pos, end - pos);
        const size_t eq = kv.find('=');
        if (eq == std::string::npos || eq == 0) { set_error("mec_create_opt: bad option \"" + kv + "\" (key=value)"); return -1; }
        char* tail = nullptr;
        const long v = std::strtol(kv.c_str() + eq + 1, &tail, 10);
        if (!tail || *tail || tail == kv.c_str() + eq + 1) { set_error("mec_create_opt: bad value in \"" + kv + "\""); return -1; }
        if (set_option(o, kv.substr(0, eq), (int)v) != 0) return -1;
        pos = end + 1;
      }
    }
    MEC_HIP(hipSetDevice(device));
    Model* impl = nullptr;
    int rc = -1;
    switch (kind) {
      // speech and fusion are fp32 at either precision
      case KIND_SPEECH: { auto* p = new SpeechModel(); impl = p; p->opts = o; rc = p->create(host_blob, n); break; }
      case KIND_TEXT: { auto* p = new TextModel(); p->prec = precision; impl = p; p->opts = o; rc = p->create(host_blob, n); break; }
      case KIND_IMAGE: { auto* p = new ImageModel(); p->prec = precision; impl = p; p->opts = o; rc = p->create(host_blob, n); break; }
      case KIND_FUSION: { auto* p = new FusionModel(); impl = p; p->opts = o; rc = p->create(host_blob, n); break; }
      case KIND_IMAGE_MBV2: { auto* p = new MobileNetModel(); p->prec = precision; impl = p; p->opts = o; rc = p->create(host_blob, n); break; }
      case KIND_AUDIO: { auto* p = new AudioModel(); impl = p; p->opts = o; rc = p->create(host_blob, n); break; }
    }
    if (rc != 0) { delete impl; return -1; }
    impl->kind = kind;
    impl->device = device;
    impl->prec = (kind == KIND_SPEECH || kind == KIND_FUSION || kind == KIND_AUDIO) ? MEC_PREC_FP32 : precision;
    if (impl->prec == PREC_FP32X3 && impl->alloc_range_flag() != 0) { delete impl; return -1; }
    if (impl->prec == PREC_FP32X3)
      impl->x3_report = "x3_headroom=" + std::to_string(o.x3_headroom) + " x3_plane_scale=" +
                        std::to_string(o.x3_plane_scale) + "\n" + impl->x3_report;
    *out = new mec_model{impl};
    return 0;
  })
}

const char* mec_model_x3_report(mec_model* m) {
  if (!m || !m->impl) { set_error("mec_model_x3_report: null handle"); return nullptr; }
  return m->impl->x3_report.c_str();
}

int mec_destroy(mec_model* m) {
  if (!m) return 0;
  if (m->impl) (void)hipSetDevice(m->impl->device);
  delete m->impl;
  delete m;
  return 0;
}

int mec_speech_fwd(mec_model* m, const float* x, int B, float* feat, float* logits, float* probs, void* stream) {
  API_GUARD({
    auto* p = as<SpeechModel>(m, KIND_SPEECH);
    if (!p) return -1;
    OptScope sc(&p->opts, &p->tune, p->range_dev);
    return p->forward(x, B, feat, logits, probs, S(stream));
  })
}

int mec_text_fwd(mec_model* m, const int32_t* ids, const int32_t* mask, int B, int L, float* cls, float* logits,
                 float* probs, void* stream) {
  API_GUARD({
    auto* p = as<TextModel>(m, KIND_TEXT);
    if (!p) return -1;
    OptScope sc(&p->opts, &p->tune, p->range_dev);
    return p->forward(ids, mask, B, L, cls, logits, probs, S(stream));
  })
}

int mec_image_fwd(mec_model* m, const uint8_t* gray, int B, float* feat, float* logits, float* probs,
                  void* stream) {
  API_GUARD({
    auto* p = image_net(m);
    if (!p) return -1;
    OptScope sc(&p->opts, &p->tune, p->range_dev);
    return p->forward(gray, B, feat, logits, probs, S(stream));
  })
}

int mec_image_fwd_u8(mec_model* m, const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits,
                     float* probs, void* stream) {
  API_GUARD({
    auto* p = image_net(m);
    if (!p) return -1;
    OptScope sc(&p->opts, &p->tune, p->range_dev);
    return p->forward_u8(img, B, H, W, C, feat, logits, probs, S(stream));
  })
}

int mec_fusion_fwd(mec_model* m, const float* s_feat, const float* t_feat, const float* i_feat, const float* s_pred,
                   const float* t_pred, const float* i_pred, int B, float* logits, float* probs, float* attn_w,
                   float* dec_w, void* stream) {
  API_GUARD({
    auto* p = as<FusionModel>(m, KIND_FUSION);
    if (!p) return -1;
    OptScope sc(&p->opts, &p->tune, p->range_dev);
    return p->forward(s_feat, t_feat, i_feat, s_pred, t_pred, i_pred, B, logits, probs, attn_w, dec_w, S(stream));
  })
}

int mec_audio_fwd(mec_model* m, const float* wave, int B, int n_samples, float* feat, float* tuning, void* stream) {
  API_GUARD({
    auto* p = as<AudioModel>(m, KIND_AUDIO);
    if (!p) return -1;
    OptScope sc(&p->opts, &p->tune, p->range_dev);
    return p->forward(wave, B, n_samples, feat, tuning, S(stream));
  })
}

int mec_fuse_weighted(const float* s, const float* t, const float* i, int B, double* out, void* stream) {
  API_GUARD({ return fuse_weighted(s, t, i, B, out, S(stream)); })
}

int mec_fuse_weighted_f64(const double* s, const double* t, const double* i, int B, double* out, void* stream) {
  API_GUARD({ return fuse_weighted_f64(s, t, i, B, out, S(stream)); })
}

int mec_resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, void* stream) {
  API_GUARD({ return resize_u8(in, B, H, W, out, OH, OW, S(stream)); })
}

int mec_gemm_f16(const void* A, const void* B, const float* bias, const void* R, int r_is_f32, void* C16,
                 float* C32, int M, int N, int K, int act, void* stream) {
  API_GUARD({
    GemmParams g;
    g.A = A; g.B = reinterpret_cast<const f16*>(B); g.bias = bias; g.R = R; g.r_f32 = r_is_f32;
    g.C16 = reinterpret_cast<f16*>(C16); g.C32 = C32; g.M = M; g.N = N; g.K = K; g.act = act;
    return launch_gemm(g, S(stream), nullptr, TAG_NONE);
  })
}

int mec_gemm_f16x3(const void* A, long long a_lo, const void* B, long long b_lo, float oscale, const float* bias,
                   const float* R, void* C16, long long c_lo, float* C32, int M, int N, int K, int act,
                   void* stream) {
  API_GUARD({
    MEC_REQUIRE(a_lo != 0 && b_lo != 0, "mec_gemm_f16x3: a_lo / b_lo must locate the lo planes");
    GemmParams g;
    g.split = 1; g.A = A; g.a_lo = a_lo; g.B = reinterpret_cast<const f16*>(B); g.b_lo = b_lo; g.oscale = oscale;
    g.bias = bias; g.R = R; g.r_f32 = R != nullptr; g.C16 = reinterpret_cast<f16*>(C16); g.c_lo = C16 ? c_lo : 0;
    g.C32 = C32; g.M = M; g.N = N; g.K = K; g.act = act;
    return launch_gemm(g, S(stream), nullptr, TAG_NONE);
  })
}

int mec_conv_f16(const void* x, const void* w, const float* bias, const void* R, void* y, int n, int H, int W,
                 int C, int Cout, int ks, int stride, int pad, int act, void* stream) {
  API_GUARD({
    GemmParams g;
    g.amode = A_CONV; g.A = x; g.B = reinterpret_cast<const f16*>(w); g.bias = bias; g.R = R;
    g.C16 = reinterpret_cast<f16*>(y); g.act = act;
    g.H = H; g.W = W; g.C = C; g.ks = ks; g.stride = stride; g.pad = pad;
    g.OH = (H + 2 * pad - ks) / stride + 1; g.OW = (W + 2 * pad - ks) / stride + 1;
    g.M = n * g.OH * g.OW; g.N = Cout; g.K = ks * ks * C;
    return launch_gemm(g, S(stream), nullptr, TAG_NONE);
  })
}

}  // extern "C"

namespace mec {
// One knob of `o` (include/mec.h lists them). The probe-build values (*_debug, bert_qkv_attn
// 2 | 3, speech_spin_limit >= 0) return wrong results and exist only in -DMEC_PROBES builds.
int set_option(Options& o, const std::string& k, int value) {
  const bool probe = kProbes;
  if (k == "fusion_r" && (value == 1 || value == 2 || value == 4)) { o.fusion_r = value; return 0; }
  if (k == "gemm_f32_family" && (value == 0 || value == 16 || value == 32)) {
    o.gemm_f32_family = value;
    return 0;
  }
  if (k == "bert_cls_last" && (value == 0 || value == 1)) { o.bert_cls_last = value; return 0; }
  if (k == "gemm_x3_order" && (value == 0 || value == 1)) { o.gemm_x3_order = value; return 0; }
  if (k == "gelu_x3" && (value == 0 || value == 1)) { o.gelu_x3 = value; return 0; }
  if (k == "bert_ln_rows" && (value == 1 || value == 2 || value == 4)) {
    o.bert_ln_rows = value;
    return 0;
  }
  if (k == "gemm_group_m" && (value == 0 || value == 2 || value == 4 || value == 8 || value == 16)) {
    o.gemm_group_m = value;
    return 0;
  }
  if (k == "gemm_glds_group_m" && (value == 0 || value == 2 || value == 4 || value == 8 || value == 16)) {
    o.gemm_glds_group_m = value;
    return 0;
  }
  if (k == "fusion_split" && (value == 0 || value == 1)) { o.fusion_split = value; return 0; }
  if (k == "speech_spin_limit" && (value == -1 || (probe && value >= 0))) { o.speech_spin_limit = value; return 0; }
  if (k == "gemm_debug" && (value == 0 || (probe && value >= 1 && value <= 6))) { o.gemm_debug = value; return 0; }
  if (k == "gemm_autotune" && (value == 0 || value == 1)) { o.gemm_autotune = value; return 0; }
  if (k == "gemm_f32_tile" && value >= 0 && value <= 8) { o.gemm_f32_tile = value; return 0; }
  if (k == "gemm_f32_tag" && value >= 0 && value / 100000 > 0 && value / 100000 < TAG_COUNT && value % 100000 <= 8) {
    o.gemm_f32_tag[value / 100000] = value % 100000;
    return 0;
  }
  if (k == "gemm_prefetch_r" && (value == 0 || value == 1)) { o.gemm_prefetch_r = value; return 0; }
  if (k == "mbv2_impl" && value >= 0 && value <= 2) { o.mbv2_impl = value; return 0; }
  if (k == "mbv2_x3_tile" && (value == 0 || value == 4)) { o.mbv2_x3_tile = value; return 0; }
  if (k == "mbv2_x3_tpw" && value >= 1 && value <= 16) { o.mbv2_x3_tpw = value; return 0; }
  if (k == "mbv2_x3_occ" && (value == 3 || value == 4)) { o.mbv2_x3_occ = value; return 0; }
  if (k == "mbv2_x3_sesw" && (value == 0 || value == 1)) { o.mbv2_x3_sesw = value; return 0; }
  if (k == "x3_plane_scale" && (value == 0 || value == 1)) { o.x3_plane_scale = value; return 0; }
  if (k == "x3_headroom" && value >= 0 && value <= 24) { o.x3_headroom = value; return 0; }
  if (k == "gemm_x3_restage" && value >= 0 && value <= 2) { o.gemm_x3_restage = value; return 0; }
  if (k == "gemm_x3_stagger" && value >= 0 && value <= 200) { o.gemm_x3_stagger = value; return 0; }
  if (k == "gemm_x3_late_dma" && value >= 0 && value <= 3) { o.gemm_x3_late_dma = value; return 0; }
  if (k == "gemm_x3_prio" && (value == 0 || value == 1)) { o.gemm_x3_prio = value; return 0; }
  if (k == "qkv_x3_late_dma" && value >= 0 && value <= 2) { o.qkv_x3_late_dma = value; return 0; }
  if (k == "mbv2_layered" && (value == 0 || (value >= 7 && value <= 17))) { o.mbv2_layered = value; return 0; }
  if (k == "mbv2_layered16" && (value == 0 || (value >= 7 && value <= 17))) { o.mbv2_layered16 = value; return 0; }
  if (k == "conv3x3_direct" && (value == 0 || value == 1)) { o.conv3x3_direct = value; return 0; }
  if (k == "conv3x3_halo" && (value == 0 || value == 1)) { o.conv3x3_halo = value; return 0; }
  if (k == "stem_gray_f32" && (value == 0 || value == 1)) { o.stem_gray_f32 = value; return 0; }
  if (k == "resnet_chunk" && value >= 0) { o.resnet_chunk = value; return 0; }
  if (k == "bert_qkv_attn" && (value == 0 || value == 1 || (probe && (value == 2 || value == 3)))) {
    o.bert_qkv_attn = value;
    return 0;
  }
  if (k == "stem_debug" && (value == 0 || (probe && (value == 1 || value == 2 || value == 4 || value == 7)))) {
    o.stem_debug = value;
    return 0;
  }
  if (k == "pw_chain" && (value >= 0 && value <= 2)) { o.pw_chain = value; return 0; }
  if (k == "pw_chain_form" && (value >= 0 && value <= 2)) { o.pw_chain_form = value; return 0; }
  if (k == "pw_chain_x3" && (value >= 0 && value <= 2)) { o.pw_chain_x3 = value; return 0; }
  if (k == "pw_seam_x3" && (value >= 0 && value <= 2)) { o.pw_seam_x3 = value; return 0; }
  if (k == "bert_qkv_attn_x3_heads" && (value == 1 || value == 2)) { o.bert_qkv_attn_x3_heads = value; return 0; }
  if (k == "bert_qkv_attn_heads" && (value == 1 || value == 2)) { o.bert_qkv_attn_heads = value; return 0; }
  if (k == "conv3x3_debug" && (value == 0 || (probe && (value == 1 || value == 2 || value == 4 || value == 7)))) {
    o.conv3x3_debug = value;
    return 0;
  }
  if (k == "speech_debug" && (value == 0 || (probe && value == 1))) {
    o.speech_debug = value;
    return 0;
  }
  if (k == "audio_debug" && (value == 0 || (probe && (value == 1 || value == 2 || value == 4 || value == 8 || value == 15 ||
                                                       value == 32 || value == 64 || value == 96 || value == 128)))) {
    o.audio_debug = value;
    return 0;
  }
  auto tile_ok = [](int id) {
    const int v = id % 10000;
    const bool deep = id == 20256 || id == 30256 || id == 20128 || id == 40256 || id == 41256 || id == 50128 ||
                      id == 60128 || id == 50256 || id == 70256 || id == 70128 || id == 71128 || id == 71064 ||
                      id == 70064 || id == 72128;
    return id == 0 || deep || (id < 20000 && (v == 64 || v == 128 || v == 256 || v == 1064 || v == 1128));
  };
  if (k == "gemm_bn" && tile_ok(value)) {
    o.gemm_bn = value;
    return 0;
  }
  // one launch class only: value = tag * 100000 + tile id (tags: mec_common.h KernelTag)
  if (k == "gemm_bn_tag" && value >= 0 && value / 100000 > 0 && value / 100000 < TAG_COUNT && tile_ok(value % 100000)) {
    o.gemm_bn_tag[value / 100000] = value % 100000;
    return 0;
  }
  if (k == "gemm_x3_tag" && value >= 0 && value / 100000 > 0 && value / 100000 < TAG_COUNT &&
      (value % 100000 == 0 || (value % 100000 >= 70000 && tile_ok(value % 100000)))) {
    o.gemm_x3_tag[value / 100000] = value % 100000;
    return 0;
  }
  set_error("mec_set_option: unknown key or bad value: " + k + " = " + std::to_string(value) +
            (probe ? "" : " (probe values need a -DMEC_PROBES build)"));
  return -1;
}
}  // namespace mec

extern "C" {

int mec_set_option(const char* key, int value) { return set_option(default_options(), key ? key : "", value); }

int mec_model_set_option(mec_model* m, const char* key, int value) {
  if (!m || !m->impl) { set_error("null model handle"); return -1; }
  const std::string k = key ? key : "";
  if (k == "x3_plane_scale" || k == "x3_headroom") {  // read while the weights are packed: too late here
    set_error("mec_model_set_option: \"" + k + "\" is a creation-time option (pass it to mec_create_opt, or set "
              "the process default with mec_set_option before mec_create_ex)");
    return -1;
  }
  return set_option(m->impl->opts, k, value);
}

int mec_build_flags(void) { return kProbes ? MEC_BUILD_PROBES : 0; }

int mec_model_gemm_query(mec_model* m, int amode, int M, int N, int K) {
  if (!m || !m->impl) { set_error("null model handle"); return -1; }
  OptScope sc(&m->impl->opts, &m->impl->tune);
  return m->impl->prec == PREC_FP32 ? gemm_f32_tuned(amode, M, N, K) : gemm_tuned_bn(amode, M, N, K);
}

int mec_gemm_query(int amode, int M, int N, int K) { return gemm_tuned_bn(amode, M, N, K); }

int mec_gemm_f32_query(int amode, int M, int N, int K) { return gemm_f32_tuned(amode, M, N, K); }

int mec_precision(const mec_model* m) {
  if (!m || !m->impl) { set_error("null model handle"); return -1; }
  return m->impl->prec;
}

int mec_gemm_f32(const float* A, const float* B, const float* bias, const float* R, float* C, int M, int N, int K,
                 int act, void* stream) {
  API_GUARD({
    GemmParams g;
    g.A = A; g.B32 = B; g.bias = bias; g.R = R; g.r_f32 = 1; g.C32 = C; g.M = M; g.N = N; g.K = K; g.act = act;
    return launch_gemm_f32(g, S(stream), nullptr, TAG_NONE);
  })
}

int mec_conv_f32(const float* x, const float* w, const float* bias, const float* R, float* y, int n, int H, int W,
                 int C, int Cout, int ks, int stride, int pad, int act, void* stream) {
  API_GUARD({
    GemmParams g;
    g.amode = A_CONV; g.A = x; g.B32 = w; g.bias = bias; g.R = R; g.r_f32 = 1; g.C32 = y; g.act = act;
    g.H = H; g.W = W; g.C = C; g.ks = ks; g.stride = stride; g.pad = pad;
    g.OH = (H + 2 * pad - ks) / stride + 1; g.OW = (W + 2 * pad - ks) / stride + 1;
    g.M = n * g.OH * g.OW; g.N = Cout; g.K = ks * ks * C;
    return launch_gemm_f32(g, S(stream), nullptr, TAG_NONE);
  })
}

int mec_prof_enable(mec_model* m, int tag) {
  if (!m || !m->impl) { set_error("null model handle"); return -1; }
  m->impl->prof.tag = tag;
  m->impl->prof.reset();
  return 0;
}

int mec_model_check(mec_model* m) {
  if (!m || !m->impl) { set_error("mec_model_check: null handle"); return -1; }
  return m->impl->check();
}

int mec_prof_read(mec_model* m, double* total_ms, int* count) {
  if (!m || !m->impl || !total_ms || !count) { set_error("mec_prof_read: bad args"); return -1; }
  return m->impl->prof.read(total_ms, count);
}

}  // extern "C"
