// Model handles behind the C-ABI (include/mec.h). Each handle owns its packed device
// weights and a grow-only activation workspace; forwards are asynchronous on the caller's
// stream. One handle is used by one host thread at a time (the Python wrapper locks).
#pragma once
#include "mec_common.h"

namespace mec {

enum ModelKind : int { KIND_SPEECH = 0, KIND_TEXT = 1, KIND_IMAGE = 2, KIND_FUSION = 3, KIND_IMAGE_MBV2 = 4, KIND_AUDIO = 5 };

size_t blob_floats(int kind);

// Arithmetic of a handle (mec_create_ex): PREC_F16 = f16 MFMA operands with fp32
// accumulation / LayerNorm / softmax / residual stream (the fast path); PREC_FP32 = every
// operand and product in fp32 (v_mfma_f32_32x32x2_f32), the reference's own precision.
// PREC_FP32X3 = fp32 arithmetic on the f16 MFMA: every fp32 GEMM operand x is carried as an
// exact pair of f16 planes x = hi + lo, and each product as hi.hi + hi.lo + lo.hi in one fp32
// accumulator (gemm_glds.hip split mode; 22 significant bits per operand against fp32's 24,
// the dropped lo.lo term below 2^-22 of the product); LayerNorm, softmax, attention, GELU, the
// residual stream and the heads are fp32 exactly as on the fp32 path.
enum Precision : int { PREC_F16 = 0, PREC_FP32 = 1, PREC_FP32X3 = 2 };

struct Model {
  int kind = -1;
  int device = 0;
  int prec = PREC_F16;
  Options opts = default_options();  // this handle's knobs (mec_model_set_option)
  TuneCache tune;                    // this handle's GEMM autotune results
  Prof prof;
  // fp32x3 handles: host-mapped pinned word (range_host) and its device view (range_dev), raised by
  // the kernels that write activation planes when a value leaves the f16 range (x3_raise)
  unsigned* range_host = nullptr;
  unsigned* range_dev = nullptr;
  int alloc_range_flag();
  // fp32x3 handles: one line per activation tensor (group) written at creation, "name s=<exponent>
  // bound=<bound or BN estimate>" plus the headroom the exponents were chosen with (mec_model_x3_report)
  std::string x3_report;
  void x3_note(const std::string& name, int s, double bound);
  virtual ~Model();
  // errors a kernel could only report after the fact (mec_model_check): 0 = none since the last
  // check. Call after the stream that ran the handle's forwards has been synchronized.
  virtual int check();
};

// ---------------------------------------------------------------- speech DNN
struct SpeechModel : Model {
  DevBuf w;  // fp32: mean, scale, {W,b,inv,shift} x5, W6, b6
  size_t off_mean = 0, off_scale = 0, off_W[6] = {}, off_b[6] = {}, off_inv[5] = {}, off_shift[5] = {};
  // speech_flow_kernel: hand-off buffers of layers 0-3 (f32 [16 * chunks, N_l]) and the
  // per-chunk arrival counters + the launch's error word (zeroed on the stream before every
  // launch); host_err: host-mapped pinned flag a launch with an expired wait raises
  DevBuf flow_act, flow_sync;
  int flow_chunks = 0;
  unsigned* host_err = nullptr;
  ~SpeechModel() override;
  int create(const float* blob, size_t n);
  int forward(const float* x, int B, float* feat, float* logits, float* probs, hipStream_t s);
  int check() override;
};

// ---------------------------------------------------------------- speech features (audio.hip)
// blob = [sample_rate, n_fft, hop, n_mels, n_mfcc] (config.py:57-59 + librosa defaults); the
// handle owns the filterbank / window / twiddle tables and a grow-only workspace.
struct AudioModel : Model {
  int sr = 22050, n_mfcc = 40, lo_bin = 0, hi_bin = 0, mel_nnz = 0, mel_ch = 0;
  DevBuf tables, ws;
  size_t off_hann = 0, off_tw = 0, off_post = 0, off_freq = 0, off_dct = 0, off_chroma = 0, off_meloff = 0,
         off_melbin = 0, off_melw = 0, off_melseg = 0;
  int create(const float* blob, size_t n);
  // wave f32 [B, L] -> feat f32 [B, n_mfcc + 16]; tuning f32 [B] (estimate_tuning) or null
  int forward(const float* wave, int B, int L, float* feat, float* tuning, hipStream_t s);
};

// ---------------------------------------------------------------- fusion model
struct FusionModel : Model {
  DevBuf w;  // fp32, transposed Linear weights ([in][out]) + biases + LN params
  std::vector<size_t> off;  // offsets by FusionParam index
  DevBuf ws;  // split form: projected (P) and fusion-projected (T) features, f32 [B, 768] each
  int ws_batch = 0;
  int create(const float* blob, size_t n);
  int forward(const float* sf, const float* tf, const float* imf, const float* sp, const float* tp,
              const float* ip, int B, float* logits, float* probs, float* attn_w, float* dec_w,
              hipStream_t s);
};

int fuse_weighted(const float* s, const float* t, const float* i, int B, double* out, hipStream_t st);
int fuse_weighted_f64(const double* s, const double* t, const double* i, int B, double* out, hipStream_t st);

// ---------------------------------------------------------------- BERT-base
struct TextModel : Model {
  DevBuf emb;      // fp32 word | pos | type | ln_g | ln_b
  DevBuf wts;      // f16 per layer: Wqkv[2304x768] Wo[768x768] Wi[3072x768] Wo2[768x3072]
  DevBuf prm;      // fp32 per layer: bqkv bo ln1g ln1b bi bo2 ln2g ln2b ; head: WpT bp WcT bc
  DevBuf wts32;    // fp32 path: the same GEMM weights in f32
  DevBuf ws;       // workspace
  int ws_tokens = 0;
  int create(const float* blob, size_t n);
  int forward(const int32_t* ids, const int32_t* mask, int B, int L, float* cls, float* logits,
              float* probs, hipStream_t s);
  int forward_f32(const int32_t* ids, const int32_t* mask, int B, int L, float* cls, float* logits,
                  float* probs, hipStream_t s);  // bert_f32.hip
  // fp32x3 path: wts holds the hi planes, then the lo planes (at x3_lo halfs); per GEMM B matrix
  // (4 per layer) the epilogue scale 2^-e of its planes
  size_t x3_lo = 0;
  std::vector<float> x3_scale;
  // activation-plane exponents (activation_exp, rigorous bounds): the embedding LN's, per layer LN1's,
  // LN2's, Q's, K's, V's (= the context's) and the FFN intermediate's; x3b: bq 2^s_q | bk 2^s_k | bv 2^s_v
  // per layer (the Wqkv planes carry the same factors). The epilogue scales in x3_scale already fold them
  // in (2^-e 2^(s_out - s_in))
  int x3_s_emb = 0;
  std::vector<int> x3_s_ln1, x3_s_ln2, x3_s_q, x3_s_k, x3_s_v, x3_s_ffn;
  DevBuf x3b;
  int forward_x3(const int32_t* ids, const int32_t* mask, int B, int L, float* cls, float* logits,
                 float* probs, hipStream_t s);  // bert_f32.hip
};
// lo != 0 (fp32x3 path): h16 is written as a hi plane and h16 + lo as the lo plane f16(y - hi)
// (planes of y up: up = 2^s, the planes' activation scale, activation_exp)
int launch_bert_embed_ln(const int32_t* ids, int M, int L, const float* emb, float* h32, f16* h16, hipStream_t s,
                         long long lo = 0, float up = 1.f);
int launch_bert_layernorm(const float* x, int M, const float* g, const float* b, float* h32, f16* h16, float2* stats,
                          hipStream_t s, long long lo = 0, float up = 1.f);
// fp32x3 attention (bert.hip): Q|K|V as f16 hi / lo planes [B*128, 2304] (lo at qkv + lo) of q 2^s_q,
// k 2^s_k, v 2^s_v; ctx 2^s_v written as hi / lo planes [B*128, 768] (lo at ctx + clo); qks = 1/8
// 2^-(s_q + s_k) (the scores' scale)
int launch_bert_attention_x3(const f16* qkv, long long lo, const int32_t* mask, f16* ctx, long long clo, int B,
                             float qks, hipStream_t s);
// its [CLS]-only form (bert_cls_last): K | V planes [B*128, 1536] (lo at kv + lo), the [CLS] query
// planes [B, 768] (lo at qc + qclo), the [CLS] context planes [B, 768] (lo at ctx + clo)
int launch_bert_attention_x3_cls(const f16* kv, long long lo, const int32_t* mask, const f16* qc, long long qclo,
                                 f16* ctx, long long clo, int B, float qks, hipStream_t s);

// fp32x3 QKV projection + attention of one (sequence, head pair) per workgroup (bert.hip, L = 128):
// h planes [B*128, 768] (lo at hs + hlo), Wqkv planes (lo at wqkv + wlo, epilogue scale oscale) ->
// ctx planes [B*128, 768] (lo at ctx + clo); Q / K / V never reach HBM
int launch_bert_qkv_attn_x3(const f16* hs, long long hlo, const f16* wqkv, long long wlo, float oscale,
                            const float* bqkv, const int32_t* mask, f16* ctx, long long clo, int B, float qks,
                            hipStream_t s);

// Split n fp32 weights into f16 planes for the fp32x3 path: hi = f16(w 2^e), lo = f16(w 2^e - hi)
// with e the largest power of two keeping max |w| 2^e <= 2^14 (so hi never overflows and lo
// stays out of the f16 subnormals for all but the smallest weights); returns 2^-e, the GEMM
// epilogue's oscale. Host code (runtime.hip).
float split_planes(const float* w, size_t n, f16* hi, f16* lo);

// fp32x3 activation planes. An activation x is carried as hi = f16(x 2^s), lo = f16(x 2^s - hi)
// with s fixed per tensor at handle creation; its consumer folds 2^-s into its epilogue scale (exact).
// The lo plane is a normal f16 -- 22 significant bits -- while |x 2^s| >= 2^-3, and hi stays finite
// while |x 2^s| < 65520. activation_exp(bound, target) = the largest s with bound 2^s <= target:
//   * a rigorous bound (BERT: LayerNorm outputs, |y| <= sqrt(H - 1) max|gamma| + max|beta|, and the
//     projections of such rows, max_j (bound ||W_j||_1 + |b_j|)) with target 2^15: never overflows;
//   * a BatchNorm estimate (ResNet50 / MobileNetV2: max_c |beta_c| + 6 |gamma_c| per BN output, summed
//     along residual paths) with target 2^10: 64x headroom to the f16 range over that estimate, and
//     the estimate's typical values near 2^7, far above the 2^-3 floor.
// Clamped to [-40, 40]; 0 for a zero or non-finite bound. Host code (runtime.hip).
int activation_exp(double bound, double target);
constexpr double kX3BoundTarget = 32768.0, kX3EstimateTarget = 1024.0;

// ---------------------------------------------------------------- image encoders
// Both backbones take the same u8 inputs and produce the same (512-d feature, logits, probs).
struct ImageNet : Model {
  // img u8 [B,H,W,C]: (48,48,1) gray FER2013 (GPU resize), (224,224,1) gray, (224,224,3) RGB
  virtual int forward_u8(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                         hipStream_t s) = 0;
  int forward(const uint8_t* gray, int B, float* feat, float* logits, float* probs, hipStream_t s) {
    return forward_u8(gray, B, 48, 48, 1, feat, logits, probs, s);
  }
};

// ---------------------------------------------------------------- ResNet50 + head
struct ConvLayer {
  size_t w_off = 0;   // f16 [Cout][kh][kw][Cin] (BN scale folded)
  size_t b_off = 0;   // f32 [Cout] (BN shift)
  int cin = 0, cout = 0, ks = 1, stride = 1, pad = 0;
  // fp32x3 path: the epilogue scale 2^-e 2^(x3_s - s_in) (weight planes' pre-scale, activation-plane
  // scales of output and input), the BN output estimate, the output planes' exponent x3_s, and the BN
  // shift times 2^x3_s (at x3b_off in prm)
  float x3_scale = 1.f;
  double x3_est = 0.0;
  int x3_s = 0;
  size_t x3b_off = 0;
};
struct Bottleneck {
  ConvLayer c1, c2, c3, ds;  // fp32x3: c3.x3_s = the stage's residual-stream exponent (the block output)
  int x3_s_in = 0;           // fp32x3: the block input planes' exponent
  bool has_ds = false;
  size_t c3ds_w_off = 0, c3ds_b_off = 0;  // block 0: [conv3 | downsample] weights [4w][w+cin], summed bias
  float c3ds_x3_scale = 1.f;              // fp32x3 path: its planes' scale (in wts_dual) and lo offset
  size_t c3ds_x3_lo = 0;
};
struct ImageModel : ImageNet {
  DevBuf wts;   // f16 conv weights
  DevBuf prm;   // fp32 biases, stem weights, head
  DevBuf ws;    // workspace
  int ws_batch = 0;
  ConvLayer stem;      // gray input (channels folded): f16 [64][64] pixel taps
  ConvLayer stem_rgb;  // RGB input: f16 [64][3*64]
  size_t stem_corr_off = 0;  // f32 [16 border classes][64] -mean/std term
  std::vector<Bottleneck> blocks;
  size_t fc1_off = 0, fc1b_off = 0, fc2_off = 0, fc2b_off = 0;
  // fp32 path (resnet_f32.hip): f32 weights, same [Cout][kh][kw][Cin] layout; the stem is a
  // [64][160] GEMM over an explicit im2col of the normalized image (k = c*49 + kh*7 + kw)
  DevBuf wts32;
  size_t stem_gray32_off = 0;  // f32 [49][2][64]: gray-input stem folded to (pixel, inside) taps
  int create(const float* blob, size_t n);
  int create_f32(const float* blob, size_t n);
  int forward_u8(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                 hipStream_t s) override;
  int forward_f32(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                  hipStream_t s);
  // fp32x3 path (resnet_f32.hip): wts holds every bottleneck conv's f16 hi planes, then the lo
  // planes at x3_lo halfs (w_off indexes both); the stem, pooling and head run as on the fp32 path
  size_t x3_lo = 0;
  float stem_x3_up = 1.f;  // 2^e: the gray stem's weight pre-scale (stem.x3_scale = 2^-e)
  int x3_s_out = 0;        // the last stage's activation-plane exponent (undone by the average pool)
  DevBuf wts_dual;  // fp32x3: block 0's [conv3 | downsample] hi / lo planes (c3ds_w_off, c3ds_x3_lo)
  int forward_x3(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                 hipStream_t s);
};

// ---------------------------------------------------------------- MobileNetV2 + head
// One inverted-residual block (features[1..17]) as packed for mbv2_block_kernel: channel
// counts padded (cin -> cinp % 32, hidden -> hidp % 32, cout -> coutp % 16) with zero weights.
struct MbBlock {
  int t = 1, cin = 0, hid = 0, cout = 0, stride = 1;
  int cinp = 0, hidp = 0, coutp = 0;
  size_t we_off = 0, wp_off = 0;          // f16: expand [hidp][cinp], project [coutp][hidp]
  size_t be_off = 0, wd_off = 0, bd_off = 0, bp_off = 0;  // f32: expand bias, dw [hidp/8][9][8], dw bias, project bias
  // fp32x3 layered form (hidp % 64 == 0): expand [hidp][lcinp], project [lcoutp][hidp] (lcoutp = cout padded
  // to 64, lcinp = the previous block's lcoutp), project bias [lcoutp]
  int lcinp = 0, lcoutp = 0;
  size_t lwe_off = 0, lwp_off = 0, lbp_off = 0;
  // fp32x3 activation planes (activation_exp, BN estimates): the block input's and output's exponents
  // (a stage's outputs share one, as a residual block's output and input must), the project BN
  // estimate, and the layered project bias times 2^x3_s_out (lbp_x3_off)
  int x3_s_in = 0, x3_s_out = 0;
  double x3_est = 0.0;
  size_t lbp_x3_off = 0;
};
struct MobileNetModel : ImageNet {
  DevBuf wts;   // f16 1x1 weights
  DevBuf prm;   // fp32 stem, depthwise weights, biases, head
  DevBuf ws;    // workspace
  int ws_batch = 0;
  size_t stem_w_off = 0, stem_rgb_off = 0, stem_corr_off = 0;  // f32 [9][32], [3*9][32], [4 classes][32]
  std::vector<MbBlock> blocks;
  size_t last_w_off = 0, last_b_off = 0;  // features[18]: f16 [1280][320], f32 [1280]
  size_t fc1_off = 0, fc1b_off = 0, fc2_off = 0, fc2b_off = 0;
  DevBuf wts32;  // fp32 path (mobilenet_f32.hip): f32 weights, channels padded to 64
  int create(const float* blob, size_t n);
  int create_f32(const float* blob, size_t n);
  int forward_u8(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                 hipStream_t s) override;
  int forward_f32(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                  hipStream_t s);
  // fp32x3 path (mobilenet_x3.hip): wts holds every 1x1 matrix's f16 hi planes (f16 path layouts), then
  // the lo planes at x3_lo halfs; x3_scale: per block (expand, project) epilogue scales, then features[18]
  size_t x3_lo = 0;
  std::vector<float> x3_scale;
  std::vector<float> lx3_scale;  // layered form: per block (expand, project) epilogue scales
  int create_x3(const float* blob, size_t n);
  int forward_x3(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                 hipStream_t s);
};

int resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, hipStream_t s);
// layer1 seam: conv3 (64 -> 256) + residual + ReLU, then the next block's conv1 (256 -> N2)
int launch_pw_chain(const f16* t2, const f16* xin, const f16* w3, const float* b3, const f16* w1, const float* b1,
                    f16* xout, f16* t1, int M, int N2, hipStream_t s);
// layer1 block 1 -> 2 seam: conv3 + downsample (K = [T2 | X0]) + ReLU, then block 2's conv1
int launch_pw_chain_dual(const f16* t2, const f16* x0, const f16* w3ds, const float* b3ds, const f16* w1,
                         const float* b1, f16* xout, f16* t1, int M, hipStream_t s);
// fp32x3 layer1 seam (pw_chain_x3.hip): the same two products on hi / lo planes (lo planes L
// elements after their hi planes; weight lo planes at w*_lo, pre-scales undone by os*); dual =
// conv3 + downsample over K = [T2 | X0] (xin = X0), else conv3 + identity residual (xin)
int launch_pw_chain_x3(const f16* t2, const f16* xin, long long L, const f16* w3, long long w3_lo, float os3,
                       const float* b3, const f16* w1, long long w1_lo, float os1, const float* b1, f16* xout, f16* t1,
                       int M, int N2, bool dual, hipStream_t s);
// fp32x3 layer-2 seam (pw_seam_x3.hip): conv3 (K3 = 128 -> 512) + identity residual + ReLU, then the next
// conv1 (512 -> N1 = 128 | 256), the block output walked in 32-channel chunks; any M (row tails masked)
int launch_pw_seam_x3(const f16* t2, const f16* xin, long long L, const f16* w3, long long w3_lo, float os3,
                      const float* b3, const f16* w1, long long w1_lo, float os1, const float* b1, f16* xout, f16* t1,
                      int M, int K3, int N1, hipStream_t s);


}  // namespace mec
