// Shared definitions for the MI355X (gfx950) emotion-inference HIP library.
#pragma once
#include <hip/hip_runtime.h>
#include <array>
#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

typedef _Float16 f16;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace mec {

void set_error(const std::string& msg);

#define MEC_HIP(x)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      ::mec::set_error(std::string(#x) + " failed: " + hipGetErrorString(e_) + " @" +     \
                       __FILE__ + ":" + std::to_string(__LINE__));                        \
      return -1;                                                                          \
    }                                                                                     \
  } while (0)

#define MEC_REQUIRE(cond, msg)                                                            \
  do {                                                                                    \
    if (!(cond)) {                                                                        \
      ::mec::set_error(std::string("requirement failed: ") + (msg));                     \
      return -1;                                                                          \
    }                                                                                     \
  } while (0)

#define MEC_TRY(x)                                                                        \
  do {                                                                                    \
    if ((x) != 0) return -1;                                                              \
  } while (0)

#define MEC_LAUNCH_CHECK() MEC_HIP(hipGetLastError())

// Kernel tags for the hipEvent timing hook (mec_prof_enable); see DESIGN.md §Measurement.
enum KernelTag : int {
  TAG_NONE = 0,
  TAG_BERT_QKV = 1,
  TAG_BERT_ATTN = 2,
  TAG_BERT_OPROJ = 3,
  TAG_BERT_FFN1 = 4,
  TAG_BERT_FFN2 = 5,
  TAG_BERT_LN = 6,
  TAG_RESNET_CONV3X3 = 7,
  TAG_RESNET_CONV1X1 = 8,
  TAG_RESNET_STEM = 9,
  TAG_SPEECH = 10,
  TAG_FUSION = 11,
  TAG_MBV2_BLOCK = 12,
  TAG_MBV2_LAST = 13,
  TAG_AUDIO = 14,
  TAG_COUNT = 15,
};

// Tuning knobs (mec_set_option / mec_model_set_option, include/mec.h). Every model handle
// owns a copy, taken from the process defaults when it is created, and kernels read the
// options of the handle whose call they serve (opt()), so handles never perturb each other.
// Every setting of a knob gives the same results bit for bit, with these exceptions:
//   * conv3x3_halo 0 vs 1, fusion_r 4 vs 1|2 and gemm_x3_order 0 vs 1 sum in other fp32 orders,
//     gelu_x3 0 vs 1 evaluates erf another way (same values to rounding, not the same bits;
//     include/mec.h);
//   * the probe-build values (compiled only with -DMEC_PROBES: they skip work to time a
//     kernel's parts and return wrong results).
struct Options {
  int gemm_bn = 0;          // forced f16 GEMM tile id (0 = autotune)
  int gemm_autotune = 1;
  int gemm_prefetch_r = 1;  // f16 (and split hi / lo) residual prefetch in short-K GEMMs
  int gemm_f32_tile = 0;    // forced fp32 GEMM tile id (0 = autotune)
  // fp32 autotune family: 0 both, 16 = 16x16x4 tiles only, 32 = 32x32x2 only. 16 (default): one k
  // order for every shape, so the fp32 path is batch-invariant bit for bit, at no measured cost
  // (ResNet50 20.73 vs 20.77 ms, BERT 45.95 vs 45.85 ms at B = 256; tools/ab_f32_family.py)
  int gemm_f32_family = 16;
  // fp32 engine, per launch class: BERT FFN1 pinned to 256x256 on 16x16x4 (it and the 32x32x2
  // form time within 0.3%, so the autotune flipped between them run to run)
  int gemm_f32_tag[TAG_COUNT] = {0, 0, 0, 0, /*TAG_BERT_FFN1*/ 8};
  // per launch class (profiling tag): forced tile, 0 = autotune. The BERT O-projection is
  // pinned to 128 x 128 (its candidates time within 2% alone; in the encoder 128 x 128 wins)
  int gemm_bn_tag[TAG_COUNT] = {0, 0, 0, /*TAG_BERT_OPROJ*/ 11128};
  int conv3x3_direct = 1;   // ResNet layer1 conv2 on the halo-tile kernel (conv3x3.hip)
  int conv3x3_halo = 1;     // layers 2-3 stride-1 conv2 on the halo kernel (conv3x3_halo.hip)
  int stem_gray_f32 = 1;    // fp32 gray stem as one conv + pool kernel (else im2col + GEMM + pool)
  int resnet_chunk = 0;
  int pw_chain = 2;         // layer1 seam kernels (pw_chain.hip)
  int pw_chain_form = 0;
  // fp32x3 layer1 seam kernels (pw_chain_x3.hip): 0 off, 1 the 256 -> 64 seams (block 1 -> 2 with
  // the downsample, 2 -> 3), 2 also the 256 -> 128 seam into layer2
  int pw_chain_x3 = 2;
  // fp32x3 layer-2 seam kernels (pw_seam_x3.hip): 0 off, 1 the 512 -> 128 seams (blocks 2 -> 3, 3 -> 4),
  // 2 also the 512 -> 256 seam into layer3's first conv1 (whole-batch runs only: resnet_chunk 0). Same bits
  // at every setting. Per seam at B = 256: 512 -> 128 356-364 us against 379 for the two split GEMMs,
  // 512 -> 256 477 against 451 (profiles/r06l_seam_*.txt): 1 by default
  int pw_seam_x3 = 1;
  int bert_qkv_attn = 1;    // fused BERT QKV projection + attention
  // fp32x3 fused QKV + attention: heads per workgroup (2: 8 waves, 128 KB of LDS, one per CU; 1: 4 waves,
  // 80 KB, two per CU so one's attention overlaps the other's GEMM); same bits
  int bert_qkv_attn_x3_heads = 1;
  int bert_qkv_attn_heads = 1;  // the same for the f16 fused kernel (bert_qkv_attn_kernel)
  int bert_ln_rows = 2;     // BERT LayerNorm rows per wave (1 | 2 | 4): 27.0 / 25.7 / 26.3 us at B = 256
  // BERT's last layer on the [CLS] rows only (the outputs -- pooler, logits, CLS feature -- read
  // nothing else of it): K / V for every token, Q, attention, O-projection, LayerNorms and FFN for
  // the B [CLS] rows. Same bits as the full layer (every kernel is row-independent; the attention
  // computes the [CLS] query with the full kernel's instruction sequence). 0 = the full layer
  int bert_cls_last = 1;
  int mbv2_impl = 0;
  // fp32x3 MobileNetV2, stride-2 blocks at 56 / 28 outputs: 4 = 4x4 output tiles (9x9 inputs, four
  // workgroups per CU), 0 = 8x8 / 7x7 (17x17 / 15x15 inputs, one per CU); same bits. 4: 2.99 -> 2.92 ms
  // at B = 256 (profiles/r04_ab_mbv2x3_tile.txt)
  int mbv2_x3_tile = 4;
  int mbv2_x3_tpw = 2;  // fp32x3 MobileNetV2 fused blocks: output tiles per workgroup (next tile's input prefetched)
  // fp32x3 MobileNetV2 4x4-tile (stride-2) fused blocks: workgroups per CU their registers are allocated for
  // (4: 128 VGPRs and an 84-B spill per lane; 3: 168 VGPRs, no spill); same bits
  int mbv2_x3_occ = 3;
  // fp32x3 activation-plane scales (models.h activation_exp), read when a handle is created: 1 = per-tensor
  // exponents from bounds / BN estimates, 0 = every exponent 0 (round 4's unscaled planes; A/B only: small
  // activations then lose bits to the f16 subnormals, large ones overflow)
  int x3_plane_scale = 1;
  // fp32x3 extra headroom, read when a handle is created: every activation-plane exponent is chosen for a
  // target 2^-x3_headroom times the default (models.h activation_exp), so the planes take values that many
  // binades above the bound / BN estimate before the range flag trips. engine.HipModel re-creates a handle
  // with more headroom after a trip (the batch itself is re-run on the fp32 engine)
  int x3_headroom = 0;
  // fp32x3 MobileNetV2 fused blocks: the expanded chunk's f32 rows with a per-tile-shape 16-B chunk swizzle
  // (1; fewer LDS bank conflicts on the depthwise reads) or unswizzled 36-float rows (0); same bits
  int mbv2_x3_sesw = 1;
  // fp32x3 MobileNetV2: features[k..17] as expand GEMM -> depthwise kernel -> project GEMM on hi / lo
  // planes (the "layered" form; k = 7..17, 0 = every block fused but features[17], which is always layered)
  int mbv2_layered = 8;
  int mbv2_layered16 = 8;  // the same on the f16 path (features[k..17] on f16 GEMMs; 0 = every block fused)
  // ping-pong GEMM tile order inside each XCD's contiguous tile range: 0 = row-major (all N
  // panels of one M panel in turn), G = groups of G M panels walked M-fastest, so the 32
  // tiles an XCD runs at once share G A panels and 32/G weight panels
  // (8: FFN1 reads 290 -> 227 MB per launch at B = 256, time unchanged; profiles/ffn1_traffic_gm*.json)
  int gemm_group_m = 8;
  // the same tile order for the multi-stage (glds) engine, every tile and A mode; 0 = row-major
  // (8: the fp32x3 FFN1 reads 911 -> 663 MB per launch at B = 256, time unchanged;
  // profiles/ffn1_x3_traffic*.json)
  int gemm_glds_group_m = 8;
  // split-f16 (fp32x3) GEMM term order: 0 = pass-major (all of K for lo.hi, then hi.lo, then
  // hi.hi), 1 = K-interleaved (each 32-deep k chunk's three terms back to back; tiles 7xxxx). Both
  // are fp32-accurate; they sum in different orders (not the same bits). 1: every operand byte is
  // fetched and staged once (not 1.5x) and 4 fragment reads feed 3 MFMAs (not 6): less energy per
  // MFMA, a higher held clock: text 18.84 -> 17.96 ms, ResNet50 10.06 -> 9.00, fused step 28.05 ->
  // 26.19 ms at B = 256 (profiles/r03_ab_x3order_*.txt)
  int gemm_x3_order = 1;
  // K-interleaved split tiles with a 2-stage ring (70256, 71128, 71064, 70064): early restage (a stage is
  // refilled for k step t + 2 as soon as every wave holds step t's fragments: two steps in flight) for
  // 1 = every A mode, 2 = the implicit-GEMM convs only (ResNet), 0 = none (the ring refilled after the barrier
  // of step t: one step in flight); same bits. Measured (same process, B = 256): ResNet50 alone gains up to
  // 1 % (8.79 -> 8.71 ms), but the fused step loses 0.8 % (2) / 1.7 % (1) and BERT up to 0.9 %: 0 by default
  // (profiles/r05_ab_restage_*.txt)
  int gemm_x3_restage = 0;
  // split tiles with two or more workgroups per CU: the later-dispatched workgroups of the first pass start
  // this many microseconds late (GemmParams::stagger), desynchronizing co-resident workgroups; 0 = off
  int gemm_x3_stagger = 0;
  // interleaved split tiles (not the restage schedule): the second wave of each SIMD issues its share of the
  // next stage's LDS DMA after its first term group of MFMAs (1), after its second (2), or its hi planes after
  // the first and lo planes after the second (3), not right after the step's barrier (0), so the two waves of
  // a SIMD do not both sit in DMA issue while the matrix core idles; same bits. 1: fused fp32x3 step -1.2 /
  // -1.6 %, BERT alone -0.7 / -1.4 %, ResNet50 neutral (profiles/r06f_ab_late_dma.txt, r06g_ab_late_dma.txt)
  int gemm_x3_late_dma = 1;
  // the same kernels: MFMA sections at wave priority 1, DMA issue and barriers at 0 (A/B knob)
  int gemm_x3_prio = 0;
  // fp32x3 fused QKV + attention (one head per workgroup): every other 256-block of workgroups issues its stage
  // refill after its first (1) or second (2) MFMA term group instead of right after the barrier (0); same bits
  int qkv_x3_late_dma = 0;
  // K-interleaved split engine, per launch class: forced tile (7xxxx), 0 = autotune. BERT FFN1 is
  // pinned to 70256 by default: it and the other tiles time within a few % of each other alone, so an
  // autotune would flip between them run to run, and the bench's roofline kernel (and its PMC traffic
  // file) must be one kernel. BERT FFN2 is pinned to the one-stage 72128 (two workgroups per CU: BERT
  // alone 17.44 -> 17.12 ms, profiles/r05l_ab_tile72128_text_fp32x3.txt), a tile the autotuner does not
  // offer: where the autotuner took it for a ResNet50 1x1 conv, and the one-stage 128-row tiles for most of
  // them, the image leg ran faster alone but the fused step slower (profiles/r05s_ab_tile73xxx_*.txt). The
  // fused step (FusedPipeline) pins FFN2 back to 70256 (profiles/r05m_ab_x3tag_ffn2.txt). A pin applies only
  // where its grid fills at least half the chip (kX3PinMinTiles tiles: FFN1 from B = 22; the one-stage 72128 from 512
  // tiles, two workgroups on every CU: FFN2 from B = 171, gemm.hip): a small batch
  // (latency-mode text inference) autotunes among the 7xxxx tiles instead, which give the same bits
  int gemm_x3_tag[TAG_COUNT] = {0, 0, 0, 0, /*TAG_BERT_FFN1*/ 70256, /*TAG_BERT_FFN2*/ 72128};
  // fp32x3 BERT FFN1 GELU: 1 = ACT_GELU_F32 (branch-free erf, one-instruction exp; max |error| /
  // max(|x|, 1) 1.21e-7 against float64, the correctly rounded erf's 1.06e-7), 0 = libm erff
  int gelu_x3 = 1;
  int fusion_r = 4;         // samples per fusion workgroup
  int fusion_split = 1;     // fusion as 3 launches
  int gemm_debug = 0, conv3x3_debug = 0, stem_debug = 0, audio_debug = 0, speech_debug = 0;  // probe builds only
  int speech_spin_limit = -1;  // probe builds only: speech_flow_kernel wait limit (forces expired waits)
};

constexpr long kX3PinMinTiles = 128;  // gemm_x3_tag pins apply from this many tiles (half of 256 CUs)

// GEMM autotuner results: tile id per (engine, shape), per handle.
struct TuneCache {
  std::map<std::array<int, 11>, int> m;
  std::mutex mu;
  int find(const std::array<int, 11>& k) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = m.find(k);
    return it == m.end() ? 0 : it->second;
  }
  void put(const std::array<int, 11>& k, int v) {
    std::lock_guard<std::mutex> lk(mu);
    m[k] = v;
  }
  int find_shape(int engine, int amode, int M, int N, int K) {  // any geometry
    std::lock_guard<std::mutex> lk(mu);
    for (const auto& kv : m)
      if (kv.first[0] == engine && kv.first[1] == amode && kv.first[2] == M && kv.first[3] == N && kv.first[4] == K)
        return kv.second;
    return 0;
  }
};

Options& default_options();      // process defaults (mec_set_option), copied into new handles
TuneCache& default_tune_cache(); // for the handle-less kernel entry points
const Options& opt();            // options of the handle the calling thread is serving
TuneCache& tune_cache();         // its autotune cache
// its fp32x3 range flag (device view of a host-mapped word; null on other precisions): raised by
// every kernel that writes an activation as f16 hi / lo planes when a value leaves the f16 range,
// reported by mec_model_check
unsigned* range_flag();
struct OptScope {                // set for the duration of one C-ABI call on a handle
  const Options* po;
  TuneCache* pt;
  unsigned* pf;
  OptScope(const Options* o, TuneCache* t, unsigned* flag = nullptr);
  ~OptScope();
};

// fp32x3 range guard. An activation x is carried as hi = f16(x), lo = f16(x - hi): |x| >= 65520
// rounds hi to inf (hi + lo = NaN downstream), and a NaN / inf input is no fp32 value either. Any
// such value raises the handle's flag (a vector store of 1; only on that rare path), so the
// forward fails loudly at mec_model_check instead of returning NaN probabilities.
__device__ __forceinline__ bool x3_out_of_range(float v) { return !(__builtin_fabsf(v) < 65520.f); }
__device__ __forceinline__ bool x3_out_of_range4(float4 v) {
  return x3_out_of_range(v.x) || x3_out_of_range(v.y) || x3_out_of_range(v.z) || x3_out_of_range(v.w);
}
__device__ __forceinline__ void x3_raise(unsigned* flag, bool bad) {
  if (bad && flag) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
int set_option(Options& o, const std::string& key, int value);  // 0 = ok, -1 = unknown key / bad value
constexpr bool kProbes =
#ifdef MEC_PROBES
    true;
#else
    false;
#endif

// hipEvent pairs recorded around every launch whose tag matches `tag`.
struct Prof {
  int tag = TAG_NONE;
  std::vector<hipEvent_t> ev;
  size_t used = 0;
  int begin(int t, hipStream_t s);
  int end(int t, hipStream_t s);
  int read(double* total_ms, int* count);
  void reset() { used = 0; }
  ~Prof();
};

// Device buffer owned by a model handle (grow-only).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t n);
  void release();
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
  ~DevBuf() { release(); }
};

int upload(DevBuf& b, const void* host, size_t bytes);

// Sequential reader over the canonical fp32 host blob (mec/synthetic.py: spec()).
struct BlobReader {
  const float* p;
  size_t n, off = 0;
  bool ok = true;
  BlobReader(const float* p_, size_t n_) : p(p_), n(n_) {}
  const float* take(size_t count) {
    if (off + count > n) { ok = false; return p; }
    const float* r = p + off;
    off += count;
    return r;
  }
};

// fp16 MFMA GEMM / implicit-GEMM convolution ------------------------------------------
// C[M,N] = epilogue( A'[M,K] . B[N,K]^T ), A' = A (plain) or the im2col view of an NHWC
// tensor (conv).
enum AMode : int { A_PLAIN = 0, A_CONV = 1, A_DUAL = 2 };
// ACT_GELU: a (4, 3) rational Phi (f16 path, gemm_common.h gelu_rat); ACT_GELU_EXACT: libm erff,
// x * 0.5 * (1 + erf(x / sqrt2)) as torch's CPU gelu kernel orders it (fp32 path); ACT_GELU_F32:
// the same expression with the library's erf polynomials evaluated branch-free and a one-instruction
// exp (gemm_common.h gelu_f32; fp32x3 path)
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_RELU6 = 3, ACT_GELU_EXACT = 4, ACT_GELU_F32 = 5 };

struct GemmParams {
  const void* A = nullptr;   // f16 [M,K] | f16 NHWC [n,H,W,C]
  const f16* B = nullptr;    // f16 [N,K], K contiguous
  const float* B32 = nullptr;   // f32 [N,K] (fp32 engine, gemm_f32.hip; A is then f32 too)
  const float* bias = nullptr;  // [N]
  const void* R = nullptr;      // residual [M,N] (f16 or f32) or null
  int r_f32 = 0;
  // deferred LayerNorm of an f32 residual: R' = fma((R - mean[row]) * rstd[row], r_g, r_b),
  // the exact expression bert_layernorm_kernel evaluates (so R' is that kernel's output)
  const float2* r_stats = nullptr;  // [M] (mean, rstd) or null
  const float* r_g = nullptr;       // [N]
  const float* r_b = nullptr;       // [N]
  f16* C16 = nullptr;           // [M,N] f16 out or null
  float* C32 = nullptr;         // [M,N] f32 out or null
  int M = 0, N = 0, K = 0;
  int act = ACT_NONE;
  int amode = A_PLAIN;
  const void* A2 = nullptr;  // A_DUAL second source (NHWC, geometry below), K1 = columns of A
  int K1 = 0;
  // conv geometry (NHWC input)
  int H = 1, W = 1, C = 0, OH = 1, OW = 1, ks = 1, stride = 1, pad = 0;
  int group_m = 0;  // ping-pong tile order inside an XCD's range: 0 row-major, G = G-row groups
  // Split-f16 operands (the MEC_PREC_FP32X3 path, f16 engine only): A and B are each an f16
  // hi plane and an f16 lo plane (x = hi + lo exactly, |lo| <= 2^-11 |hi|), the lo planes at
  // element offsets a_lo / b_lo from A / B (A_DUAL: from A and from A2 alike). The K loop makes three passes over K, A_lo.B_hi,
  // A_hi.B_lo, A_hi.B_hi, into one fp32 accumulator (the dropped A_lo.B_lo term is below
  // 2^-22 |A B|). oscale (a power of two: undoes the weights' pre-scale, exact) multiplies the
  // accumulator before the bias; it is 1 (an exact no-op) everywhere else.
  int split = 0;
  long long a_lo = 0, b_lo = 0;
  float oscale = 1.f;
  long long c_lo = 0;  // != 0: C16 is written as a hi plane and a lo plane (C16 + c_lo): f16(v), f16(v - hi)
  // split output's activation-plane scale (a power of two, exact): the planes carry v * cscale, v the
  // value after the activation (C32, when also written, carries v). Chosen per tensor at handle
  // creation so the planes' magnitudes sit where the lo plane is a normal f16 (activation_exp below)
  float cscale = 1.f;
  unsigned* ovf = nullptr;  // split output's range flag (x3_raise); launch_gemm fills in range_flag()
  long long r_lo = 0;  // != 0: the f16 residual R is a hi plane + a lo plane at R + r_lo (R = hi + lo)
  // start stagger (opt().gemm_x3_stagger): blocks [stagger_lo, stagger_hi) -- the second resident workgroup of
  // each CU in dispatch order -- wait `stagger` ticks of the 100-MHz realtime clock before starting, so the
  // two workgroups sharing a CU run half a tile apart and one's epilogue (GELU, plane stores) overlaps the
  // other's MFMAs instead of both bursting together. Speed only: no result depends on it
  int stagger = 0, stagger_lo = 0, stagger_hi = 0;
  int late_dma = 0;  // opt().gemm_x3_late_dma (gemm_glds_kernel, interleaved split tiles)
  int x3_prio = 0;   // opt().gemm_x3_prio (the same kernels)
};

int launch_gemm(const GemmParams& p, hipStream_t s, Prof* prof, int tag);
int launch_gemm_glds(const GemmParams& p, hipStream_t s, int force_bn);
// 3x3/1 conv 64 -> 64 on 56x56 (+ BN shift + ReLU) as a halo-tile kernel (conv3x3.hip);
// launch_gemm routes matching A_CONV shapes to it while opt().conv3x3_direct is set
int launch_conv3x3_c64(const f16* x, const f16* w, const float* bias, f16* y, int B, int H, int C, int Cout,
                       hipStream_t s);
// 3x3/1 convs C -> C on 28x28x128 and 14x14x256 (+ BN shift + ReLU): halo kernel
// (conv3x3_halo.hip), routed from launch_gemm while opt().conv3x3_halo is set. Same fp32
// accumulation as the GEMM path in another summation order (not bit-identical to it).
bool conv3x3_halo_supported(int H, int C, int N);
int launch_conv3x3_halo(const f16* x, const f16* w, const float* bias, f16* y, int B, int H, int C, hipStream_t s);
int gemm_tuned_bn(int amode, int M, int N, int K);
// fp32 engine (gemm_f32.hip): f32 A (plain or NHWC conv) and B32, v_mfma_f32_32x32x2_f32
int launch_gemm_f32(const GemmParams& p, hipStream_t s, Prof* prof, int tag);
int gemm_f32_tuned(int amode, int M, int N, int K);

}  // namespace mec
