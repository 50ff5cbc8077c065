// Speech DNN and fusion step: one fused launch each, R samples per workgroup, all
// activations in LDS, fp32 arithmetic (the reference computes both in fp32).
//
// speech_kernel   restates inference/speech_inference.py:66-69, :93-103 over the Keras
//                 Sequential of model_training/train_speech_model.py:55-90:
//                 StandardScaler -> 5 x [Dense, BN(eps 1e-3), ReLU] -> Dense7 -> softmax,
//                 emitting the block-5 ReLU (layers[-3]) 64-d feature too.
// fusion_kernel   restates MultiModalFusionModel.forward (inference/multimodal_fusion.py:
//                 156-180) + the softmax of fuse_with_attention (:221).
// fuse_weighted   restates fuse_predictions (:184-199) in float64 like numpy.
#include "block_ops.h"
#include "models.h"

namespace mec {

// =============================================================== speech
struct SpeechW {
  const float *mean, *scale;
  const float* W[6];
  const float* b[6];
  const float* inv[5];
  const float* shift[5];
};

constexpr int SF_THREADS = 512;  // fusion kernels

// ---- speech_flow_kernel: the network with every layer split by output columns over
// workgroups, so each weight byte is read by one workgroup per 16-sample chunk instead of
// by every workgroup (a one-workgroup-per-4-samples form streamed all 1.85 MB of weights
// through each CU, which bounded it at ~40 us for any batch). Per chunk of 16 samples, five
// stages:
//   stage 0  L0  56->512   8 WGs x 64 columns (4 waves = 4 column tiles, K 56 padded to 64)
//   stage 1  L1 512->512  32 WGs x 16 columns (4 waves = 4 K quarters, summed in LDS)
//   stage 2  L2 512->256  16 WGs x 16 columns
//   stage 3  L3 256->128   8 WGs x 16 columns
//   stage 4  L4 128->64 + Dense7 + softmax, 1 WG (writes feat / logits / probs)
// on v_mfma_f32_16x16x4f32 (exact f32 products, fp32 accumulate). A stage's workgroup loads
// its weight fragments into registers, then reads its inputs from the previous stage.
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 hand-off
// table): the producer stores its activations write-through (sc1), every storing wave drains
// them (vmcnt(0)), a workgroup barrier, then one agent-scope atomic add on the chunk's
// per-stage counter; the consumer polls that counter with one lane (sc1 dword loads + s_sleep)
// and every wave reads its inputs with sc1 loads. Blocks are numbered stage-major, so every
// producer precedes its consumers in dispatch order; every spin is bounded (an expired wait
// sets the launch's error word and the stage proceeds; the chunk's probs then come out NaN,
// and the last stage raises the handle's host-visible error flag, which mec_model_check
// reports). The counters and the error word are zeroed by a memset on the stream before
// every launch, so an expired wait (whose late producer may still arrive after the chunk's
// last stage) never leaks a count or an error into the next launch. Measured hop on MI355X, B = 32:
// ~1.9 us from the last arrival to the wait's exit, ~1.2 us for the sc1 input loads.
// (Tagged 8-B granules polled directly, with or without the counter, measured no faster at
// B = 32 and up to 2x slower at B = 256, where 1,040 polling blocks flood the memory system.)
constexpr int SPF_SB = 16;    // samples per chunk
constexpr int SPF_LINE = 32;  // u32 words between counters (one 128-B line each)
constexpr int SPF_WG_PER_CHUNK = 8 + 32 + 16 + 8 + 1;
constexpr int SPF_SPIN_LIMIT = 1 << 22;
__host__ __device__ constexpr int spf_groups(int st) {
  return st == 0 ? 8 : st == 1 ? 32 : st == 2 ? 16 : st == 3 ? 8 : 1;
}

struct SpeechFlow {
  float* act[4];               // stage outputs, f32 [16 * chunks, N_l]
  unsigned* cnt;               // [chunks][4] arrival counters, SPF_LINE apart
  unsigned* err;               // this launch: a wait expired
  unsigned* host_err;          // host-mapped pinned flag of the handle (mec_model_check)
  int chunks;
  int spin_limit;              // SPF_SPIN_LIMIT (probe builds: option speech_spin_limit)
};

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 ld_sc1x4(const float* p) {
  f32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void st_sc1x4(float* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

struct SpfShared {
  float red[4][256];          // per-wave 16x16 partial sums (K-split stages)
  float hs[SPF_SB][64 + 1];   // stage 4: block-5 ReLU output
  float lg[SPF_SB][8];        // stage 4: logits
  float w5[64 * 7 + 8];       // stage 4: Dense(7) kernel + bias, loaded at entry
};

// DBG (probe build, option speech_debug; wrong results): lane 0 of every block writes six
// s_memrealtime stamps (100 MHz) into feat as u64 [block][6] (entry, weights issued, wait
// over, inputs landed, outputs drained, arrival) and stage 4 skips its outputs.
template <int ST, int DBG>
__device__ __forceinline__ void spf_stage(const SpeechW& w, const SpeechFlow& f, const float* __restrict__ x, int B,
                                          int chunk, int g, float* feat, float* logits, float* probs,
                                          SpfShared& sh) {
  auto stamp = [&](int i) {
    if constexpr (DBG) {
      if (threadIdx.x == 0)
        reinterpret_cast<unsigned long long*>(feat)[blockIdx.x * 6 + i] = __builtin_amdgcn_s_memrealtime();
    }
  };
  stamp(0);
  constexpr int K = ST == 0 ? 56 : ST == 1 ? 512 : ST == 2 ? 512 : ST == 3 ? 256 : 128;
  constexpr int N = ST == 0 ? 512 : ST == 1 ? 512 : ST == 2 ? 256 : ST == 3 ? 128 : 64;
  constexpr int CT = (ST == 0 || ST == 4) ? 4 : 1;  // column tiles per WG (one per wave)
  constexpr int KS = 4 / CT;                          // K split over waves
  constexpr int KP = ST == 0 ? 64 : K;
  constexpr int T = KP / (16 * KS);                   // 16-deep k groups per wave
  static_assert(N % (16 * CT) == 0 && N / (16 * CT) == spf_groups(ST), "stage geometry");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int ct = wave % CT, ks = wave / CT;
  const int n0 = g * 16 * CT;
  const int n = n0 + ct * 16 + c16;
  const int kb = ks * (KP / KS);
  const int row0 = chunk * SPF_SB;
  const int r = row0 + c16;

  // B fragments (lane: k = kb + 16t + 4q + j, column n) and the epilogue constants: independent
  // of the previous stage, so they load while it runs
  const float* W = w.W[ST];
  float bw[T][4];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kb + 16 * t + 4 * q + j;
      bw[t][j] = (KP == K || k < K) ? W[(size_t)k * N + n] : 0.f;
    }
  const int fin_c = n0 + (tid & 3) * 4;  // K-split finisher: 4 columns
  float ep_b[4], ep_i[4], ep_s[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nn = KS == 1 ? n : fin_c + i;
    ep_b[i] = w.b[ST][nn];
    ep_i[i] = w.inv[ST][nn];
    ep_s[i] = w.shift[ST][nn];
  }
  if constexpr (ST == 4)
    for (int i = tid; i < 64 * 7 + 7; i += blockDim.x) sh.w5[i] = i < 64 * 7 ? w.W[5][i] : w.b[5][i - 64 * 7];
  stamp(1);
  if constexpr (ST > 0) {
    if (tid == 0) {
      const unsigned* c = f.cnt + (size_t)(chunk * 4 + ST - 1) * SPF_LINE;
      for (int spins = 0; __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < spf_groups(ST - 1);) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > f.spin_limit) {
          __hip_atomic_fetch_or(f.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
  }
  stamp(2);

  // A fragments (lane: row c16 of the chunk, k = kb + 16t + 4q + j)
  f32x4 a[T];
  if constexpr (ST == 0) {
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = kb + 16 * t + 4 * q + j;
        // sklearn StandardScaler.transform: (X - mean_) / scale_
        a[t][j] = (r < B && k < K) ? (x[(size_t)r * K + k] - w.mean[k]) / w.scale[k] : 0.f;
      }
  } else {
    const float* in = f.act[ST - 1] + (size_t)r * K + kb + 4 * q;
#pragma unroll
    for (int t = 0; t < T; ++t) a[t] = ld_sc1x4(in + 16 * t);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < T; ++t) asm volatile("" : "+v"(a[t]));  // uses stay behind the wait
  }
  stamp(3);

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][j], bw[t][j], acc, 0, 0, 0);

  // Dense bias, then tf.nn.batch_normalization x * inv + (beta - mean * inv), then ReLU.
  // D layout: lane holds rows 4q + e of column c16.
  if constexpr (KS == 1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 4 * q + e;
      const float v = fmaxf((acc[e] + ep_b[0]) * ep_i[0] + ep_s[0], 0.f);
      if constexpr (ST < 4)
        st_sc1(f.act[ST] + (size_t)(row0 + row) * N + n, v);
      else
        sh.hs[row][n] = v;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) sh.red[wave][(4 * q + e) * 16 + c16] = acc[e];
    __syncthreads();
    if (tid < 64) {
      const int row = tid >> 2, c4 = (tid & 3) * 4;
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = row * 16 + c4 + i;
        const float s = ((sh.red[0][o] + sh.red[1][o]) + sh.red[2][o]) + sh.red[3][o];
        v[i] = fmaxf((s + ep_b[i]) * ep_i[i] + ep_s[i], 0.f);
      }
      st_sc1x4(f.act[ST] + (size_t)(row0 + row) * N + n0 + c4, v);
    }
  }

  if constexpr (ST < 4) {  // publish: every storing wave drained, a barrier, one arrival
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(4);
    if (tid == 0)
      __hip_atomic_fetch_add(f.cnt + (size_t)(chunk * 4 + ST) * SPF_LINE, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __syncthreads();
    stamp(4);
    if constexpr (DBG) {
      stamp(5);
      return;
    }
    const int nr = min(SPF_SB, B - row0);
    for (int i = tid; i < nr * 64; i += blockDim.x) feat[(size_t)row0 * 64 + i] = sh.hs[i >> 6][i & 63];
    if (tid < SPF_SB * 7) {  // Dense(7): feat @ W + b
      const int row = tid / 7, o = tid - row * 7;
      float s = 0.f;
#pragma unroll 16
      for (int k = 0; k < 64; ++k) s = fmaf(sh.hs[row][k], sh.w5[k * 7 + o], s);
      sh.lg[row][o] = s + sh.w5[64 * 7 + o];
    }
    __syncthreads();
    const bool bad = __hip_atomic_load(f.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (bad && tid == 0) __hip_atomic_store(f.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid < nr) {
      const float* z = sh.lg[tid];
      float m = z[0];
      for (int o = 1; o < 7; ++o) m = fmaxf(m, z[o]);
      float e[7], s = 0.f;
      for (int o = 0; o < 7; ++o) { e[o] = expf(z[o] - m); s += e[o]; }
      const size_t ro = (size_t)(row0 + tid) * 7;
      for (int o = 0; o < 7; ++o) {
        logits[ro + o] = z[o];
        probs[ro + o] = bad ? __builtin_nanf("") : e[o] / s;
      }
    }
  }
  stamp(5);
}

template <int DBG>
__global__ __launch_bounds__(256) void speech_flow_kernel(SpeechW w, SpeechFlow f, const float* __restrict__ x, int B,
                                                          float* feat, float* logits, float* probs) {
  __shared__ SpfShared sh;
  const int nc = f.chunks;
  int b = blockIdx.x;
  if (b < 8 * nc) return spf_stage<0, DBG>(w, f, x, B, b / 8, b % 8, feat, logits, probs, sh);
  b -= 8 * nc;
  if (b < 32 * nc) return spf_stage<1, DBG>(w, f, x, B, b / 32, b % 32, feat, logits, probs, sh);
  b -= 32 * nc;
  if (b < 16 * nc) return spf_stage<2, DBG>(w, f, x, B, b / 16, b % 16, feat, logits, probs, sh);
  b -= 16 * nc;
  if (b < 8 * nc) return spf_stage<3, DBG>(w, f, x, B, b / 8, b % 8, feat, logits, probs, sh);
  b -= 8 * nc;
  spf_stage<4, DBG>(w, f, x, B, b, 0, feat, logits, probs, sh);
}

int SpeechModel::create(const float* blob, size_t n) {
  BlobReader rd(blob, n);
  const int dims[6] = {56, 512, 512, 256, 128, 64};
  std::vector<float> h;
  auto put = [&](const float* src, size_t cnt) {
    size_t o = h.size();
    h.insert(h.end(), src, src + cnt);
    return o;
  };
  off_mean = put(rd.take(56), 56);
  off_scale = put(rd.take(56), 56);
  for (int l = 0; l < 5; ++l) {
    const int K = dims[l], N = dims[l + 1];
    off_W[l] = put(rd.take((size_t)K * N), (size_t)K * N);  // Keras kernel is [in,out] already
    off_b[l] = put(rd.take(N), N);
    const float* g = rd.take(N);
    const float* be = rd.take(N);
    const float* mm = rd.take(N);
    const float* mv = rd.take(N);
    std::vector<float> inv(N), sh(N);
    for (int i = 0; i < N; ++i) {
      inv[i] = (1.0f / sqrtf(mv[i] + 1e-3f)) * g[i];
      sh[i] = be[i] - mm[i] * inv[i];
    }
    off_inv[l] = put(inv.data(), N);
    off_shift[l] = put(sh.data(), N);
  }
  off_W[5] = put(rd.take(64 * 7), 64 * 7);
  off_b[5] = put(rd.take(7), 7);
  MEC_REQUIRE(rd.ok && rd.off == n, "speech blob size mismatch");
  return upload(w, h.data(), h.size() * sizeof(float));
}

SpeechModel::~SpeechModel() {
  if (host_err) (void)hipHostFree(host_err);
}

int SpeechModel::check() {
  if (!host_err || !*reinterpret_cast<volatile unsigned*>(host_err)) return 0;
  *host_err = 0;
  set_error("speech: a stage hand-off wait expired (spin limit) in a forward since the last check; "
            "that forward's probs are NaN");
  return -1;
}

int SpeechModel::forward(const float* x, int B, float* feat, float* logits, float* probs, hipStream_t s) {
  MEC_REQUIRE(B >= 0, "speech: B < 0");
  if (B == 0) return 0;
  MEC_REQUIRE(x && feat && logits && probs, "speech: null pointer");
  const float* base = w.as<float>();
  SpeechW p;
  p.mean = base + off_mean;
  p.scale = base + off_scale;
  for (int l = 0; l < 6; ++l) { p.W[l] = base + off_W[l]; p.b[l] = base + off_b[l]; }
  for (int l = 0; l < 5; ++l) { p.inv[l] = base + off_inv[l]; p.shift[l] = base + off_shift[l]; }
  const int nch = (B + SPF_SB - 1) / SPF_SB;
  MEC_REQUIRE(nch <= (1 << 24) / SPF_WG_PER_CHUNK, "speech: batch too large");
  if (nch > flow_chunks) {
    MEC_TRY(flow_act.ensure((size_t)nch * SPF_SB * (512 + 512 + 256 + 128) * sizeof(float)));
    MEC_TRY(flow_sync.ensure(((size_t)nch * 4 + 1) * SPF_LINE * sizeof(unsigned)));
    flow_chunks = nch;
  }
  if (!host_err) {
    MEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&host_err), sizeof(unsigned), hipHostMallocMapped));
    *host_err = 0;
  }
  // every launch starts from zeroed counters and error word (one memset on the stream)
  MEC_HIP(hipMemsetAsync(flow_sync.p, 0, ((size_t)flow_chunks * 4 + 1) * SPF_LINE * sizeof(unsigned), s));
  SpeechFlow fl;
  float* a = flow_act.as<float>();
  const size_t rows = (size_t)flow_chunks * SPF_SB;
  fl.act[0] = a;
  fl.act[1] = a + rows * 512;
  fl.act[2] = a + rows * 1024;
  fl.act[3] = a + rows * 1280;
  fl.cnt = flow_sync.as<unsigned>();
  fl.err = fl.cnt + (size_t)flow_chunks * 4 * SPF_LINE;
  MEC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&fl.host_err), host_err, 0));
  fl.chunks = nch;
  fl.spin_limit = SPF_SPIN_LIMIT;
#ifdef MEC_PROBES
  if (opt().speech_spin_limit >= 0) fl.spin_limit = opt().speech_spin_limit;  // probe: force expiries
#endif
  MEC_TRY(prof.begin(TAG_SPEECH, s));
#ifdef MEC_PROBES
  if (opt().speech_debug) {
    MEC_REQUIRE((size_t)B * 64 >= (size_t)nch * SPF_WG_PER_CHUNK * 12, "speech_debug: feat too small for the trace");
    hipLaunchKernelGGL(speech_flow_kernel<1>, dim3(nch * SPF_WG_PER_CHUNK), dim3(256), 0, s, p, fl, x, B, feat, logits,
                       probs);
  } else
#endif
  hipLaunchKernelGGL(speech_flow_kernel<0>, dim3(nch * SPF_WG_PER_CHUNK), dim3(256), 0, s, p, fl, x, B, feat, logits,
                     probs);
  MEC_LAUNCH_CHECK();
  MEC_TRY(prof.end(TAG_SPEECH, s));
  return 0;
}

// =============================================================== fusion
// Pointer table layout (see FusionModel::create):
//   [4m + {0 W,1 b,2 ln_g,3 ln_b}]        modality projections, m = speech/text/image
//   [12 + 10m + {WqT,bq,WkT,bk,WvT,bv,WoT,bo,ln_g,ln_b}]   cross_attn_{m}
//   [42 + 4j + {W,b,ln_g,ln_b}]          attention_fusion.projections.j
//   54..69 att0 W,b | att2 W,b | dec0 W,b | dec2 W,b | cls0 W,b | cls1 g,b | cls4 W,b | cls7 W,b
constexpr int FUSION_NP = 70;
struct FusionW { const float* p[FUSION_NP]; };

// samples per workgroup (mec_set_option "fusion_r": 1, 2, 4). B = 256 on MI355X: split form
// 145 / 139 / 118 us at R = 1 / 2 / 4, the single kernel 174 us at R = 2.
constexpr int F_LDIN = 1368, F_LDP = 768, F_LDT = 1280;

template <int FUSION_R>
__device__ void cross_attention_rows(float* T, int ldt, int nr) {
  // T[r][0:256]=q, [256]=k0, [512]=k1, [768]=v0, [1024]=v1; writes o into T[r][0:256].
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = wave; r < FUSION_R; r += (blockDim.x >> 6)) {
    float* t = T + r * ldt;
    float q[4], s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) q[c] = t[4 * lane + c] * 0.125f;  // q * sqrt(1/head_dim)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      s0 = fmaf(q[c], t[256 + 4 * lane + c], s0);
      s1 = fmaf(q[c], t[512 + 4 * lane + c], s1);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {  // reduce within the 16 lanes of one head
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
    }
    const float m = fmaxf(s0, s1);
    const float e0 = expf(s0 - m), e1 = expf(s1 - m);
    const float den = e0 + e1;
    const float a0 = e0 / den, a1 = e1 / den;
#pragma unroll
    for (int c = 0; c < 4; ++c) t[4 * lane + c] = a0 * t[768 + 4 * lane + c] + a1 * t[1024 + 4 * lane + c];
  }
  __syncthreads();
}

template <int FUSION_R>
__global__ __launch_bounds__(512) void fusion_kernel(FusionW w, const float* __restrict__ sf,
                                                     const float* __restrict__ tf, const float* __restrict__ imf,
                                                     const float* __restrict__ sp, const float* __restrict__ tp,
                                                     const float* __restrict__ ip, int B, float* logits,
                                                     float* probs, float* attn_w, float* dec_w) {
  constexpr int R = FUSION_R;
  __shared__ __attribute__((aligned(16))) float IN[R * F_LDIN], P[R * F_LDP], E[R * F_LDP], T[R * F_LDT], red[4 * R * SF_THREADS];
  const int tid = threadIdx.x, T_ = blockDim.x;
  const int r0 = blockIdx.x * R;
  const int nr = min(R, B - r0);
  for (int idx = tid; idx < R * F_LDIN; idx += T_) {
    const int r = idx / F_LDIN, k = idx - r * F_LDIN;
    const size_t b = (size_t)(r0 + r);
    float v = 0.f;
    if (r < nr) {
      if (k < 64) v = sf[b * 64 + k];
      else if (k < 832) v = tf[b * 768 + (k - 64)];
      else if (k < 1344) v = imf[b * 512 + (k - 832)];
      else if (k < 1351) v = sp[b * 7 + (k - 1344)];
      else if (k < 1358) v = tp[b * 7 + (k - 1351)];
      else if (k < 1365) v = ip[b * 7 + (k - 1358)];
    }
    IN[idx] = v;
  }
  __syncthreads();
  const int in_off[3] = {0, 64, 832}, in_dim[3] = {64, 768, 512};
  // modality projections: ReLU(LN(Linear)) (multimodal_fusion.py:113-130, :157-159)
  for (int m = 0; m < 3; ++m) {
    block_linear<R>(IN + in_off[m], F_LDIN, in_dim[m], w.p[4 * m], 256, w.p[4 * m + 1], 256, P + 256 * m, F_LDP, red, BACT_NONE);
    block_layernorm<R>(P + 256 * m, F_LDP, 256, w.p[4 * m + 2], w.p[4 * m + 3], 1e-5f, true);
  }
  // cross-modal attention (:161-167): query m attends to the other two (in order)
  const int others[3][2] = {{1, 2}, {0, 2}, {0, 1}};
  for (int m = 0; m < 3; ++m) {
    const float* const* c = w.p + 12 + 10 * m;
    block_linear<R>(P + 256 * m, F_LDP, 256, c[0], 256, c[1], 256, T + 0, F_LDT, red, BACT_NONE);
    block_linear<R>(P + 256 * others[m][0], F_LDP, 256, c[2], 256, c[3], 256, T + 256, F_LDT, red, BACT_NONE);
    block_linear<R>(P + 256 * others[m][1], F_LDP, 256, c[2], 256, c[3], 256, T + 512, F_LDT, red, BACT_NONE);
    block_linear<R>(P + 256 * others[m][0], F_LDP, 256, c[4], 256, c[5], 256, T + 768, F_LDT, red, BACT_NONE);
    block_linear<R>(P + 256 * others[m][1], F_LDP, 256, c[4], 256, c[5], 256, T + 1024, F_LDT, red, BACT_NONE);
    cross_attention_rows<FUSION_R>(T, F_LDT, nr);
    block_linear<R>(T, F_LDT, 256, c[6], 256, c[7], 256, E + 256 * m, F_LDP, red, BACT_NONE);
    for (int idx = tid; idx < R * 256; idx += T_) {
      const int r = idx >> 8, n = idx & 255;
      E[r * F_LDP + 256 * m + n] = P[r * F_LDP + 256 * m + n] + E[r * F_LDP + 256 * m + n];
    }
    __syncthreads();
    block_layernorm<R>(E + 256 * m, F_LDP, 256, c[8], c[9], 1e-5f, false);
  }
  // AttentionFusion (:79-106): per-modality projection, attention over the 768 concat
  for (int j = 0; j < 3; ++j) {
    block_linear<R>(E + 256 * j, F_LDP, 256, w.p[42 + 4 * j], 256, w.p[43 + 4 * j], 256, T + 256 * j, F_LDT, red, BACT_NONE);
    block_layernorm<R>(T + 256 * j, F_LDT, 256, w.p[44 + 4 * j], w.p[45 + 4 * j], 1e-5f, true);
  }
  block_linear<R>(T, F_LDT, 768, w.p[54], 256, w.p[55], 256, T + 768, F_LDT, red, BACT_TANH);
  block_linear<R>(T + 768, F_LDT, 256, w.p[56], 3, w.p[57], 3, P, F_LDP, red, BACT_NONE);
  block_softmax_small<R>(P, F_LDP, 3, nullptr, 0);
  for (int idx = tid; idx < R * 256; idx += T_) {  // fused = sum_j w_j * proj_j
    const int r = idx >> 8, n = idx & 255;
    const float* a = P + r * F_LDP;
    const float* t = T + r * F_LDT;
    E[r * F_LDP + n] = a[0] * t[n] + a[1] * t[256 + n] + a[2] * t[512 + n];
  }
  for (int idx = tid; idx < nr * 3; idx += T_) {
    const int r = idx / 3, j = idx - r * 3;
    attn_w[(size_t)(r0 + r) * 3 + j] = P[r * F_LDP + j];
  }
  __syncthreads();
  // decision weights over the 21-d concat of softmax outputs (:138-143, :171-175)
  block_linear<R>(IN + 1344, F_LDIN, 21, w.p[58], 64, w.p[59], 64, P + 256, F_LDP, red, BACT_RELU);
  block_linear<R>(P + 256, F_LDP, 64, w.p[60], 3, w.p[61], 3, P + 384, F_LDP, red, BACT_NONE);
  block_softmax_small<R>(P + 384, F_LDP, 3, nullptr, 0);
  for (int idx = tid; idx < R * 7; idx += T_) {
    const int r = idx / 7, c = idx - r * 7;
    const float* d = P + r * F_LDP + 384;
    const float* pr = IN + r * F_LDIN + 1344;
    E[r * F_LDP + 256 + c] = pr[c] * d[0] + pr[7 + c] * d[1] + pr[14 + c] * d[2];
  }
  for (int idx = tid; idx < nr * 3; idx += T_) {
    const int r = idx / 3, j = idx - r * 3;
    dec_w[(size_t)(r0 + r) * 3 + j] = P[r * F_LDP + 384 + j];
  }
  __syncthreads();
  // classifier on [fused, weighted_preds] (:145-154, :177-178)
  block_linear<R>(E, F_LDP, 263, w.p[62], 256, w.p[63], 256, T, F_LDT, red, BACT_NONE);
  block_layernorm<R>(T, F_LDT, 256, w.p[64], w.p[65], 1e-5f, true);
  block_linear<R>(T, F_LDT, 256, w.p[66], 128, w.p[67], 128, T + 256, F_LDT, red, BACT_RELU);
  block_linear<R>(T + 256, F_LDT, 128, w.p[68], 7, w.p[69], 7, T + 384, F_LDT, red, BACT_NONE);
  for (int idx = tid; idx < nr * 7; idx += T_) {
    const int r = idx / 7, c = idx - r * 7;
    logits[(size_t)(r0 + r) * 7 + c] = T[r * F_LDT + 384 + c];
  }
  __syncthreads();
  block_softmax_small<R>(T + 384, F_LDT, 7, nullptr, 0);
  for (int idx = tid; idx < nr * 7; idx += T_) {
    const int r = idx / 7, c = idx - r * 7;
    probs[(size_t)(r0 + r) * 7 + c] = T[r * F_LDT + 384 + c];
  }
}

// ---- split form: the same block_linear / block_layernorm calls as fusion_kernel (so the
// same bits), over three launches. The three modality chains of the projection and
// cross-attention stages are independent, so stages 1-2 run one block per (sample group,
// modality): 3x the blocks and a third of the serial layer chain per block.
//   fusion_proj_kernel   grid (groups, 3): P_m = ReLU(LN(Linear_m(x_m)))           -> Pg
//   fusion_cross_kernel  grid (groups, 3): E_m = LN(P_m + CrossAttn_m(P_m; P_o1, P_o2)),
//                                          T_m = ReLU(LN(Proj_m(E_m)))             -> Tg
//   fusion_head_kernel   grid (groups):    attention over T, decision weights, classifier

template <int R>
__global__ __launch_bounds__(512) void fusion_proj_kernel(FusionW w, const float* __restrict__ sf,
                                                          const float* __restrict__ tf, const float* __restrict__ imf,
                                                          int B, float* __restrict__ Pg) {
  __shared__ __attribute__((aligned(16))) float IN[R * 768], P[R * 256], red[4 * R * SF_THREADS];
  const int tid = threadIdx.x, m = blockIdx.y;
  const int r0 = blockIdx.x * R, nr = min(R, B - r0);
  const int dim = m == 0 ? 64 : (m == 1 ? 768 : 512);
  const float* src = m == 0 ? sf : (m == 1 ? tf : imf);
  for (int idx = tid; idx < R * dim; idx += blockDim.x) {
    const int r = idx / dim, k = idx - r * dim;
    IN[r * 768 + k] = r < nr ? src[(size_t)(r0 + r) * dim + k] : 0.f;
  }
  __syncthreads();
  block_linear<R>(IN, 768, dim, w.p[4 * m], 256, w.p[4 * m + 1], 256, P, 256, red, BACT_NONE);
  block_layernorm<R>(P, 256, 256, w.p[4 * m + 2], w.p[4 * m + 3], 1e-5f, true);
  for (int idx = tid; idx < nr * 256; idx += blockDim.x) {
    const int r = idx >> 8, n = idx & 255;
    Pg[(size_t)(r0 + r) * 768 + 256 * m + n] = P[r * 256 + n];
  }
}

template <int R>
__global__ __launch_bounds__(512) void fusion_cross_kernel(FusionW w, const float* __restrict__ Pg, int B,
                                                           float* __restrict__ Tg) {
  __shared__ __attribute__((aligned(16))) float P[R * F_LDP], E[R * 256], T[R * F_LDT], red[4 * R * SF_THREADS];
  const int tid = threadIdx.x, m = blockIdx.y;
  const int r0 = blockIdx.x * R, nr = min(R, B - r0);
  for (int idx = tid; idx < R * 768; idx += blockDim.x) {
    const int r = idx / 768, k = idx - r * 768;
    P[r * F_LDP + k] = r < nr ? Pg[(size_t)(r0 + r) * 768 + k] : 0.f;
  }
  __syncthreads();
  const int o0 = m == 0 ? 1 : 0, o1 = m == 2 ? 1 : 2;  // the other two modalities, in order
  const float* const* c = w.p + 12 + 10 * m;
  block_linear<R>(P + 256 * m, F_LDP, 256, c[0], 256, c[1], 256, T + 0, F_LDT, red, BACT_NONE);
  block_linear<R>(P + 256 * o0, F_LDP, 256, c[2], 256, c[3], 256, T + 256, F_LDT, red, BACT_NONE);
  block_linear<R>(P + 256 * o1, F_LDP, 256, c[2], 256, c[3], 256, T + 512, F_LDT, red, BACT_NONE);
  block_linear<R>(P + 256 * o0, F_LDP, 256, c[4], 256, c[5], 256, T + 768, F_LDT, red, BACT_NONE);
  block_linear<R>(P + 256 * o1, F_LDP, 256, c[4], 256, c[5], 256, T + 1024, F_LDT, red, BACT_NONE);
  cross_attention_rows<R>(T, F_LDT, nr);
  block_linear<R>(T, F_LDT, 256, c[6], 256, c[7], 256, E, 256, red, BACT_NONE);
  for (int idx = tid; idx < R * 256; idx += blockDim.x) {
    const int r = idx >> 8, n = idx & 255;
    E[r * 256 + n] = P[r * F_LDP + 256 * m + n] + E[r * 256 + n];
  }
  __syncthreads();
  block_layernorm<R>(E, 256, 256, c[8], c[9], 1e-5f, false);
  block_linear<R>(E, 256, 256, w.p[42 + 4 * m], 256, w.p[43 + 4 * m], 256, T, F_LDT, red, BACT_NONE);
  block_layernorm<R>(T, F_LDT, 256, w.p[44 + 4 * m], w.p[45 + 4 * m], 1e-5f, true);
  for (int idx = tid; idx < nr * 256; idx += blockDim.x) {
    const int r = idx >> 8, n = idx & 255;
    Tg[(size_t)(r0 + r) * 768 + 256 * m + n] = T[r * F_LDT + n];
  }
}

template <int R>
__global__ __launch_bounds__(512) void fusion_head_kernel(FusionW w, const float* __restrict__ Tg,
                                                          const float* __restrict__ sp, const float* __restrict__ tp,
                                                          const float* __restrict__ ip, int B, float* logits,
                                                          float* probs, float* attn_w, float* dec_w) {
  constexpr int LDPR = 24;
  __shared__ __attribute__((aligned(16))) float PR[R * LDPR], P[R * F_LDP], E[R * F_LDP], T[R * F_LDT], red[4 * R * SF_THREADS];
  const int tid = threadIdx.x, T_ = blockDim.x;
  const int r0 = blockIdx.x * R;
  const int nr = min(R, B - r0);
  for (int idx = tid; idx < R * 768; idx += T_) {
    const int r = idx / 768, k = idx - r * 768;
    T[r * F_LDT + k] = r < nr ? Tg[(size_t)(r0 + r) * 768 + k] : 0.f;
  }
  for (int idx = tid; idx < R * LDPR; idx += T_) {
    const int r = idx / LDPR, k = idx - r * LDPR;
    const size_t b = (size_t)(r0 + r);
    float v = 0.f;
    if (r < nr) {
      if (k < 7) v = sp[b * 7 + k];
      else if (k < 14) v = tp[b * 7 + (k - 7)];
      else if (k < 21) v = ip[b * 7 + (k - 14)];
    }
    PR[idx] = v;
  }
  __syncthreads();
  block_linear<R>(T, F_LDT, 768, w.p[54], 256, w.p[55], 256, T + 768, F_LDT, red, BACT_TANH);
  block_linear<R>(T + 768, F_LDT, 256, w.p[56], 3, w.p[57], 3, P, F_LDP, red, BACT_NONE);
  block_softmax_small<R>(P, F_LDP, 3, nullptr, 0);
  for (int idx = tid; idx < R * 256; idx += T_) {  // fused = sum_j w_j * proj_j
    const int r = idx >> 8, n = idx & 255;
    const float* a = P + r * F_LDP;
    const float* t = T + r * F_LDT;
    E[r * F_LDP + n] = a[0] * t[n] + a[1] * t[256 + n] + a[2] * t[512 + n];
  }
  for (int idx = tid; idx < nr * 3; idx += T_) {
    const int r = idx / 3, j = idx - r * 3;
    attn_w[(size_t)(r0 + r) * 3 + j] = P[r * F_LDP + j];
  }
  __syncthreads();
  block_linear<R>(PR, LDPR, 21, w.p[58], 64, w.p[59], 64, P + 256, F_LDP, red, BACT_RELU);
  block_linear<R>(P + 256, F_LDP, 64, w.p[60], 3, w.p[61], 3, P + 384, F_LDP, red, BACT_NONE);
  block_softmax_small<R>(P + 384, F_LDP, 3, nullptr, 0);
  for (int idx = tid; idx < R * 7; idx += T_) {
    const int r = idx / 7, c = idx - r * 7;
    const float* d = P + r * F_LDP + 384;
    const float* pr = PR + r * LDPR;
    E[r * F_LDP + 256 + c] = pr[c] * d[0] + pr[7 + c] * d[1] + pr[14 + c] * d[2];
  }
  for (int idx = tid; idx < nr * 3; idx += T_) {
    const int r = idx / 3, j = idx - r * 3;
    dec_w[(size_t)(r0 + r) * 3 + j] = P[r * F_LDP + 384 + j];
  }
  __syncthreads();
  block_linear<R>(E, F_LDP, 263, w.p[62], 256, w.p[63], 256, T, F_LDT, red, BACT_NONE);
  block_layernorm<R>(T, F_LDT, 256, w.p[64], w.p[65], 1e-5f, true);
  block_linear<R>(T, F_LDT, 256, w.p[66], 128, w.p[67], 128, T + 256, F_LDT, red, BACT_RELU);
  block_linear<R>(T + 256, F_LDT, 128, w.p[68], 7, w.p[69], 7, T + 384, F_LDT, red, BACT_NONE);
  for (int idx = tid; idx < nr * 7; idx += T_) {
    const int r = idx / 7, c = idx - r * 7;
    logits[(size_t)(r0 + r) * 7 + c] = T[r * F_LDT + 384 + c];
  }
  __syncthreads();
  block_softmax_small<R>(T + 384, F_LDT, 7, nullptr, 0);
  for (int idx = tid; idx < nr * 7; idx += T_) {
    const int r = idx / 7, c = idx - r * 7;
    probs[(size_t)(r0 + r) * 7 + c] = T[r * F_LDT + 384 + c];
  }
}

template <int R>
static void launch_fusion_split(const FusionW& p, const float* sf, const float* tf, const float* imf, const float* sp,
                                const float* tp, const float* ip, int B, float* Pg, float* Tg, float* logits,
                                float* probs, float* attn_w, float* dec_w, hipStream_t s) {
  const int groups = (B + R - 1) / R;
  hipLaunchKernelGGL((fusion_proj_kernel<R>), dim3(groups, 3), dim3(SF_THREADS), 0, s, p, sf, tf, imf, B, Pg);
  hipLaunchKernelGGL((fusion_cross_kernel<R>), dim3(groups, 3), dim3(SF_THREADS), 0, s, p, Pg, B, Tg);
  hipLaunchKernelGGL((fusion_head_kernel<R>), dim3(groups), dim3(SF_THREADS), 0, s, p, Tg, sp, tp, ip, B, logits, probs,
                     attn_w, dec_w);
}

int FusionModel::create(const float* blob, size_t n) {
  BlobReader rd(blob, n);
  std::vector<float> h;
  off.assign(FUSION_NP, 0);
  auto put = [&](const float* src, size_t cnt) {
    size_t o = h.size();
    h.insert(h.end(), src, src + cnt);
    return o;
  };
  auto putT = [&](const float* src, int out, int in) {  // torch [out,in] -> [in][out]
    size_t o = h.size();
    h.resize(o + (size_t)out * in);
    for (int i = 0; i < in; ++i)
      for (int j = 0; j < out; ++j) h[o + (size_t)i * out + j] = src[(size_t)j * in + i];
    return o;
  };
  auto lin = [&](int idx, int out, int in) {
    off[idx] = putT(rd.take((size_t)out * in), out, in);
    off[idx + 1] = put(rd.take(out), out);
  };
  auto ln = [&](int idx, int c) {
    off[idx] = put(rd.take(c), c);
    off[idx + 1] = put(rd.take(c), c);
  };
  const int dims[3] = {64, 768, 512};
  for (int m = 0; m < 3; ++m) { lin(4 * m, 256, dims[m]); ln(4 * m + 2, 256); }
  for (int m = 0; m < 3; ++m) {
    const int b = 12 + 10 * m;
    const float* ipw = rd.take(768 * 256);
    const float* ipb = rd.take(768);
    for (int q = 0; q < 3; ++q) {
      off[b + 2 * q] = putT(ipw + (size_t)q * 256 * 256, 256, 256);
      off[b + 2 * q + 1] = put(ipb + q * 256, 256);
    }
    lin(b + 6, 256, 256);
    ln(b + 8, 256);
  }
  for (int j = 0; j < 3; ++j) { lin(42 + 4 * j, 256, 256); ln(44 + 4 * j, 256); }
  lin(54, 256, 768);
  lin(56, 3, 256);
  lin(58, 64, 21);
  lin(60, 3, 64);
  lin(62, 256, 263);
  ln(64, 256);
  lin(66, 128, 256);
  lin(68, 7, 128);
  MEC_REQUIRE(rd.ok && rd.off == n, "fusion blob size mismatch");
  return upload(w, h.data(), h.size() * sizeof(float));
}

int FusionModel::forward(const float* sf, const float* tf, const float* imf, const float* sp,
                         const float* tp, const float* ip, int B, float* logits, float* probs,
                         float* attn_w, float* dec_w, hipStream_t s) {
  MEC_REQUIRE(B >= 0, "fusion: B < 0");
  if (B == 0) return 0;
  MEC_REQUIRE(sf && tf && imf && sp && tp && ip && logits && probs && attn_w && dec_w,
              "fusion: null pointer (the attention model needs all three modalities)");
  FusionW p;
  const float* base = w.as<float>();
  for (int i = 0; i < FUSION_NP; ++i) p.p[i] = base + off[i];
  MEC_TRY(prof.begin(TAG_FUSION, s));
  const int R = opt().fusion_r;
  const dim3 grid((B + R - 1) / R), blk(SF_THREADS);
  if (opt().fusion_split) {
    if (B > ws_batch) {
      MEC_TRY(ws.ensure((size_t)B * 768 * 2 * sizeof(float)));
      ws_batch = B;
    }
    float* Pg = ws.as<float>();
    float* Tg = Pg + (size_t)B * 768;
    switch (R) {
      case 1: launch_fusion_split<1>(p, sf, tf, imf, sp, tp, ip, B, Pg, Tg, logits, probs, attn_w, dec_w, s); break;
      case 4: launch_fusion_split<4>(p, sf, tf, imf, sp, tp, ip, B, Pg, Tg, logits, probs, attn_w, dec_w, s); break;
      default: launch_fusion_split<2>(p, sf, tf, imf, sp, tp, ip, B, Pg, Tg, logits, probs, attn_w, dec_w, s); break;
    }
    MEC_LAUNCH_CHECK();
    MEC_TRY(prof.end(TAG_FUSION, s));
    return 0;
  }
  switch (R) {
    case 1: hipLaunchKernelGGL((fusion_kernel<1>), grid, blk, 0, s, p, sf, tf, imf, sp, tp, ip, B, logits, probs, attn_w, dec_w); break;
    case 4: hipLaunchKernelGGL((fusion_kernel<4>), grid, blk, 0, s, p, sf, tf, imf, sp, tp, ip, B, logits, probs, attn_w, dec_w); break;
    default: hipLaunchKernelGGL((fusion_kernel<2>), grid, blk, 0, s, p, sf, tf, imf, sp, tp, ip, B, logits, probs, attn_w, dec_w); break;
  }
  MEC_LAUNCH_CHECK();
  MEC_TRY(prof.end(TAG_FUSION, s));
  return 0;
}

// =============================================================== weighted average
template <class T>
__global__ void fuse_weighted_kernel(const T* s, const T* t, const T* i, int B, double* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double w[7];
  for (int c = 0; c < 7; ++c) {
    const double vs = s ? (double)s[b * 7 + c] : 0.0;
    const double vt = t ? (double)t[b * 7 + c] : 0.0;
    const double vi = i ? (double)i[b * 7 + c] : 0.0;
    w[c] = 0.3 * vs + 0.35 * vt + 0.35 * vi;  // weights [0.3, 0.35, 0.35] (multimodal_fusion.py:23)
  }
  double sum = 0.0;
  for (int c = 0; c < 7; ++c) sum += w[c];
  for (int c = 0; c < 7; ++c) out[b * 7 + c] = sum > 0.0 ? w[c] / sum : w[c];
}

template <class T>
static int fuse_weighted_t(const T* s, const T* t, const T* i, int B, double* out, hipStream_t st) {
  MEC_REQUIRE(B >= 0 && (B == 0 || out), "fuse_weighted: bad args");
  if (B == 0) return 0;
  hipLaunchKernelGGL((fuse_weighted_kernel<T>), dim3((B + 255) / 256), dim3(256), 0, st, s, t, i, B, out);
  MEC_LAUNCH_CHECK();
  return 0;
}

int fuse_weighted(const float* s, const float* t, const float* i, int B, double* out, hipStream_t st) {
  return fuse_weighted_t<float>(s, t, i, B, out, st);
}

int fuse_weighted_f64(const double* s, const double* t, const double* i, int B, double* out, hipStream_t st) {
  return fuse_weighted_t<double>(s, t, i, B, out, st);
}

}  // namespace mec
