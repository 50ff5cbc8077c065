// BERT-base in fp32 end to end (mec_create_ex(..., MEC_PREC_FP32)): the reference's own
// precision (transformers BertForSequenceClassification in fp32, inference/text_inference.py:
// 41, :92-93). Every GEMM runs on the fp32 engine (gemm_f32.hip, v_mfma_f32_32x32x2_f32) and
// the attention on f32 MFMAs; LayerNorm, GELU (libm erff), softmax and the residual stream are
// fp32 as on the f16 path. Per layer (M = B*L rows):
//   qkv32 = h32 . Wqkv^T + b                   gemm_f32 (N = 2304)
//   ctx32 = softmax(QK^T/8 + mask_bias) V      bert_attention_f32_kernel
//   t32   = ctx32 . Wo^T + bo + h32            gemm_f32, residual fused
//   h32   = LN(t32)                            bert_layernorm_kernel (f32 out only)
//   i32   = GELU(h32 . Wi^T + bi)              gemm_f32 (N = 3072), exact erf
//   t32   = i32 . Wo2^T + bo2 + h32            gemm_f32
//   h32   = LN(t32)
// Head as on the f16 path (pooler tanh + classifier + softmax, block_ops.h).
#include "block_ops.h"
#include "models.h"

namespace mec {

namespace {
constexpr int H = 768, FF = 3072, NH = 12, DH = 64, NL = 12, AL = 128;
constexpr size_t PRM_LAYER = 2304 + 768 * 3 + 3072 + 768 * 3;
constexpr size_t WT_LAYER = (size_t)2304 * 768 + 768 * 768 + 3072 * 768 + 768 * 3072;
}  // namespace

// K rows in LDS: 16 chunks of 16 B per 256-B row, chunk c stored at c ^ (row & 15), so the 16
// rows of a ds_read_b128 lane group cover all 64 banks.
__device__ __forceinline__ int kswz(int row, int c) { return c ^ (row & 15); }

// One workgroup per (sequence, head), 4 waves; wave w owns queries 32w .. 32w+31.
// S^T = K Q^T on v_mfma_f32_32x32x2_f32 (A = K rows from LDS, B = Q^T from registers), so each
// lane holds one query's scores over 64 keys (the other 64 in lane ^ 32): the row softmax is
// lane-local plus one shuffle. O^T = V^T P^T: A = V[key][d] read as one f32 per lane (row-major
// V, 32 consecutive d per half wave), B = the lane's own probabilities, in the k order the
// score tile left them (two keys per MFMA: key f(e) + 4h of block t for lane half h).
// SPLIT (fp32x3 path): ctx is written as f16 hi / lo planes (ctx16, ctx16 + lo) for the split
// O-projection GEMM instead of f32.
// CLS = 1 (the last layer with bert_cls_last): qkv holds K | V only ([B*128, 1536]), the [CLS] query
// row comes from qc ([B, 768]) and the context is written compact ([B, 768]); wave 0 computes
// queries 0..31 with Q zero for all but query 0 (an MFMA output column depends only on its own B
// column: the [CLS] context has the full kernel's bits), waves 1-3 only stage K and V.
template <int SPLIT = 0, int CLS = 0>
__global__ __launch_bounds__(256, 2) void bert_attention_f32_kernel(const float* __restrict__ qkv,
                                                                    const int32_t* __restrict__ mask,
                                                                    float* __restrict__ ctx, f16* __restrict__ ctx16,
                                                                    long long lo, const float* __restrict__ qc) {
  constexpr int LD = CLS ? 2 * H : 3 * H, KO = CLS ? 0 : H;
  __shared__ __attribute__((aligned(16))) float sK[AL * DH];
  __shared__ __attribute__((aligned(16))) float sV[AL * DH];
  __shared__ float sBias[AL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / NH, h = blockIdx.x - (blockIdx.x / NH) * NH;
  const float* base = qkv + (size_t)b * AL * LD + h * DH;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + 256 * i;
    const int row = c >> 4, kc = c & 15;
    const float* src = base + (size_t)row * LD + kc * 4;
    const float4 k = *reinterpret_cast<const float4*>(src + KO);
    const float4 v = *reinterpret_cast<const float4*>(src + KO + H);
    *reinterpret_cast<float4*>(sK + row * DH + kswz(row, kc) * 4) = k;
    *reinterpret_cast<float4*>(sV + row * DH + kc * 4) = v;
  }
  if (tid < AL) sBias[tid] = mask[(size_t)b * AL + tid] ? 0.f : -3.4028234663852886e38f;  // finfo(f32).min
  const int lr = lane & 31, lh = lane >> 5;
  const int q = 32 * wave + lr;
  float4 qf[8];  // Q[q][8s + 4lh .. +3]
  if constexpr (CLS) {
    const bool own = wave == 0 && lr == 0;
    const float* qrow = qc + (size_t)b * H + h * DH;
#pragma unroll
    for (int s = 0; s < 8; ++s)
      qf[s] = own ? *reinterpret_cast<const float4*>(qrow + (2 * s + lh) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const float4*>(base + (size_t)q * LD + (2 * s + lh) * 4);
  }
  __syncthreads();
  if (CLS && wave != 0) return;

  floatx16 st[4];  // st[t][e] = S[q][key 32t + (e&3) + 8(e>>2) + 4lh]
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int e = 0; e < 16; ++e) st[t][e] = 0.f;
    const int rk = 32 * t + lr;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float4 kf = *reinterpret_cast<const float4*>(sK + rk * DH + kswz(rk, 2 * s + lh) * 4);
      st[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.x, qf[s].x, st[t], 0, 0, 0);
      st[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.y, qf[s].y, st[t], 0, 0, 0);
      st[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.z, qf[s].z, st[t], 0, 0, 0);
      st[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.w, qf[s].w, st[t], 0, 0, 0);
    }
  }
  // scores / sqrt(64) + additive mask (HF eager order), softmax over the 128 keys
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int key = 32 * t + (e & 3) + 8 * (e >> 2) + 4 * lh;
      const float v = st[t][e] * 0.125f + sBias[key];
      st[t][e] = v;
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float p = expf(st[t][e] - mx);
      st[t][e] = p;
      sum += p;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.0f / sum;

  floatx16 o[2];  // o[u][e] = O[q][d = 32u + (e&3) + 8(e>>2) + 4lh]
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[u][e] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int key = 32 * t + (e & 3) + 8 * (e >> 2) + 4 * lh;
      const float p = st[t][e] * inv;
#pragma unroll
      for (int u = 0; u < 2; ++u) o[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(sV[key * DH + 32 * u + lr], p, o[u], 0, 0, 0);
    }
  if (CLS && lr != 0) return;
  const size_t obase = ((size_t)b * (CLS ? 1 : AL) + q) * H + h * DH;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const size_t oi = obase + 32 * u + 8 * g + 4 * lh;
      if constexpr (SPLIT) {
        half4 hh, hl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          hh[e] = (f16)o[u][4 * g + e];
          hl[e] = (f16)(o[u][4 * g + e] - (float)hh[e]);
        }
        *reinterpret_cast<half4*>(ctx16 + oi) = hh;
        *reinterpret_cast<half4*>(ctx16 + lo + oi) = hl;
      } else {
        *reinterpret_cast<float4*>(ctx + oi) =
            make_float4(o[u][4 * g + 0], o[u][4 * g + 1], o[u][4 * g + 2], o[u][4 * g + 3]);
      }
    }
}

int TextModel::forward_f32(const int32_t* ids, const int32_t* mask, int B, int L, float* cls, float* logits,
                           float* probs, hipStream_t s) {
  MEC_REQUIRE(wts32.p, "text: fp32 weights missing (handle created at f16 precision)");
  const int M = B * L;
  // workspace: h32 | t32 | ctx32 (f32 [M,768]) ; big32 f32 [M,3072] (qkv [M,2304], then FFN) ; pooled [B,768] ;
  // the [CLS]-row buffers of the last layer (bert_cls_last): h32c | t32c | qc | ctxc [B,768], fc [B,3072]
  const size_t need = (size_t)M * H * 4 * 3 + (size_t)M * FF * 4 + (size_t)B * H * 4 * 5 + (size_t)B * FF * 4;
  if (ws.bytes < need) MEC_TRY(ws.ensure(need));
  char* p = ws.as<char>();
  float* h32 = reinterpret_cast<float*>(p); p += (size_t)M * H * 4;
  float* t32 = reinterpret_cast<float*>(p); p += (size_t)M * H * 4;
  float* ctx32 = reinterpret_cast<float*>(p); p += (size_t)M * H * 4;
  float* big32 = reinterpret_cast<float*>(p); p += (size_t)M * FF * 4;
  float* pooled = reinterpret_cast<float*>(p); p += (size_t)B * H * 4;
  float* h32c = reinterpret_cast<float*>(p); p += (size_t)B * H * 4;
  float* t32c = reinterpret_cast<float*>(p); p += (size_t)B * H * 4;
  float* qc = reinterpret_cast<float*>(p); p += (size_t)B * H * 4;
  float* ctxc = reinterpret_cast<float*>(p); p += (size_t)B * H * 4;
  float* fc = reinterpret_cast<float*>(p);
  const bool cls_last = opt().bert_cls_last != 0;

  MEC_TRY(launch_bert_embed_ln(ids, M, L, emb.as<float>(), h32, nullptr, s));
  const float* W = wts32.as<float>();
  const float* P = prm.as<float>();
  for (int l = 0; l < NL; ++l) {
    const float* wqkv = W + WT_LAYER * l;
    const float* wo = wqkv + (size_t)2304 * H;
    const float* wi = wo + (size_t)H * H;
    const float* wo2 = wi + (size_t)FF * H;
    const float* pl = P + PRM_LAYER * l;
    const float *bqkv = pl, *bo = pl + 2304, *g1 = pl + 3072, *b1 = pl + 3840, *bi = pl + 4608, *bo2 = pl + 7680,
                *g2 = pl + 8448, *b2 = pl + 9216;
    GemmParams g;
    if (cls_last && l == NL - 1) {
      // [CLS]-only last layer (TextModel::forward): K / V for every token, the rest on the [CLS] rows
      RowGather rg{};
      rg.n = 1;
      rg.src[0] = reinterpret_cast<const char*>(h32); rg.dst[0] = reinterpret_cast<char*>(h32c);
      rg.sstride[0] = (long long)AL * H * 4; rg.bytes[0] = H * 4;
      MEC_TRY(launch_gather_rows(rg, B, s));
      g.A = h32; g.B32 = wqkv + (size_t)H * H; g.bias = bqkv + H; g.C32 = big32; g.M = M; g.N = 2 * H; g.K = H;
      MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_NONE));  // K | V [M, 1536]
      g = GemmParams();
      g.A = h32c; g.B32 = wqkv; g.bias = bqkv; g.C32 = qc; g.M = B; g.N = H; g.K = H;
      MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_NONE));  // Q of the [CLS] rows
      hipLaunchKernelGGL((bert_attention_f32_kernel<0, 1>), dim3(B * NH), dim3(256), 0, s, big32, mask, ctxc, nullptr,
                         0LL, qc);
      MEC_LAUNCH_CHECK();
      g = GemmParams();
      g.A = ctxc; g.B32 = wo; g.bias = bo; g.R = h32c; g.r_f32 = 1; g.C32 = t32c; g.M = B; g.N = H; g.K = H;
      MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_NONE));
      MEC_TRY(launch_bert_layernorm(t32c, B, g1, b1, h32c, nullptr, nullptr, s));
      g = GemmParams();
      g.A = h32c; g.B32 = wi; g.bias = bi; g.act = ACT_GELU_EXACT; g.C32 = fc; g.M = B; g.N = FF; g.K = H;
      MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_NONE));
      g = GemmParams();
      g.A = fc; g.B32 = wo2; g.bias = bo2; g.R = h32c; g.r_f32 = 1; g.C32 = t32c; g.M = B; g.N = H; g.K = FF;
      MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_NONE));
      MEC_TRY(launch_bert_layernorm(t32c, B, g2, b2, h32c, nullptr, nullptr, s));
      break;
    }
    g.A = h32; g.B32 = wqkv; g.bias = bqkv; g.C32 = big32; g.M = M; g.N = 2304; g.K = H;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_BERT_QKV));
    MEC_TRY(prof.begin(TAG_BERT_ATTN, s));
    hipLaunchKernelGGL((bert_attention_f32_kernel<0, 0>), dim3(B * NH), dim3(256), 0, s, big32, mask, ctx32, nullptr, 0LL,
                       nullptr);
    MEC_LAUNCH_CHECK();
    MEC_TRY(prof.end(TAG_BERT_ATTN, s));
    g = GemmParams();
    g.A = ctx32; g.B32 = wo; g.bias = bo; g.R = h32; g.r_f32 = 1; g.C32 = t32; g.M = M; g.N = H; g.K = H;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_BERT_OPROJ));
    MEC_TRY(prof.begin(TAG_BERT_LN, s));
    MEC_TRY(launch_bert_layernorm(t32, M, g1, b1, h32, nullptr, nullptr, s));
    MEC_TRY(prof.end(TAG_BERT_LN, s));
    g = GemmParams();
    g.A = h32; g.B32 = wi; g.bias = bi; g.act = ACT_GELU_EXACT; g.C32 = big32; g.M = M; g.N = FF; g.K = H;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_BERT_FFN1));
    g = GemmParams();
    g.A = big32; g.B32 = wo2; g.bias = bo2; g.R = h32; g.r_f32 = 1; g.C32 = t32; g.M = M; g.N = H; g.K = FF;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_BERT_FFN2));
    MEC_TRY(prof.begin(TAG_BERT_LN, s));
    MEC_TRY(launch_bert_layernorm(t32, M, g2, b2, h32, nullptr, nullptr, s));
    MEC_TRY(prof.end(TAG_BERT_LN, s));
  }
  const float* head = P + PRM_LAYER * NL;
  const float *WpT = head, *bp = WpT + (size_t)H * H, *WcT = bp + H, *bc = WcT + (size_t)H * 7;
  MEC_TRY(launch_linear_mfma<BACT_TANH>(cls_last ? h32c : h32, cls_last ? (size_t)H : (size_t)L * H, B, H, WpT, bp,
                                        H, pooled, H, cls, H, s));
  MEC_TRY(launch_head7(pooled, B, H, WcT, bc, logits, probs, s));
  return 0;
}

// fp32x3 path: the fp32 path's structure with every GEMM on split-f16 operands (gemm_glds.hip
// split mode, three f16 MFMA passes into one fp32 accumulator). Per layer (M = B*L rows):
//   qkv hi/lo   = [h_hi|h_lo] . [Wqkv_hi|Wqkv_lo]^T 2^-e + b        split GEMM, split out
//   ctx hi/lo   = softmax(QK^T/8 + mask_bias) V                     bert_attention_x3_kernel (split
//                                                                    MFMA products, fp32 softmax)
//   t32         = ctx . Wo^T 2^-e + bo + LN2'(h32)                  split GEMM, f32 residual (deferred LN)
//   h hi/lo, st1 = LN(t32)                                          bert_layernorm_kernel (lo plane, stats)
//   i hi/lo     = GELU(h . Wi^T 2^-e + bi)                          split GEMM, exact erf, split out
//   h32         = i . Wo2^T 2^-e + bo2 + LN1'(t32)                  split GEMM (deferred LN)
//   h hi/lo, st2 = LN(h32)
int TextModel::forward_x3(const int32_t* ids, const int32_t* mask, int B, int L, float* cls, float* logits,
                          float* probs, hipStream_t s) {
  MEC_REQUIRE(wts.p && x3_lo && x3_scale.size() == 4 * NL, "text: fp32x3 weights missing");
  const int M = B * L;
  const long long MH = (long long)M * H, MF = (long long)M * FF;
  // workspace: h32 | t32 (f32 [M,768]) ; h hi|lo, ctx hi|lo (f16 2x[M,768]) ; big: qkv hi|lo
  // (f16 2x[M,2304]), then the FFN intermediate hi|lo (f16 2x[M,3072]) ; pooled [B,768]
  // + the [CLS]-row buffers of the last layer (bert_cls_last): h32c | t32c (f32 [B,768]) ; hsc | qsc | csc
  // (f16 planes 2x[B,768]) ; fsc (f16 planes 2x[B,3072])
  const long long BHc = (long long)B * H, BFc = (long long)B * FF;
  // + the LayerNorm row stats st1 | st2 ([M] float2; deferred LayerNorm, below) and st2c ([B] float2)
  const size_t need = (size_t)MH * 4 * 2 + (size_t)MH * 2 * 4 + (size_t)MF * 4 + (size_t)B * H * 4 +
                      (size_t)BHc * 4 * 2 + (size_t)BHc * 4 * 3 + (size_t)BFc * 4 + (size_t)M * 8 * 2 + (size_t)B * 8;
  if (ws.bytes < need) MEC_TRY(ws.ensure(need));
  char* p = ws.as<char>();
  float* h32 = reinterpret_cast<float*>(p); p += (size_t)MH * 4;
  float* t32 = reinterpret_cast<float*>(p); p += (size_t)MH * 4;
  f16* hs = reinterpret_cast<f16*>(p); p += (size_t)MH * 2 * 2;
  f16* cs = reinterpret_cast<f16*>(p); p += (size_t)MH * 2 * 2;
  float* big32 = reinterpret_cast<float*>(p);
  f16* bigs = reinterpret_cast<f16*>(p); p += (size_t)MF * 4;
  float* pooled = reinterpret_cast<float*>(p); p += (size_t)B * H * 4;
  float* h32c = reinterpret_cast<float*>(p); p += (size_t)BHc * 4;
  float* t32c = reinterpret_cast<float*>(p); p += (size_t)BHc * 4;
  f16* hsc = reinterpret_cast<f16*>(p); p += (size_t)BHc * 4;
  f16* qsc = reinterpret_cast<f16*>(p); p += (size_t)BHc * 4;
  f16* csc = reinterpret_cast<f16*>(p); p += (size_t)BHc * 4;
  f16* fsc = reinterpret_cast<f16*>(p); p += (size_t)BFc * 4;
  float2* st1 = reinterpret_cast<float2*>(p);  // LN1 row stats [M]
  float2* st2 = st1 + M;                       // LN2 row stats [M]
  float2* st2c = st2 + M;                      // LN2 row stats of the [CLS] rows [B]
  const bool cls_last = opt().bert_cls_last != 0;
  const int gelu_act = opt().gelu_x3 ? ACT_GELU_F32 : ACT_GELU_EXACT;  // FFN1's erf GELU

  MEC_TRY(launch_bert_embed_ln(ids, M, L, emb.as<float>(), h32, hs, s, MH, std::ldexp(1.0f, x3_s_emb)));
  const f16* W = wts.as<f16>();
  const float* P = prm.as<float>();
  const long long wlo = (long long)x3_lo;
  for (int l = 0; l < NL; ++l) {
    const f16* wqkv = W + WT_LAYER * l;
    const f16* wo = wqkv + (size_t)2304 * H;
    const f16* wi = wo + (size_t)H * H;
    const f16* wo2 = wi + (size_t)FF * H;
    const float* sc = x3_scale.data() + 4 * l;
    const float* pl = P + PRM_LAYER * l;
    const float *bo = pl + 2304, *g1 = pl + 3072, *b1 = pl + 3840, *bi = pl + 4608, *bo2 = pl + 7680,
                *g2 = pl + 8448, *b2 = pl + 9216;
    // activation-plane scales (TextModel::create): Q / K / V through the pre-scaled Wqkv planes and bqkv
    // (x3b), the scores by 1/8 2^-(s_q + s_k), the LN outputs by up1 / up2, the FFN intermediate by
    // cscale (ffs)
    const float* bqkv = x3b.as<float>() + (size_t)2304 * l;
    const float qks = std::ldexp(0.125f, -(x3_s_q[l] + x3_s_k[l]));
    const float up1 = std::ldexp(1.0f, x3_s_ln1[l]), up2 = std::ldexp(1.0f, x3_s_ln2[l]);
    const float ffs = std::ldexp(1.0f, x3_s_ffn[l]);
    GemmParams g;
    if (cls_last && l == NL - 1) {
      // [CLS]-only last layer (TextModel::forward): K / V for every token, the rest on the [CLS] rows
      RowGather rg{};
      rg.n = 3;
      rg.src[0] = reinterpret_cast<const char*>(h32); rg.dst[0] = reinterpret_cast<char*>(h32c);
      rg.sstride[0] = (long long)AL * H * 4; rg.bytes[0] = H * 4;
      rg.src[1] = reinterpret_cast<const char*>(hs); rg.dst[1] = reinterpret_cast<char*>(hsc);
      rg.sstride[1] = (long long)AL * H * 2; rg.bytes[1] = H * 2;
      rg.src[2] = reinterpret_cast<const char*>(hs + MH); rg.dst[2] = reinterpret_cast<char*>(hsc + BHc);
      rg.sstride[2] = (long long)AL * H * 2; rg.bytes[2] = H * 2;
      if (l > 0) {  // h32 holds layer l-1's pre-LN2 sum (deferred LayerNorm): its stats too
        rg.n = 4;
        rg.src[3] = reinterpret_cast<const char*>(st2); rg.dst[3] = reinterpret_cast<char*>(st2c);
        rg.sstride[3] = (long long)AL * 8; rg.bytes[3] = 8;
      }
      MEC_TRY(launch_gather_rows(rg, B, s));
      const float* pg2 = P + PRM_LAYER * (l - 1) + 8448;  // layer l-1's LN2 (g2, b2)
      const long long kvlo = (long long)M * 2 * H;
      g.split = 1; g.A = hs; g.a_lo = MH; g.B = wqkv + (size_t)H * H; g.b_lo = wlo; g.oscale = sc[0];
      g.bias = bqkv + H; g.C16 = bigs; g.c_lo = kvlo; g.M = M; g.N = 2 * H; g.K = H;
      MEC_TRY(launch_gemm(g, s, &prof, TAG_NONE));  // K | V planes [M, 1536]
      g = GemmParams();
      g.split = 1; g.A = hsc; g.a_lo = BHc; g.B = wqkv; g.b_lo = wlo; g.oscale = sc[0];
      g.bias = bqkv; g.C16 = qsc; g.c_lo = BHc; g.M = B; g.N = H; g.K = H;
      MEC_TRY(launch_gemm(g, s, &prof, TAG_NONE));  // Q planes of the [CLS] rows
      MEC_TRY(launch_bert_attention_x3_cls(bigs, kvlo, mask, qsc, BHc, csc, BHc, B, qks, s));
      g = GemmParams();
      g.split = 1; g.A = csc; g.a_lo = BHc; g.B = wo; g.b_lo = wlo; g.oscale = sc[1];
      g.bias = bo; g.R = h32c; g.r_f32 = 1; g.C32 = t32c; g.M = B; g.N = H; g.K = H;
      if (l > 0) { g.r_stats = st2c; g.r_g = pg2; g.r_b = pg2 + H; }
      MEC_TRY(launch_gemm(g, s, &prof, TAG_NONE));
      MEC_TRY(launch_bert_layernorm(t32c, B, g1, b1, h32c, hsc, nullptr, s, BHc, up1));
      g = GemmParams();
      g.split = 1; g.A = hsc; g.a_lo = BHc; g.B = wi; g.b_lo = wlo; g.oscale = sc[2];
      g.bias = bi; g.act = gelu_act; g.C16 = fsc; g.c_lo = BFc; g.cscale = ffs; g.M = B; g.N = FF; g.K = H;
      MEC_TRY(launch_gemm(g, s, &prof, TAG_NONE));
      g = GemmParams();
      g.split = 1; g.A = fsc; g.a_lo = BFc; g.B = wo2; g.b_lo = wlo; g.oscale = sc[3];
      g.bias = bo2; g.R = h32c; g.r_f32 = 1; g.C32 = t32c; g.M = B; g.N = H; g.K = FF;
      MEC_TRY(launch_gemm(g, s, &prof, TAG_NONE));
      MEC_TRY(launch_bert_layernorm(t32c, B, g2, b2, h32c, hsc, nullptr, s, BHc, up2));
      break;
    }
    // QKV projection + attention fused (Q / K / V stay on chip). The fused kernel sums in the K-interleaved
    // term order only, so with gemm_x3_order 0 (pass-major) the split GEMM + attention pair runs instead
    // and every split product of the forward keeps one term order
    if (opt().bert_qkv_attn == 1 && L == 128 && opt().gemm_x3_order == 1) {
      MEC_TRY(prof.begin(TAG_BERT_QKV, s));
      MEC_TRY(launch_bert_qkv_attn_x3(hs, MH, wqkv, wlo, sc[0], bqkv, mask, cs, MH, B, qks, s));
      MEC_TRY(prof.end(TAG_BERT_QKV, s));
    } else {
      g.split = 1; g.A = hs; g.a_lo = MH; g.B = wqkv; g.b_lo = wlo; g.oscale = sc[0];
      g.bias = bqkv; g.C16 = bigs; g.c_lo = (long long)M * 2304; g.M = M; g.N = 2304; g.K = H;
      MEC_TRY(launch_gemm(g, s, &prof, TAG_BERT_QKV));
      MEC_TRY(prof.begin(TAG_BERT_ATTN, s));
      MEC_TRY(launch_bert_attention_x3(bigs, (long long)M * 2304, mask, cs, MH, B, qks, s));
      MEC_TRY(prof.end(TAG_BERT_ATTN, s));
    }
    // deferred LayerNorm (as on the f16 path): the LN kernels write the GEMM operand planes and the
    // row (mean, rstd) only; the f32 LN output is needed only as the next residual, which the
    // O-proj / FFN2 epilogue re-derives from the pre-LN sum with the LN kernel's own expression
    // (GemmParams::r_stats): same bits, two 100-MB f32 writes per layer fewer at B = 256. The f32
    // stream ping-pongs (O-proj h32 -> t32, FFN2 t32 -> h32) so no GEMM reads its own output.
    const bool first = l == 0, last = l == NL - 1;
    const float* pg2 = P + PRM_LAYER * (l - 1) + 8448;  // layer l-1's LN2 (g2, b2)
    g = GemmParams();
    g.split = 1; g.A = cs; g.a_lo = MH; g.B = wo; g.b_lo = wlo; g.oscale = sc[1];
    g.bias = bo; g.R = h32; g.r_f32 = 1; g.C32 = t32; g.M = M; g.N = H; g.K = H;
    if (!first) { g.r_stats = st2; g.r_g = pg2; g.r_b = pg2 + H; }  // else: the embedding LN, written in full
    MEC_TRY(launch_gemm(g, s, &prof, TAG_BERT_OPROJ));
    MEC_TRY(prof.begin(TAG_BERT_LN, s));
    MEC_TRY(launch_bert_layernorm(t32, M, g1, b1, nullptr, hs, st1, s, MH, up1));
    MEC_TRY(prof.end(TAG_BERT_LN, s));
    g = GemmParams();
    g.split = 1; g.A = hs; g.a_lo = MH; g.B = wi; g.b_lo = wlo; g.oscale = sc[2];
    g.bias = bi; g.act = gelu_act; g.C16 = bigs; g.c_lo = MF; g.cscale = ffs; g.M = M; g.N = FF; g.K = H;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_BERT_FFN1));
    g = GemmParams();
    g.split = 1; g.A = bigs; g.a_lo = MF; g.B = wo2; g.b_lo = wlo; g.oscale = sc[3];
    g.bias = bo2; g.R = t32; g.r_f32 = 1; g.r_stats = st1; g.r_g = g1; g.r_b = b1; g.C32 = h32;
    g.M = M; g.N = H; g.K = FF;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_BERT_FFN2));
    MEC_TRY(prof.begin(TAG_BERT_LN, s));
    // the last LN's f32 output feeds the pooler, so it is written in full (in place)
    MEC_TRY(launch_bert_layernorm(h32, M, g2, b2, last ? h32 : nullptr, hs, st2, s, MH, up2));
    MEC_TRY(prof.end(TAG_BERT_LN, s));
  }
  const float* head = P + PRM_LAYER * NL;
  const float *WpT = head, *bp = WpT + (size_t)H * H, *WcT = bp + H, *bc = WcT + (size_t)H * 7;
  MEC_TRY(launch_linear_mfma<BACT_TANH>(cls_last ? h32c : h32, cls_last ? (size_t)H : (size_t)L * H, B, H, WpT, bp,
                                        H, pooled, H, cls, H, s));
  MEC_TRY(launch_head7(pooled, B, H, WcT, bc, logits, probs, s));
  return 0;
}

}  // namespace mec
