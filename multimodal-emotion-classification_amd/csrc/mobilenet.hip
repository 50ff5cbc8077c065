// Image path on a MobileNetV2 backbone (README.md:13; BASELINE config "Image-only:
// MobileNetV2 on 48x48x1 FER2013 tensors"): the reference's transform (PIL-exact resize,
// ToTensor, Normalize; inference/image_inference.py:28-32) -> torchvision mobilenet_v2
// features -> avgpool -> the reference's Dropout/Linear(.,512)/ReLU/Dropout/Linear(512,7)
// head on 1280 features (image_inference.py:59-65). Restated by oracle/image_mbv2.py.
//
// Every inverted-residual block is ONE kernel (mbv2_block_kernel): a workgroup owns a
// TOxTO tile of output pixels of one image, stages the block input tile (with the 3x3
// halo) in LDS once, and walks the hidden channels in chunks of 32:
//   expand  1x1 conv + BN + ReLU6 on MFMA (v_mfma_f32_16x16x32_f16) -> LDS (f16)
//   dw      3x3 depthwise/s + BN + ReLU6 on VALU, fp32 accumulate   -> LDS (f16)
//   project 1x1 conv on MFMA, accumulated over the chunks in registers
// then adds BN shift + the residual (from the staged input tile) and writes the output
// tile with 16-B stores. The expanded (6x wider) activations never touch HBM: a block
// reads its input once (plus halo) and writes its output once, so the backbone is bound by
// those bytes, not by the hidden tensors. Block 1 (t = 1) also computes the stem conv
// (3x3/2 on the raw u8 image, ToTensor/Normalize and BN folded into the weights, border
// taps handled by a 4-class bias table) for its tile, so the 112x112x32 stem output is
// never written either.
#include <algorithm>
#include <cmath>

#include "block_ops.h"
#include "models.h"

namespace mec {

constexpr int MB_HC = 32;  // hidden channels per chunk

struct MbArgs {
  const f16* x;        // block input NHWC [B,H,H,cin] (STEM == 0) or u8 image [B,224,224,C]
  f16* y;              // block output NHWC [B,OH,OH,cout]
  int H, OH, cin, cout, hidp;
  const f16* We;       // [hidp][CINP]
  const float* be;     // [hidp]
  const float* Wd;     // [hidp/8][9][8]
  const float* bd;     // [hidp]
  const f16* Wp;       // [COUTP][hidp]
  const float* bp;     // [COUTP]
  const float* stem_w;     // [C*9][32] folded stem weights (STEM > 0)
  const float* stem_corr;  // [4][32] bias per border class (STEM > 0)
};

__device__ __forceinline__ float relu6f(float v) { return fminf(fmaxf(v, 0.f), 6.f); }

// S stride, TO output tile side, CINP / HIDP / COUTP padded channel counts, EXPAND (t != 1),
// RES (stride 1 and cin == cout), STEM: 0 = input from HBM, 1 / 3 = stem from u8 gray / RGB.
// Latency: every global load a phase needs is issued a phase early (the input tile in one
// unrolled burst; depthwise weights and all biases staged in LDS next to it; the project
// weights of chunk c at the start of chunk c; the expand weights of chunk c+1 right after
// chunk c's expand), so a chunk costs its LDS/MFMA/VALU work, not three load round trips.
template <int S, int TO, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM>
__global__ __launch_bounds__(256) void mbv2_block_kernel(const MbArgs a) {
  constexpr int IR = (TO - 1) * S + 3;        // input tile side (with halo)
  constexpr int NP = IR * IR;
  constexpr int MP = (NP + 15) / 16 * 16;     // input pixels padded to MFMA tiles
  constexpr int XLD = CINP + 8;               // LDS row strides (halfs), +16 B against conflicts
  constexpr int ELD = MB_HC + 8;
  constexpr int OLD = COUTP + 8;
  constexpr int NQ = TO * TO;                 // output pixels (<= 64: four 16-pixel tiles)
  constexpr int OT = COUTP / 16;              // project M tiles
  constexpr int KX = CINP / 32;               // expand k steps
  static_assert(NQ <= 64, "tile");
  static_assert(!STEM || (CINP == 32 && HIDP == 32 && !EXPAND && S == 1), "stem fuses into block 1 only");
  __shared__ __attribute__((aligned(16))) f16 sX[MP * XLD];
  __shared__ __attribute__((aligned(16))) f16 sE[EXPAND ? MP * ELD : 8];
  __shared__ __attribute__((aligned(16))) f16 sD[64 * ELD];
  __shared__ __attribute__((aligned(16))) f16 sO[64 * OLD];
  __shared__ __attribute__((aligned(16))) float sWd[HIDP * 9];   // [HIDP/8][9][8]
  __shared__ __attribute__((aligned(16))) float sBd[HIDP];
  __shared__ __attribute__((aligned(16))) float sBe[EXPAND ? HIDP : 4];
  __shared__ __attribute__((aligned(16))) float sBp[COUTP];
  constexpr int PR = 2 * (TO + 2) + 1;        // stem: u8 patch side (STEM > 0)
  __shared__ __attribute__((aligned(16))) float sSW[STEM ? STEM * 9 * 32 : 4];
  __shared__ uint8_t sPatch[STEM ? PR * PR * STEM : 4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpr = a.OH / TO;
  const int n = blockIdx.x / (tpr * tpr);
  const int tt = blockIdx.x - n * tpr * tpr;
  const int oy0 = (tt / tpr) * TO, ox0 = (tt - (tt / tpr) * tpr) * TO;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;  // input tile origin (pad 1)
  const int H = a.H;
  const int l16 = lane & 15, lq = lane >> 4;

  // ---- per-block constants -> LDS (float4 copies; every count is a multiple of 4)
  for (int i = tid; i < HIDP * 9 / 4; i += 256)
    reinterpret_cast<float4*>(sWd)[i] = reinterpret_cast<const float4*>(a.Wd)[i];
  for (int i = tid; i < HIDP / 4; i += 256) {
    reinterpret_cast<float4*>(sBd)[i] = reinterpret_cast<const float4*>(a.bd)[i];
    if constexpr (EXPAND) reinterpret_cast<float4*>(sBe)[i] = reinterpret_cast<const float4*>(a.be)[i];
  }
  if (tid < COUTP / 4) reinterpret_cast<float4*>(sBp)[tid] = reinterpret_cast<const float4*>(a.bp)[tid];

  // expand weights of the first chunk (A fragments, rows = hidden channels)
  half8 af[2][KX];
  if constexpr (EXPAND) {
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
      for (int k = 0; k < KX; ++k)
        af[ht][k] = *reinterpret_cast<const half8*>(a.We + (size_t)(16 * ht + l16) * CINP + 32 * k + 8 * lq);
  }

  // ---- stage the block input tile: sX[p][c], zeros outside the image and past cin
  if constexpr (STEM == 0) {
    constexpr int C8 = CINP / 8;
    constexpr int NIT = (MP * C8 + 255) / 256;
    const f16* xin = a.x + (size_t)n * H * H * a.cin;
    half8 v[NIT];
#pragma unroll
    for (int j = 0; j < NIT; ++j) {  // all loads first ...
      const int i = tid + 256 * j;
      const int p = i / C8, c8 = i - (i / C8) * C8;
      const int py = p / IR, px = p - (p / IR) * IR;
      const int iy = iy0 + py, ix = ix0 + px;
      v[j] = half8{0, 0, 0, 0, 0, 0, 0, 0};
      if (i < MP * C8 && p < NP && iy >= 0 && iy < H && ix >= 0 && ix < H && c8 * 8 < a.cin)
        v[j] = *reinterpret_cast<const half8*>(xin + ((size_t)iy * H + ix) * a.cin + c8 * 8);
    }
#pragma unroll
    for (int j = 0; j < NIT; ++j) {  // ... then the LDS stores
      const int i = tid + 256 * j;
      const int p = i / C8, c8 = i - (i / C8) * C8;
      if (i < MP * C8) *reinterpret_cast<half8*>(sX + p * XLD + c8 * 8) = v[j];
    }
  } else {
    // stem conv 3x3/2 pad 1 on the u8 image for stem pixel (iy, ix) of the 112x112 grid:
    // the u8 patch and the folded weights go to LDS, then 8 channels per item in fp32.
    const uint8_t* img = reinterpret_cast<const uint8_t*>(a.x) + (size_t)n * 224 * 224 * STEM;
    const int ry0 = 2 * iy0 - 1, rx0 = 2 * ix0 - 1;
    for (int i = tid; i < PR * PR * STEM; i += 256) {
      const int c = i % STEM, pix = i / STEM;
      const int yy = ry0 + pix / PR, xx = rx0 + pix % PR;
      sPatch[i] = (yy >= 0 && yy < 224 && xx >= 0 && xx < 224) ? img[((size_t)yy * 224 + xx) * STEM + c] : 0;
    }
    for (int i = tid; i < STEM * 9 * 8; i += 256)
      reinterpret_cast<float4*>(sSW)[i] = reinterpret_cast<const float4*>(a.stem_w)[i];
    __syncthreads();
    for (int i = tid; i < MP * 4; i += 256) {
      const int p = i >> 2, cg = i & 3;
      const int py = p / IR, px = p - (p / IR) * IR;
      const int iy = iy0 + py, ix = ix0 + px;
      half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (p < NP && iy >= 0 && iy < 112 && ix >= 0 && ix < 112) {
        const int cls = (iy == 0 ? 2 : 0) + (ix == 0 ? 1 : 0);
        float acc[8];
        const float4 c0 = *reinterpret_cast<const float4*>(a.stem_corr + cls * 32 + cg * 8);
        const float4 c1 = *reinterpret_cast<const float4*>(a.stem_corr + cls * 32 + cg * 8 + 4);
        acc[0] = c0.x; acc[1] = c0.y; acc[2] = c0.z; acc[3] = c0.w;
        acc[4] = c1.x; acc[5] = c1.y; acc[6] = c1.z; acc[7] = c1.w;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int c = 0; c < STEM; ++c) {
              const float u = (float)sPatch[((2 * py + ky) * PR + 2 * px + kx) * STEM + c];
              const float* w = sSW + ((c * 3 + ky) * 3 + kx) * 32 + cg * 8;
              const float4 w0 = *reinterpret_cast<const float4*>(w);
              const float4 w1 = *reinterpret_cast<const float4*>(w + 4);
              acc[0] = __builtin_fmaf(u, w0.x, acc[0]); acc[1] = __builtin_fmaf(u, w0.y, acc[1]);
              acc[2] = __builtin_fmaf(u, w0.z, acc[2]); acc[3] = __builtin_fmaf(u, w0.w, acc[3]);
              acc[4] = __builtin_fmaf(u, w1.x, acc[4]); acc[5] = __builtin_fmaf(u, w1.y, acc[5]);
              acc[6] = __builtin_fmaf(u, w1.z, acc[6]); acc[7] = __builtin_fmaf(u, w1.w, acc[7]);
            }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (f16)relu6f(acc[j]);
      }
      *reinterpret_cast<half8*>(sX + p * XLD + cg * 8) = v;
    }
  }
  __syncthreads();

  floatx4 acc[OT];
#pragma unroll
  for (int o = 0; o < OT; ++o) acc[o] = floatx4{0.f, 0.f, 0.f, 0.f};

  // dw item of this thread: output pixel q, channels 8*cg .. 8*cg+7 of the chunk
  const int dq = tid >> 2, dcg = tid & 3;
  const int dqy = dq / TO, dqx = dq - (dq / TO) * TO;
  const int dp0 = (dqy * S) * IR + dqx * S;  // top-left tap of the 3x3 window

#pragma unroll 1
  for (int h0 = 0; h0 < HIDP; h0 += MB_HC) {
    // project weights of this chunk: in flight during expand + depthwise
    half8 pf[OT];
#pragma unroll
    for (int o = 0; o < OT; ++o)
      pf[o] = *reinterpret_cast<const half8*>(a.Wp + (size_t)(16 * o + l16) * HIDP + h0 + 8 * lq);
    const f16* src;  // dw input for this chunk: row p at src + p * sld
    int sld;
    if constexpr (EXPAND) {
      // E^T[h][p] = sum_c We[h0+h][c] X[p][c]: A = weights (rows h), B = X^T (cols p), so
      // each lane ends with 4 consecutive hidden channels of one pixel (one 8-B LDS write).
      float eb[2][4];
#pragma unroll
      for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int e = 0; e < 4; ++e) eb[ht][e] = sBe[h0 + 16 * ht + 4 * lq + e];
      for (int pt = wave; pt < MP / 16; pt += 4) {
        const int p = pt * 16 + l16;
        const int py = p / IR, px = p - (p / IR) * IR;
        const int iy = iy0 + py, ix = ix0 + px;
        const bool valid = p < NP && iy >= 0 && iy < H && ix >= 0 && ix < H;
        floatx4 e2[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int k = 0; k < KX; ++k) {
          const half8 bf = *reinterpret_cast<const half8*>(sX + p * XLD + 32 * k + 8 * lq);
#pragma unroll
          for (int ht = 0; ht < 2; ++ht) e2[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[ht][k], bf, e2[ht], 0, 0, 0);
        }
#pragma unroll
        for (int ht = 0; ht < 2; ++ht) {
          half4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) hv[e] = valid ? (f16)relu6f(e2[ht][e] + eb[ht][e]) : (f16)0.f;  // dw zero pad
          *reinterpret_cast<half4*>(sE + p * ELD + 16 * ht + 4 * lq) = hv;
        }
      }
      if (h0 + MB_HC < HIDP) {  // next chunk's expand weights: in flight during dw + project
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
          for (int k = 0; k < KX; ++k)
            af[ht][k] = *reinterpret_cast<const half8*>(a.We + (size_t)(h0 + MB_HC + 16 * ht + l16) * CINP + 32 * k +
                                                        8 * lq);
      }
      __syncthreads();
      src = sE;
      sld = ELD;
    } else {
      src = sX + h0;
      sld = XLD;
    }

    // ---- depthwise 3x3/S + BN + ReLU6 (fp32) -> sD[q][h]
    {
      half8 out = {0, 0, 0, 0, 0, 0, 0, 0};
      if (dq < NQ) {
        const int hc = h0 + 8 * dcg;
        float d[8];
        {
          const float4 b0 = *reinterpret_cast<const float4*>(sBd + hc);
          const float4 b1 = *reinterpret_cast<const float4*>(sBd + hc + 4);
          d[0] = b0.x; d[1] = b0.y; d[2] = b0.z; d[3] = b0.w; d[4] = b1.x; d[5] = b1.y; d[6] = b1.z; d[7] = b1.w;
        }
        const float* wd = sWd + (hc / 8) * 72;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const half8 ev = *reinterpret_cast<const half8*>(src + (dp0 + ky * IR + kx) * sld + 8 * dcg);
            const float4 w0 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8);
            const float4 w1 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8 + 4);
            d[0] = __builtin_fmaf((float)ev[0], w0.x, d[0]); d[1] = __builtin_fmaf((float)ev[1], w0.y, d[1]);
            d[2] = __builtin_fmaf((float)ev[2], w0.z, d[2]); d[3] = __builtin_fmaf((float)ev[3], w0.w, d[3]);
            d[4] = __builtin_fmaf((float)ev[4], w1.x, d[4]); d[5] = __builtin_fmaf((float)ev[5], w1.y, d[5]);
            d[6] = __builtin_fmaf((float)ev[6], w1.z, d[6]); d[7] = __builtin_fmaf((float)ev[7], w1.w, d[7]);
          }
#pragma unroll
        for (int j = 0; j < 8; ++j) out[j] = (f16)relu6f(d[j]);
      }
      *reinterpret_cast<half8*>(sD + dq * ELD + 8 * dcg) = out;
    }
    __syncthreads();

    // ---- project: out^T[o][q] += Wp[o][h0..h0+31] . D[q][:]; wave w owns pixels 16w..16w+15
    {
      const half8 bf = *reinterpret_cast<const half8*>(sD + (16 * wave + l16) * ELD + 8 * lq);
#pragma unroll
      for (int o = 0; o < OT; ++o) acc[o] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf[o], bf, acc[o], 0, 0, 0);
    }
    if constexpr (!EXPAND) __syncthreads();  // next chunk's dw rewrites sD
  }

  // ---- epilogue: + BN shift (+ residual from the staged input), f16, staged for 16-B stores
  {
    const int q = 16 * wave + l16;
    const int qy = q / TO, qx = q - (q / TO) * TO;
    const int pc = (qy * S + 1) * IR + qx * S + 1;  // centre tap = the same pixel when S == 1
#pragma unroll
    for (int o = 0; o < OT; ++o) {
      const int c = 16 * o + 4 * lq;
      const float4 bv = *reinterpret_cast<const float4*>(sBp + c);
      float v[4] = {acc[o][0] + bv.x, acc[o][1] + bv.y, acc[o][2] + bv.z, acc[o][3] + bv.w};
      if constexpr (RES) {
        if (q < NQ) {
          const half4 r = *reinterpret_cast<const half4*>(sX + pc * XLD + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        }
      }
      half4 hv;
#pragma unroll
      for (int e = 0; e < 4; ++e) hv[e] = (f16)v[e];
      *reinterpret_cast<half4*>(sO + q * OLD + c) = hv;
    }
  }
  __syncthreads();
  {
    const int C8 = a.cout / 8;
    f16* yout = a.y + (size_t)n * a.OH * a.OH * a.cout;
    for (int i = tid; i < NQ * C8; i += 256) {
      const int q = i / C8, c8 = i - (i / C8) * C8;
      const int qy = q / TO, qx = q - (q / TO) * TO;
      *reinterpret_cast<half8*>(yout + ((size_t)(oy0 + qy) * a.OH + ox0 + qx) * a.cout + c8 * 8) =
          *reinterpret_cast<const half8*>(sO + q * OLD + c8 * 8);
    }
  }
}

// ----------------------------------------------------------------------------- wave-autonomous form
// The same block arithmetic (same k orders, same roundings: bit-identical outputs), organised
// so that no workgroup barrier sits inside the tile loop. Every WAVE is an independent worker
// on 4x4 output tiles (16 pixels = one MFMA q-tile) with its own LDS slices for the input
// tile (+ halo), the expanded chunk, the depthwise output and the output staging; the four
// waves of a workgroup only share the block constants (depthwise weights and biases), staged
// once. A wave's LDS writes are read back by the same wave (DS operations of one wave execute
// in order), so the hidden-channel chunks run back to back, and the waves of a CU interleave
// freely: the latency one wave exposes (HBM, weight fragments, LDS) is covered by the others.
// The 4x4 tile recomputes more halo in the expand (6x6 inputs per 16 outputs at stride 1)
// than an 8x8 tile; that is MFMA work, cheap next to the latency it removes.
constexpr int MBW_TO = 4;

template <int S, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM>
struct MbwGeom {
  static constexpr int IR = (MBW_TO - 1) * S + 3;   // input tile side (with halo): 6 or 9
  static constexpr int NP = IR * IR, MP = (NP + 15) / 16 * 16;
  static constexpr int XLD = CINP + 8, ELD = MB_HC + 8, OLD = COUTP + 8;
  static constexpr int W_X = MP * XLD;
  static constexpr int W_E = EXPAND ? MP * ELD : 0;
  static constexpr int W_D = 16 * ELD;
  // output staging: its own slice when the input tile must survive for the residual,
  // else it reuses the input tile's slice (free after the last chunk's expand)
  static constexpr int W_O = (RES || 16 * OLD > W_X) ? 16 * OLD : 0;
  static constexpr int W_TOT = W_X + W_E + W_D + W_O;  // halfs per wave (all multiples of 8)
  static constexpr bool DW_LDS = HIDP * 9 * 4 <= 16384;  // depthwise weights staged in LDS
  static constexpr int PR = 2 * IR + 1;                  // stem: u8 patch side
};

template <int S, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM>
__global__ __launch_bounds__(256) void mbv2_wave_kernel(const MbArgs a, int ntiles) {
  using G = MbwGeom<S, CINP, HIDP, COUTP, EXPAND, RES, STEM>;
  constexpr int TO = MBW_TO, IR = G::IR, NP = G::NP, MP = G::MP;
  constexpr int XLD = G::XLD, ELD = G::ELD, OLD = G::OLD;
  constexpr int OT = COUTP / 16, KX = CINP / 32;
  static_assert(!STEM || (CINP == 32 && HIDP == 32 && !EXPAND && S == 1), "stem fuses into block 1 only");
  __shared__ __attribute__((aligned(16))) f16 sw[4 * G::W_TOT];
  __shared__ __attribute__((aligned(16))) float sWd[G::DW_LDS ? HIDP * 9 : 4];
  __shared__ __attribute__((aligned(16))) float sBd[HIDP];
  __shared__ __attribute__((aligned(16))) float sBe[EXPAND ? HIDP : 4];
  __shared__ __attribute__((aligned(16))) float sBp[COUTP];
  __shared__ __attribute__((aligned(16))) float sSW[STEM ? STEM * 9 * 32 : 4];
  __shared__ uint8_t sPatch[STEM ? 4 * G::PR * G::PR * STEM : 4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  f16* sX = sw + wave * G::W_TOT;
  f16* sE = sX + G::W_X;
  f16* sD = sE + G::W_E;
  f16* sO = G::W_O ? sD + G::W_D : sX;

  if constexpr (G::DW_LDS)
    for (int i = tid; i < HIDP * 9 / 4; i += 256)
      reinterpret_cast<float4*>(sWd)[i] = reinterpret_cast<const float4*>(a.Wd)[i];
  for (int i = tid; i < HIDP / 4; i += 256) {
    reinterpret_cast<float4*>(sBd)[i] = reinterpret_cast<const float4*>(a.bd)[i];
    if constexpr (EXPAND) reinterpret_cast<float4*>(sBe)[i] = reinterpret_cast<const float4*>(a.be)[i];
  }
  if (tid < COUTP / 4) reinterpret_cast<float4*>(sBp)[tid] = reinterpret_cast<const float4*>(a.bp)[tid];
  if constexpr (STEM != 0)
    for (int i = tid; i < STEM * 9 * 8; i += 256)
      reinterpret_cast<float4*>(sSW)[i] = reinterpret_cast<const float4*>(a.stem_w)[i];
  __syncthreads();  // the only workgroup barrier

  const int H = a.H, OH = a.OH;
  const int tpr = (OH + TO - 1) / TO, tpi = tpr * tpr;
  const float* wdsrc = G::DW_LDS ? sWd : a.Wd;
  // depthwise item of this lane: output pixel dq of the tile, channels 8 dcg .. 8 dcg + 7
  const int dq = lane >> 2, dcg = lane & 3;
  const int dp0 = ((dq >> 2) * S) * IR + (dq & 3) * S;

#pragma unroll 1
  for (int tile = blockIdx.x * 4 + wave; tile < ntiles; tile += gridDim.x * 4) {
    const int n = tile / tpi, tt = tile - n * tpi;
    const int oy0 = (tt / tpr) * TO, ox0 = (tt - (tt / tpr) * tpr) * TO;
    const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

    // ---- stage the input tile (zeros outside the image and past cin)
    if constexpr (STEM == 0) {
      constexpr int C8 = CINP / 8;
      constexpr int NIT = (MP * C8 + 63) / 64;
      static_assert(NIT <= 32, "validity bits");
      const f16* xin = a.x + (size_t)n * H * H * a.cin;
      half8 v[NIT];
      uint32_t ok = 0;
#pragma unroll
      for (int j = 0; j < NIT; ++j) {  // unconditional clamped loads, zeroed at the LDS write
        const int i = lane + 64 * j;
        const int p = min(i / C8, NP - 1), c8 = i - (i / C8) * C8;
        const int iy = iy0 + p / IR, ix = ix0 + p % IR;
        const bool in = i < NP * C8 && iy >= 0 && iy < H && ix >= 0 && ix < H && c8 * 8 < a.cin;
        ok |= (uint32_t)in << j;
        const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), H - 1);
        const int cc = min(c8 * 8, a.cin - 8);
        v[j] = *reinterpret_cast<const half8*>(xin + ((size_t)cy * H + cx) * a.cin + cc);
      }
#pragma unroll
      for (int j = 0; j < NIT; ++j) {
        const int i = lane + 64 * j;
        const half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i < MP * C8) *reinterpret_cast<half8*>(sX + (i / C8) * XLD + (i % C8) * 8) = ((ok >> j) & 1) ? v[j] : z;
      }
    } else {
      constexpr int PR = G::PR;
      uint8_t* patch = sPatch + wave * PR * PR * STEM;
      const uint8_t* img = reinterpret_cast<const uint8_t*>(a.x) + (size_t)n * 224 * 224 * STEM;
      const int ry0 = 2 * iy0 - 1, rx0 = 2 * ix0 - 1;
      for (int i = lane; i < PR * PR * STEM; i += 64) {
        const int c = i % STEM, pix = i / STEM;
        const int yy = ry0 + pix / PR, xx = rx0 + pix % PR;
        const int cy = min(max(yy, 0), 223), cx = min(max(xx, 0), 223);
        const uint8_t u = img[((size_t)cy * 224 + cx) * STEM + c];
        patch[i] = (yy >= 0 && yy < 224 && xx >= 0 && xx < 224) ? u : 0;
      }
      for (int i = lane; i < MP * 4; i += 64) {
        const int p = i >> 2, cg = i & 3;
        const int py = p / IR, px = p - (p / IR) * IR;
        const int iy = iy0 + py, ix = ix0 + px;
        half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (p < NP && iy >= 0 && iy < 112 && ix >= 0 && ix < 112) {
          const int cls = (iy == 0 ? 2 : 0) + (ix == 0 ? 1 : 0);
          float acc[8];
          const float4 c0 = *reinterpret_cast<const float4*>(a.stem_corr + cls * 32 + cg * 8);
          const float4 c1 = *reinterpret_cast<const float4*>(a.stem_corr + cls * 32 + cg * 8 + 4);
          acc[0] = c0.x; acc[1] = c0.y; acc[2] = c0.z; acc[3] = c0.w;
          acc[4] = c1.x; acc[5] = c1.y; acc[6] = c1.z; acc[7] = c1.w;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx)
#pragma unroll
              for (int c = 0; c < STEM; ++c) {
                const float u = (float)patch[((2 * py + ky) * PR + 2 * px + kx) * STEM + c];
                const float* w = sSW + ((c * 3 + ky) * 3 + kx) * 32 + cg * 8;
                const float4 w0 = *reinterpret_cast<const float4*>(w);
                const float4 w1 = *reinterpret_cast<const float4*>(w + 4);
                acc[0] = __builtin_fmaf(u, w0.x, acc[0]); acc[1] = __builtin_fmaf(u, w0.y, acc[1]);
                acc[2] = __builtin_fmaf(u, w0.z, acc[2]); acc[3] = __builtin_fmaf(u, w0.w, acc[3]);
                acc[4] = __builtin_fmaf(u, w1.x, acc[4]); acc[5] = __builtin_fmaf(u, w1.y, acc[5]);
                acc[6] = __builtin_fmaf(u, w1.z, acc[6]); acc[7] = __builtin_fmaf(u, w1.w, acc[7]);
              }
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (f16)relu6f(acc[j]);
        }
        *reinterpret_cast<half8*>(sX + p * XLD + cg * 8) = v;
      }
    }

    floatx4 acc[OT];
#pragma unroll
    for (int o = 0; o < OT; ++o) acc[o] = floatx4{0.f, 0.f, 0.f, 0.f};

    // Weight fragments of a hidden-channel chunk: expand (af) and project (pf). With two
    // register sets (PF2) the next chunk's fragments are in flight while this chunk computes.
    constexpr bool PF2 = OT + (EXPAND ? 2 * KX : 0) <= 6;  // larger sets cost occupancy (measured)
    auto loadw = [&](int h0, half8 (&af)[2][KX], half8 (&pf)[OT]) {
#pragma unroll
      for (int o = 0; o < OT; ++o)
        pf[o] = *reinterpret_cast<const half8*>(a.Wp + (size_t)(16 * o + l16) * HIDP + h0 + 8 * lq);
      if constexpr (EXPAND) {
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
          for (int k = 0; k < KX; ++k)
            af[ht][k] = *reinterpret_cast<const half8*>(a.We + (size_t)(h0 + 16 * ht + l16) * CINP + 32 * k + 8 * lq);
      }
    };
    auto chunk = [&](int h0, const half8 (&af)[2][KX], const half8 (&pf)[OT]) {
      const f16* src;
      int sld;
      if constexpr (EXPAND) {
        float eb[2][4];
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
          for (int e = 0; e < 4; ++e) eb[ht][e] = sBe[h0 + 16 * ht + 4 * lq + e];
#pragma unroll
        for (int pt = 0; pt < MP / 16; ++pt) {
          const int p = pt * 16 + l16;
          const int iy = iy0 + p / IR, ix = ix0 + p % IR;
          const bool valid = p < NP && iy >= 0 && iy < H && ix >= 0 && ix < H;
          floatx4 e2[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
          for (int k = 0; k < KX; ++k) {
            const half8 bf = *reinterpret_cast<const half8*>(sX + p * XLD + 32 * k + 8 * lq);
#pragma unroll
            for (int ht = 0; ht < 2; ++ht)
              e2[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[ht][k], bf, e2[ht], 0, 0, 0);
          }
#pragma unroll
          for (int ht = 0; ht < 2; ++ht) {
            half4 hv;
#pragma unroll
            for (int e = 0; e < 4; ++e) hv[e] = valid ? (f16)relu6f(e2[ht][e] + eb[ht][e]) : (f16)0.f;
            *reinterpret_cast<half4*>(sE + p * ELD + 16 * ht + 4 * lq) = hv;
          }
        }
        src = sE;
        sld = ELD;
      } else {
        src = sX + h0;
        sld = XLD;
      }
      // ---- depthwise 3x3/S + BN + ReLU6 (fp32): 16 pixels x 32 channels, 8 per lane
      {
        const int hc = h0 + 8 * dcg;
        float d[8];
        {
          const float4 b0 = *reinterpret_cast<const float4*>(sBd + hc);
          const float4 b1 = *reinterpret_cast<const float4*>(sBd + hc + 4);
          d[0] = b0.x; d[1] = b0.y; d[2] = b0.z; d[3] = b0.w; d[4] = b1.x; d[5] = b1.y; d[6] = b1.z; d[7] = b1.w;
        }
        const float* wd = wdsrc + (size_t)(hc / 8) * 72;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const half8 ev = *reinterpret_cast<const half8*>(src + (dp0 + ky * IR + kx) * sld + 8 * dcg);
            const float4 w0 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8);
            const float4 w1 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8 + 4);
            d[0] = __builtin_fmaf((float)ev[0], w0.x, d[0]); d[1] = __builtin_fmaf((float)ev[1], w0.y, d[1]);
            d[2] = __builtin_fmaf((float)ev[2], w0.z, d[2]); d[3] = __builtin_fmaf((float)ev[3], w0.w, d[3]);
            d[4] = __builtin_fmaf((float)ev[4], w1.x, d[4]); d[5] = __builtin_fmaf((float)ev[5], w1.y, d[5]);
            d[6] = __builtin_fmaf((float)ev[6], w1.z, d[6]); d[7] = __builtin_fmaf((float)ev[7], w1.w, d[7]);
          }
        half8 out;
#pragma unroll
        for (int j = 0; j < 8; ++j) out[j] = (f16)relu6f(d[j]);
        *reinterpret_cast<half8*>(sD + dq * ELD + 8 * dcg) = out;
      }
      // ---- project: out^T[o][q] += Wp[o][h0 .. h0+31] . D[q][:]
      {
        const half8 bf = *reinterpret_cast<const half8*>(sD + l16 * ELD + 8 * lq);
#pragma unroll
        for (int o = 0; o < OT; ++o) acc[o] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf[o], bf, acc[o], 0, 0, 0);
      }
    };
    half8 afA[2][KX], pfA[OT];
    if constexpr (PF2) {
      half8 afB[2][KX], pfB[OT];
      loadw(0, afA, pfA);
#pragma unroll 1
      for (int h0 = 0; h0 < HIDP; h0 += 2 * MB_HC) {
        if (h0 + MB_HC < HIDP) loadw(h0 + MB_HC, afB, pfB);
        chunk(h0, afA, pfA);
        if (h0 + MB_HC >= HIDP) break;
        if (h0 + 2 * MB_HC < HIDP) loadw(h0 + 2 * MB_HC, afA, pfA);
        chunk(h0 + MB_HC, afB, pfB);
      }
    } else {
#pragma unroll 1
      for (int h0 = 0; h0 < HIDP; h0 += MB_HC) {
        loadw(h0, afA, pfA);
        chunk(h0, afA, pfA);
      }
    }

    // ---- epilogue: + BN shift (+ residual from the staged input tile) -> f16 -> 16-B row stores
    {
      const int q = l16;
      const int pc = ((q >> 2) * S + 1) * IR + (q & 3) * S + 1;
      half4 hv[OT];
#pragma unroll
      for (int o = 0; o < OT; ++o) {  // all residual reads before any staging write (sO may alias sX)
        const int c = 16 * o + 4 * lq;
        const float4 bv = *reinterpret_cast<const float4*>(sBp + c);
        float v[4] = {acc[o][0] + bv.x, acc[o][1] + bv.y, acc[o][2] + bv.z, acc[o][3] + bv.w};
        if constexpr (RES) {
          const half4 r = *reinterpret_cast<const half4*>(sX + pc * XLD + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) hv[o][e] = (f16)v[e];
      }
#pragma unroll
      for (int o = 0; o < OT; ++o) *reinterpret_cast<half4*>(sO + q * OLD + 16 * o + 4 * lq) = hv[o];
      const int C8 = a.cout / 8;
      f16* yout = a.y + (size_t)n * OH * OH * a.cout;
      for (int i = lane; i < 16 * C8; i += 64) {
        const int qq = i / C8, c8 = i - (i / C8) * C8;
        const int oy = oy0 + (qq >> 2), ox = ox0 + (qq & 3);
        if (oy < OH && ox < OH)
          *reinterpret_cast<half8*>(yout + ((size_t)oy * OH + ox) * a.cout + c8 * 8) =
              *reinterpret_cast<const half8*>(sO + qq * OLD + c8 * 8);
      }
    }
  }
}

// ----------------------------------------------------------------------------- model

static int pad_to(int v, int m) { return (v + m - 1) / m * m; }

int MobileNetModel::create(const float* blob, size_t n) {
  if (prec == PREC_FP32) return create_f32(blob, n);  // mobilenet_f32.hip
  if (prec == PREC_FP32X3) return create_x3(blob, n);  // mobilenet_x3.hip
  BlobReader rd(blob, n);
  std::vector<f16> w;
  std::vector<float> pr;
  auto align4 = [&]() { while (pr.size() % 4) pr.push_back(0.f); };  // 16-B aligned float4 reads
  auto bn_scale_shift = [&](int c, std::vector<double>& scale, std::vector<double>& shift) {
    const float* g = rd.take(c);
    const float* b = rd.take(c);
    const float* rm = rd.take(c);
    const float* rv = rd.take(c);
    scale.assign(c, 0.0);
    shift.assign(c, 0.0);
    if (!rd.ok) return;
    for (int i = 0; i < c; ++i) {
      scale[i] = (double)g[i] / std::sqrt((double)rv[i] + 1e-5);
      shift[i] = (double)b[i] - (double)rm[i] * scale[i];
    }
  };
  std::vector<double> sc, sh;
  // ---- stem features[0]: conv 3x3/2 (3 -> 32) + BN + ReLU6. ToTensor (/255) and Normalize
  // fold into per-pixel weights; the -mean/std term of the in-image taps becomes a bias per
  // border class (stem row 0 / col 0 lose their top / left taps; 224 = 2*112 so the bottom /
  // right taps are always inside).
  {
    const float* src = rd.take((size_t)32 * 3 * 9);
    bn_scale_shift(32, sc, sh);
    align4();
    stem_w_off = pr.size();
    pr.resize(pr.size() + 9 * 32, 0.f);
    stem_rgb_off = pr.size();
    pr.resize(pr.size() + 27 * 32, 0.f);
    stem_corr_off = pr.size();
    pr.resize(pr.size() + 4 * 32, 0.f);
    const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
    if (rd.ok) {
      for (int o = 0; o < 32; ++o) {
        double cterm[9] = {};
        for (int t = 0; t < 9; ++t) {
          double gsum = 0.0;
          for (int c = 0; c < 3; ++c) {
            const double wv = src[((size_t)o * 3 + c) * 9 + t];
            const double mf = (double)(float)mean[c], sf = (double)(float)stdv[c];
            gsum += wv / (255.0 * sf);
            cterm[t] -= wv * mf / sf;
            pr[stem_rgb_off + (size_t)(c * 9 + t) * 32 + o] = (float)(wv / (255.0 * sf) * sc[o]);
          }
          pr[stem_w_off + (size_t)t * 32 + o] = (float)(gsum * sc[o]);
        }
        for (int cls = 0; cls < 4; ++cls) {  // cls = 2 * (row 0) + (col 0)
          double sum = sh[o];
          for (int t = 0; t < 9; ++t) {
            const int ky = t / 3, kx = t % 3;
            if (((cls & 2) && ky == 0) || ((cls & 1) && kx == 0)) continue;
            sum += cterm[t] * sc[o];
          }
          pr[stem_corr_off + (size_t)cls * 32 + o] = (float)sum;
        }
      }
    }
  }
  // ---- inverted-residual blocks features[1..17]
  static const int kSet[7][4] = {{1, 16, 1, 1}, {6, 24, 2, 2}, {6, 32, 3, 2}, {6, 64, 4, 2},
                                 {6, 96, 3, 1}, {6, 160, 3, 2}, {6, 320, 1, 1}};
  blocks.clear();
  int cin = 32, prev_lcoutp = 32;
  for (int si = 0; si < 7; ++si)
    for (int r = 0; r < kSet[si][2]; ++r) {
      MbBlock b;
      b.t = kSet[si][0]; b.cin = cin; b.hid = cin * b.t; b.cout = kSet[si][1]; b.stride = r == 0 ? kSet[si][3] : 1;
      b.cinp = pad_to(cin, 32); b.hidp = pad_to(b.hid, 32); b.coutp = pad_to(b.cout, 16);
      if (b.t != 1) {  // expand 1x1 + BN (+ ReLU6)
        const float* we = rd.take((size_t)b.hid * cin);
        bn_scale_shift(b.hid, sc, sh);
        b.we_off = w.size();
        w.resize(w.size() + (size_t)b.hidp * b.cinp, (f16)0.f);
        align4();
        b.be_off = pr.size();
        pr.resize(pr.size() + b.hidp, 0.f);
        if (rd.ok)
          for (int h = 0; h < b.hid; ++h) {
            for (int c = 0; c < cin; ++c) w[b.we_off + (size_t)h * b.cinp + c] = (f16)((double)we[(size_t)h * cin + c] * sc[h]);
            pr[b.be_off + h] = (float)sh[h];
          }
      }
      {  // depthwise 3x3 + BN (+ ReLU6): fp32 [hidp/8][9 taps][8 channels]
        const float* wd = rd.take((size_t)b.hid * 9);
        bn_scale_shift(b.hid, sc, sh);
        align4();
        b.wd_off = pr.size();
        pr.resize(pr.size() + (size_t)b.hidp * 9, 0.f);
        b.bd_off = pr.size();
        pr.resize(pr.size() + b.hidp, 0.f);
        if (rd.ok)
          for (int h = 0; h < b.hid; ++h) {
            for (int t = 0; t < 9; ++t)
              pr[b.wd_off + (size_t)(h / 8) * 72 + t * 8 + (h % 8)] = (float)((double)wd[(size_t)h * 9 + t] * sc[h]);
            pr[b.bd_off + h] = (float)sh[h];
          }
      }
      {  // project 1x1 + BN (linear bottleneck)
        const float* wp = rd.take((size_t)b.cout * b.hid);
        bn_scale_shift(b.cout, sc, sh);
        b.wp_off = w.size();
        w.resize(w.size() + (size_t)b.coutp * b.hidp, (f16)0.f);
        align4();
        b.bp_off = pr.size();
        pr.resize(pr.size() + b.coutp, 0.f);
        if (rd.ok)
          for (int o = 0; o < b.cout; ++o) {
            for (int h = 0; h < b.hid; ++h)
              w[b.wp_off + (size_t)o * b.hidp + h] = (f16)((double)wp[(size_t)o * b.hid + h] * sc[o]);
            pr[b.bp_off + o] = (float)sh[o];
          }
      }
      b.lcinp = prev_lcoutp;
      b.lcoutp = pad_to(b.cout, 64);
      prev_lcoutp = b.lcoutp;
      if (b.t != 1 && b.hidp % 64 == 0) {  // layered form: the same matrices, K / N padded with zeros
        b.lwe_off = w.size();
        w.resize(w.size() + (size_t)b.hidp * b.lcinp, (f16)0.f);
        for (int h = 0; h < b.hidp; ++h)
          for (int c = 0; c < b.cinp && c < b.lcinp; ++c)
            w[b.lwe_off + (size_t)h * b.lcinp + c] = w[b.we_off + (size_t)h * b.cinp + c];
        b.lwp_off = w.size();
        w.resize(w.size() + (size_t)b.lcoutp * b.hidp, (f16)0.f);
        std::copy(w.begin() + b.wp_off, w.begin() + b.wp_off + (size_t)b.coutp * b.hidp, w.begin() + b.lwp_off);
        align4();
        b.lbp_off = pr.size();
        pr.resize(pr.size() + b.lcoutp, 0.f);
        std::copy(pr.begin() + b.bp_off, pr.begin() + b.bp_off + b.coutp, pr.begin() + b.lbp_off);
      }
      blocks.push_back(b);
      cin = b.cout;
    }
  // ---- features[18]: 1x1 320 -> 1280 + BN + ReLU6 (GEMM engine)
  {
    const float* wl = rd.take((size_t)1280 * 320);
    bn_scale_shift(1280, sc, sh);
    last_w_off = w.size();
    w.resize(w.size() + (size_t)1280 * 320, (f16)0.f);
    align4();
    last_b_off = pr.size();
    pr.resize(pr.size() + 1280, 0.f);
    if (rd.ok)
      for (int o = 0; o < 1280; ++o) {
        for (int c = 0; c < 320; ++c) w[last_w_off + (size_t)o * 320 + c] = (f16)((double)wl[(size_t)o * 320 + c] * sc[o]);
        pr[last_b_off + o] = (float)sh[o];
      }
  }
  // ---- head: classifier[1] Linear(1280,512), classifier[4] Linear(512,7), fp32 [K][N]
  const float* f1w = rd.take((size_t)512 * 1280);
  const float* f1b = rd.take(512);
  const float* f2w = rd.take((size_t)7 * 512);
  const float* f2b = rd.take(7);
  MEC_REQUIRE(rd.ok && rd.off == n, "image_mbv2 blob size mismatch");
  align4();
  fc1_off = pr.size();
  pr.resize(pr.size() + (size_t)1280 * 512);
  for (int i = 0; i < 1280; ++i)
    for (int j = 0; j < 512; ++j) pr[fc1_off + (size_t)i * 512 + j] = f1w[(size_t)j * 1280 + i];
  fc1b_off = pr.size();
  pr.insert(pr.end(), f1b, f1b + 512);
  fc2_off = pr.size();
  pr.resize(pr.size() + 512 * 7);
  for (int i = 0; i < 512; ++i)
    for (int j = 0; j < 7; ++j) pr[fc2_off + (size_t)i * 7 + j] = f2w[(size_t)j * 512 + i];
  fc2b_off = pr.size();
  pr.insert(pr.end(), f2b, f2b + 7);
  MEC_TRY(upload(wts, w.data(), w.size() * sizeof(f16)));
  MEC_TRY(upload(prm, pr.data(), pr.size() * sizeof(float)));
  return 0;
}

// mec_set_option("mbv2_impl"): 1 = workgroup tiles, 2 = wave-autonomous tiles, 0 = per block
// shape, whichever ran faster at its first launch (hipEvents, median of 3; both forms are
// bit-identical, so the choice changes speed only). Measured at B=256: the wave form wins
// the stride-2 blocks and the mid-size stride-1 ones, the workgroup form the stem block and
// the wide late blocks (their depthwise weights no longer fit beside four waves' tiles).

template <int S, int TO, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM>
static int run_block(const MbArgs& a, int B, hipStream_t s, int impl) {
  if (impl == 2) {
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      MEC_HIP(hipGetDevice(&dev));
      MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int tpr = (a.OH + MBW_TO - 1) / MBW_TO;
    const int ntiles = B * tpr * tpr;
    const int grid = std::min((ntiles + 3) / 4, 8 * ncu);  // waves loop over the remaining tiles
    hipLaunchKernelGGL((mbv2_wave_kernel<S, CINP, HIDP, COUTP, EXPAND, RES, STEM>), dim3(grid), dim3(256), 0, s, a,
                       ntiles);
  } else {
    const int tpr = a.OH / TO;
    hipLaunchKernelGGL((mbv2_block_kernel<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM>), dim3(B * tpr * tpr),
                       dim3(256), 0, s, a);
  }
  MEC_LAUNCH_CHECK();
  return 0;
}

template <int S, int TO, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM>
static int launch_block(const MbArgs& a, int B, hipStream_t s) {
  // per block shape, once tuned (engine 2 of the handle's tune cache)
  const std::array<int, 11> key = {2, S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, 0, 0};
  int choice = tune_cache().find(key);
  int impl = opt().mbv2_impl;
  if (impl == 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (!choice && hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
      constexpr int REPS = 3;
      hipEvent_t ev[REPS + 1];
      for (auto& e : ev) MEC_HIP(hipEventCreate(&e));
      float best = 1e30f;
      for (int cand = 1; cand <= 2; ++cand) {
        MEC_TRY((run_block<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM>(a, B, s, cand)));  // warm
        MEC_HIP(hipEventRecord(ev[0], s));
        for (int r = 0; r < REPS; ++r) {
          MEC_TRY((run_block<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM>(a, B, s, cand)));
          MEC_HIP(hipEventRecord(ev[r + 1], s));
        }
        MEC_HIP(hipEventSynchronize(ev[REPS]));
        float t[REPS];
        for (int r = 0; r < REPS; ++r) MEC_HIP(hipEventElapsedTime(&t[r], ev[r], ev[r + 1]));
        std::sort(t, t + REPS);
        if (t[REPS / 2] < best) { best = t[REPS / 2]; choice = cand; }
      }
      for (auto& e : ev) (void)hipEventDestroy(e);
      tune_cache().put(key, choice);
    }
    impl = choice ? choice : 1;
  }
  return run_block<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM>(a, B, s, impl);
}

// The 17 block shapes of mobilenet_v2 (width 1.0) at 224x224: (stride, tile, cinp, hidp,
// coutp, expand, residual). Output sides 112 / 56 use 8x8 tiles, 28 / 14 / 7 use 7x7 tiles.
static int dispatch_block(const MbBlock& b, const MbArgs& a, int B, int stem_c, hipStream_t s) {
  const bool res = b.stride == 1 && b.cin == b.cout;
  const int TO = (a.OH % 8 == 0) ? 8 : 7;
#define MB_CASE(S_, TO_, CI_, HI_, CO_, EX_, RS_)                                                     \
  if (b.stride == S_ && TO == TO_ && b.cinp == CI_ && b.hidp == HI_ && b.coutp == CO_ && (b.t != 1) == EX_ && \
      res == RS_)                                                                                             \
    return launch_block<S_, TO_, CI_, HI_, CO_, EX_, RS_, 0>(a, B, s);
  if (b.t == 1) {
    MEC_REQUIRE(b.stride == 1 && b.cinp == 32 && b.hidp == 32 && b.coutp == 16 && !res && TO == 8, "mbv2: block 1 shape");
    if (stem_c == 3) return launch_block<1, 8, 32, 32, 16, false, false, 3>(a, B, s);
    if (stem_c == 1) return launch_block<1, 8, 32, 32, 16, false, false, 1>(a, B, s);
    return launch_block<1, 8, 32, 32, 16, false, false, 0>(a, B, s);
  }
  MB_CASE(2, 8, 32, 96, 32, true, false)     // 16 -> 24, 112 -> 56
  MB_CASE(1, 8, 32, 160, 32, true, true)      // 24 -> 24 @ 56
  MB_CASE(2, 7, 32, 160, 32, true, false)     // 24 -> 32, 56 -> 28
  MB_CASE(1, 7, 32, 192, 32, true, true)      // 32 -> 32 @ 28
  MB_CASE(2, 7, 32, 192, 64, true, false)     // 32 -> 64, 28 -> 14
  MB_CASE(1, 7, 64, 384, 64, true, true)      // 64 -> 64 @ 14
  MB_CASE(1, 7, 64, 384, 96, true, false)     // 64 -> 96 @ 14
  MB_CASE(1, 7, 96, 576, 96, true, true)      // 96 -> 96 @ 14
  MB_CASE(2, 7, 96, 576, 160, true, false)    // 96 -> 160, 14 -> 7
  MB_CASE(1, 7, 160, 960, 160, true, true)    // 160 -> 160 @ 7
  MB_CASE(1, 7, 160, 960, 320, true, false)   // 160 -> 320 @ 7
#undef MB_CASE
  set_error("mbv2: no kernel instance for this block shape");
  return -1;
}

// Layered tail of the f16 path (mbv2_layered16 k: features[k..17] as expand GEMM -> depthwise -> project
// GEMM; the fused blocks' arithmetic with the GEMM engine's k order). Depthwise 3x3/S (pad 1) + BN shift +
// ReLU6: E f16 NHWC [B,H,H,C] -> D f16 NHWC [B,OH,OH,C], fp32 FMAs from the shift in torch's (kh, kw) tap
// order. A thread owns one output row of one 8-channel group, its 72 tap weights and a 3 x 3 window of
// input pixels in registers (mobilenet_x3.hip's mbv2_dw_x3_kernel on f16 data).
template <int S>
__global__ __launch_bounds__(256) void mbv2_dw_f16_kernel(const f16* __restrict__ E, int H, int OH, int C,
                                                          const float* __restrict__ Wd, const float* __restrict__ bd,
                                                          f16* __restrict__ D, size_t items) {
  const size_t it = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (it >= items) return;
  const int G = C / 8;
  const size_t row = it / G;  // (image, output row)
  const int g = (int)(it - row * G);
  const size_t n = row / OH;
  const int oy = (int)(row - n * OH);
  float w[9][8], bias[8];
  {
    const float* wd = Wd + (size_t)g * 72;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 w0 = *reinterpret_cast<const float4*>(wd + t * 8);
      const float4 w1 = *reinterpret_cast<const float4*>(wd + t * 8 + 4);
      w[t][0] = w0.x; w[t][1] = w0.y; w[t][2] = w0.z; w[t][3] = w0.w;
      w[t][4] = w1.x; w[t][5] = w1.y; w[t][6] = w1.z; w[t][7] = w1.w;
    }
    const float4 b0 = *reinterpret_cast<const float4*>(bd + 8 * g);
    const float4 b1 = *reinterpret_cast<const float4*>(bd + 8 * g + 4);
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w;
    bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
  }
  bool rok[3];
  const f16* rp[3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * S - 1 + ky;
    rok[ky] = iy >= 0 && iy < H;
    rp[ky] = E + ((n * H + (rok[ky] ? iy : 0)) * H) * C + 8 * g;
  }
  auto load_col = [&](int ix, half8 (&e)[3], bool& ok) {
    ok = ix >= 0 && ix < H;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
      e[ky] = (ok && rok[ky]) ? *reinterpret_cast<const half8*>(rp[ky] + (size_t)ix * C) : half8{0, 0, 0, 0, 0, 0, 0, 0};
  };
  half8 win[3][3];  // [kx][ky]: input columns ox S - 1 + kx
  bool cok[3];
  load_col(-1, win[0], cok[0]);
  load_col(0, win[1], cok[1]);
  f16* dst = D + (row * OH) * C + 8 * g;
  for (int ox = 0; ox < OH; ++ox) {
    if (S == 1) {
      load_col(ox + 1, win[2], cok[2]);
    } else {
      load_col(2 * ox, win[1], cok[1]);
      load_col(2 * ox + 1, win[2], cok[2]);
    }
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = bias[j];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      if (!rok[ky]) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        if (!cok[kx]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = __builtin_fmaf((float)win[kx][ky][j], w[ky * 3 + kx][j], d[j]);
      }
    }
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (f16)relu6f(d[j]);
    *reinterpret_cast<half8*>(dst + (size_t)ox * C) = o;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      win[0][ky] = S == 1 ? win[1][ky] : win[2][ky];
      if (S == 1) win[1][ky] = win[2][ky];
    }
    cok[0] = S == 1 ? cok[1] : cok[2];
    if (S == 1) cok[1] = cok[2];
  }
}

// f16 [rows][cin] -> [rows][ld], channels cin .. ld-1 zero (the first layered block's input rows)
__global__ __launch_bounds__(256) void mbv2_pad_f16_kernel(const f16* __restrict__ x, size_t rows, int cin, int ld,
                                                           f16* __restrict__ y) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // one 8-channel group of one row
  const int G = ld / 8;
  if (i >= rows * G) return;
  const size_t r = i / G;
  const int c = (int)(i - r * G) * 8;
  *reinterpret_cast<half8*>(y + r * ld + c) =
      c < cin ? *reinterpret_cast<const half8*>(x + r * cin + c) : half8{0, 0, 0, 0, 0, 0, 0, 0};
}

int MobileNetModel::forward_u8(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits,
                               float* probs, hipStream_t s) {
  MEC_REQUIRE(B >= 0, "image: B < 0");
  if (B == 0) return 0;
  MEC_REQUIRE(img && feat && logits && probs, "image: null pointer");
  const bool fer = (H == 48 && W == 48 && C == 1);
  MEC_REQUIRE(fer || (H == 224 && W == 224 && (C == 1 || C == 3)),
              "image: input must be u8 [B,48,48,1] (GPU resize) or [B,224,224,{1,3}] (already resized)");
  if (prec == PREC_FP32) return forward_f32(img, B, H, W, C, feat, logits, probs, s);
  if (prec == PREC_FP32X3) return forward_x3(img, B, H, W, C, feat, logits, probs, s);
  // layered tail: blocks[l0 ..] (features[l0 + 1 ..]) as expand GEMM -> depthwise -> project GEMM
  size_t l0 = blocks.size();
  if (opt().mbv2_layered16) {
    l0 = (size_t)opt().mbv2_layered16 - 1;
    for (size_t i = l0; i < blocks.size(); ++i)
      MEC_REQUIRE(blocks[i].lwe_off, "mbv2: mbv2_layered16 names a block without a layered form");
  }
  size_t pe = 0, pd = 0, pp = 0;  // per-image elements of E, D and the tail's block I/O rows
  {
    int hh = 112;
    for (size_t i = 0; i < blocks.size(); ++i) {
      const MbBlock& b = blocks[i];
      const int oh = b.stride == 2 ? hh / 2 : hh;
      if (i >= l0) {
        pe = std::max(pe, (size_t)hh * hh * b.hidp);
        pd = std::max(pd, (size_t)oh * oh * b.hidp);
        pp = std::max(pp, std::max((size_t)hh * hh * b.lcinp, (size_t)oh * oh * b.lcoutp));
      }
      hh = oh;
    }
  }
  const size_t per_big = (size_t)112 * 112 * 16;  // largest block output (features[1]), elements
  const size_t per_last = (size_t)49 * 1280;
  const size_t per_img =
      224 * 224 + (2 * per_big + per_last + pe + pd + 2 * pp) * sizeof(f16) + 1280 * sizeof(float) + 64;
  if (ws.bytes < per_img * (size_t)B + 4096) MEC_TRY(ws.ensure(per_img * (size_t)B + 4096));
  char* p = ws.as<char>();
  uint8_t* resized = reinterpret_cast<uint8_t*>(p);
  p += ((size_t)B * 224 * 224 + 255) / 256 * 256;
  f16* X = reinterpret_cast<f16*>(p); p += (size_t)B * per_big * sizeof(f16);
  f16* Y = reinterpret_cast<f16*>(p); p += (size_t)B * per_big * sizeof(f16);
  f16* L = reinterpret_cast<f16*>(p); p += (size_t)B * per_last * sizeof(f16);
  float* pooled = reinterpret_cast<float*>(p); p += ((size_t)B * 1280 * sizeof(float) + 255) / 256 * 256;
  f16* Eb = reinterpret_cast<f16*>(p); p += (size_t)B * pe * sizeof(f16);
  f16* Db = reinterpret_cast<f16*>(p); p += (size_t)B * pd * sizeof(f16);
  f16* P0 = reinterpret_cast<f16*>(p); p += (size_t)B * pp * sizeof(f16);
  f16* P1 = reinterpret_cast<f16*>(p);

  const f16* Wt = wts.as<f16>();
  const float* P = prm.as<float>();
  const uint8_t* stem_in = img;
  if (fer) {
    MEC_TRY(resize_u8(img, B, 48, 48, resized, 224, 224, s));
    stem_in = resized;
  }
  MEC_TRY(prof.begin(TAG_MBV2_BLOCK, s));
  const f16* cur = reinterpret_cast<const f16*>(stem_in);
  f16* out = X;
  int h = 112;
  for (size_t i = 0; i < blocks.size(); ++i) {
    const MbBlock& b = blocks[i];
    if (i >= l0) {
      const int oh = b.stride == 2 ? h / 2 : h;
      const f16* in = cur;
      f16* pout = (cur == P0) ? P1 : P0;
      if (i == l0 && b.cin != b.lcinp) {  // the fused blocks' rows -> the layered row stride
        const size_t rows = (size_t)B * h * h, items = rows * (b.lcinp / 8);
        hipLaunchKernelGGL(mbv2_pad_f16_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, cur, rows,
                           b.cin, b.lcinp, P1);
        MEC_LAUNCH_CHECK();
        in = P1;
        pout = P0;
      }
      GemmParams g;  // expand + BN + ReLU6 -> E f16
      g.A = in; g.B = Wt + b.lwe_off; g.bias = P + b.be_off; g.act = ACT_RELU6; g.C16 = Eb;
      g.M = B * h * h; g.N = b.hidp; g.K = b.lcinp;
      MEC_TRY(launch_gemm(g, s, nullptr, 0));  // inside the TAG_MBV2_BLOCK window
      const size_t items = (size_t)B * oh * (b.hidp / 8);  // one output row of one 8-channel group each
      if (b.stride == 2)
        hipLaunchKernelGGL(mbv2_dw_f16_kernel<2>, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, Eb, h, oh,
                           b.hidp, P + b.wd_off, P + b.bd_off, Db, items);
      else
        hipLaunchKernelGGL(mbv2_dw_f16_kernel<1>, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, Eb, h, oh,
                           b.hidp, P + b.wd_off, P + b.bd_off, Db, items);
      MEC_LAUNCH_CHECK();
      g = GemmParams();  // project + BN (+ the block input) -> f16 rows of lcoutp channels
      g.A = Db; g.B = Wt + b.lwp_off; g.bias = P + b.lbp_off; g.act = ACT_NONE; g.C16 = pout;
      if (b.stride == 1 && b.cin == b.cout) g.R = in;
      g.M = B * oh * oh; g.N = b.lcoutp; g.K = b.hidp;
      MEC_TRY(launch_gemm(g, s, nullptr, 0));
      cur = pout;
      h = oh;
      continue;
    }
    MbArgs a;
    a.x = cur; a.y = out; a.H = h; a.OH = b.stride == 2 ? h / 2 : h;
    a.cin = b.cin; a.cout = b.cout; a.hidp = b.hidp;
    a.We = Wt + b.we_off; a.be = P + b.be_off; a.Wd = P + b.wd_off; a.bd = P + b.bd_off;
    a.Wp = Wt + b.wp_off; a.bp = P + b.bp_off;
    a.stem_w = P + (C == 3 ? stem_rgb_off : stem_w_off);
    a.stem_corr = P + stem_corr_off;
    MEC_TRY(dispatch_block(b, a, B, i == 0 ? (C == 3 ? 3 : 1) : 0, s));
    cur = out;
    out = (out == X) ? Y : X;
    h = a.OH;
  }
  MEC_TRY(prof.end(TAG_MBV2_BLOCK, s));
  {  // features[18] 1x1 320 -> 1280 + BN + ReLU6
    GemmParams g;
    g.A = cur; g.B = Wt + last_w_off; g.bias = P + last_b_off; g.act = ACT_RELU6; g.C16 = L;
    g.M = B * h * h; g.N = 1280; g.K = 320;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_MBV2_LAST));
  }
  hipLaunchKernelGGL(avgpool8_kernel, dim3(B), dim3(1280 / 8 * 4), 0, s, L, h * h, 1280, pooled);
  MEC_LAUNCH_CHECK();
  // classifier[1] Linear(1280,512) + classifier[2] ReLU -> the 512-d feature, then classifier[4] + softmax
  MEC_TRY(launch_linear_mfma<BACT_RELU>(pooled, 1280, B, 1280, P + fc1_off, P + fc1b_off, 512, feat, 512, nullptr, 0, s));
  MEC_TRY(launch_head7(feat, B, 512, P + fc2_off, P + fc2b_off, logits, probs, s));
  return 0;
}

}  // namespace mec
